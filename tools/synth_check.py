import os, sys, tempfile
import numpy as np, torch
sys.path.insert(0, "kmer-cnt_amd")
import vafc, vafc_synth as S
dev = torch.device("cuda", 0)
panel = S.grch38_panel()
win = torch.from_numpy(panel.windows().reshape(-1)).to(dev)
dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(dev)
L = 150
def gen(first, n):
    s = torch.empty(n * L, dtype=torch.uint8, device=dev); o = torch.empty(n, dtype=torch.int64, device=dev); l = torch.empty(n, dtype=torch.int32, device=dev)
    vafc.synth_reads(s.data_ptr(), o.data_ptr(), l.data_ptr(), first, n, L, S.READ_SEED_R1, 0.01, win.data_ptr(), dos.data_ptr(), panel.n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize(); return s, o, l
a = gen(0, 2_000_000); b = gen(0, 3_000_000)
print("bytes equal", torch.equal(a[0], b[0][: 2_000_000 * L]), "offs equal", torch.equal(a[1], b[1][:2_000_000]))
d = tempfile.mkdtemp(); pat = os.path.join(d, "p.txt"); panel.write_patterns(pat, 21)
db = vafc.load_patterns(pat); keys, vals, _ = db.keys(21)
m = vafc.KmerMap(21, keys, vals, db.n, 0)
n = 2_000_000
for s, o, l in (a, b):
    m.reset(); m.count_device(s.data_ptr(), n * L, o.data_ptr(), l.data_ptr(), n); c, k = m.finish()
    print("sum", int(c.astype(np.uint64).sum()), "kmers", k)
# python generator for a slice
r = S.gen_reads(panel, 1000, 0, S.READ_SEED_R1, 0.01, L)
print("python == device (first 1000 reads):", bytes(r.reshape(-1)) == a[0][:1000 * L].cpu().numpy().tobytes())
