#!/usr/bin/env python3
"""Calibrate the HBM read counters on the counting kernel's own buffer (GPU box).

The MI355X guide's rule (FETCH_SIZE x 2 = bytes) is calibrated on wide
coalesced streaming reads; our kernel reads one read per lane.  This script
puts both on the same 15 GB read buffer: the C2 counting kernel, then a
streaming pass over exactly the same bytes (a torch sum of the buffer as
int32: every byte read once, coalesced).  Run it under
    rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum -d DIR -- python3 tools/traffic_calib.py
and read DIR with --report DIR: bytes per EA request from the streaming pass
(known bytes / its requests), then the counting kernel's traffic = its
requests x that.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))
R, L = 100_000_000, 150


def run():
    import numpy as np
    import torch
    import tempfile
    import vafc
    import vafc_synth as S
    dev = torch.device("cuda", 0)
    panel = S.grch38_panel()
    d = tempfile.mkdtemp()
    pat = os.path.join(d, "p.txt")
    panel.write_patterns(pat, 21)
    db = vafc.load_patterns(pat)
    keys, vals, _ = db.keys(21)
    d_seq = torch.empty(R * L, dtype=torch.uint8, device=dev)
    d_offs = torch.empty(R, dtype=torch.int64, device=dev)
    d_lens = torch.empty(R, dtype=torch.int32, device=dev)
    win = torch.from_numpy(panel.windows().reshape(-1)).to(dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(dev)
    torch.cuda.synchronize()
    vafc.synth_reads(d_seq.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), 0, R, L, S.READ_SEED_R1, 0.01,
                     win.data_ptr(), dos.data_ptr(), panel.n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    m = vafc.KmerMap(21, keys, vals, db.n, 0)
    for _ in range(2):
        m.reset()
        m.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr(), d_lens.data_ptr(), R)
        m.finish()
        s = d_seq.view(torch.int32).sum(dtype=torch.int64)      # streaming read of the same 15 GB
        o = d_offs.sum()                                          # and of the offsets (0.8 GB)
        torch.cuda.synchronize()
    print(json.dumps({"seq_bytes": R * L, "offs_bytes": R * 8, "lens_bytes": R * 4, "sum": int(s), "o": int(o)}))


def report(path):
    rows = {}
    for fn in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            k = (r["Dispatch_Id"], r["Kernel_Name"])
            rows.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
            rows[k][r["Counter_Name"]] += float(r["Counter_Value"])
    out = []
    for (disp, name), c in sorted(rows.items(), key=lambda x: int(x[0][0])):
        out.append({"dispatch": int(disp), "kernel": name[:80], **c})
    stream = [o for o in out if "reduce" in o["kernel"].lower() or "sum" in o["kernel"].lower()]
    count = [o for o in out if "vc_count_reads_kernel" in o["kernel"]]
    res = {"dispatches": out}
    if stream and count:
        big = max(stream, key=lambda o: o.get("TCC_EA0_RDREQ_sum", 0))   # the 15 GB sum
        bpr = R * L / big["TCC_EA0_RDREQ_sum"]
        cnt = count[-1]
        res.update({"stream_kernel": big["kernel"], "stream_bytes_known": R * L,
                    "stream_rdreq": big["TCC_EA0_RDREQ_sum"], "bytes_per_rdreq_streaming": bpr,
                    "count_rdreq": cnt["TCC_EA0_RDREQ_sum"], "count_bubble": cnt.get("TCC_BUBBLE_sum"),
                    "count_rdreq_32b": cnt.get("TCC_EA0_RDREQ_32B_sum"),
                    "count_traffic_bytes_calibrated": cnt["TCC_EA0_RDREQ_sum"] * bpr,
                    "count_alg_bytes": R * L + R * 12,
                    "count_traffic_over_alg": cnt["TCC_EA0_RDREQ_sum"] * bpr / (R * L + R * 12)})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        run()
