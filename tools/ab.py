#!/usr/bin/env python3
"""Interleaved A/B timing of counter variants in ONE process (same device, same
HBM-resident reads): variants differ by environment knobs read at vc_create
time (e.g. VAFC_ABLATE=0|4 with the ablation build).  Also checks that every variant produces the
same counts.  Usage (GPU box):
    VAFC_LIB=kmer-cnt_amd/lib/libvafc_abl.so python tools/ab.py --rounds 10 VAFC_ABLATE=0 VAFC_ABLATE=4
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=100_000_000)
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--f-snp", type=float, default=0.01)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--panel", default="grch38", choices=["grch38", "syn200k"])
    ap.add_argument("variants", nargs="+", help="KEY=VAL[,KEY=VAL] env settings per variant")
    a = ap.parse_args()
    import torch
    import vafc
    import vafc_synth as S
    import tempfile
    dev = torch.device("cuda", 0)
    rows = S.read_bed(S.default_bed_path()) if a.panel == "grch38" else S.synthetic_bed(200_000)
    panel = S.make_panel(rows)
    tmp = tempfile.mkdtemp()
    pat = os.path.join(tmp, "p.txt")
    panel.write_patterns(pat, a.k)
    db = vafc.load_patterns(pat)
    keys, vals, _ = db.keys(a.k)
    R, L = a.reads, a.read_len
    d_seq = torch.empty(R * L, dtype=torch.uint8, device=dev)
    d_offs = torch.empty(R, dtype=torch.int64, device=dev)
    d_lens = torch.empty(R, dtype=torch.int32, device=dev)
    win = torch.from_numpy(panel.windows().reshape(-1)).to(dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(dev)
    torch.cuda.synchronize()
    vafc.synth_reads(d_seq.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), 0, R, L, S.READ_SEED_R1,
                     a.f_snp, win.data_ptr(), dos.data_ptr(), panel.n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    maps = []
    for v in a.variants:
        saved = {}
        for kv in v.split(","):
            k_, val = kv.split("=", 1)
            saved[k_] = os.environ.get(k_)
            os.environ[k_] = val
        m = vafc.KmerMap(a.k, keys, vals, db.n, 0)
        m.set_timing(True)
        maps.append(m)
        for k_, old in saved.items():
            if old is None:
                os.environ.pop(k_, None)
            else:
                os.environ[k_] = old
    times = [[] for _ in maps]
    results = []
    for r in range(a.rounds + 1):
        for i, m in enumerate(maps):
            m.reset()
            m.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr(), d_lens.data_ptr(), R)
            ms = m.kernel_ms()
            if r > 0:
                times[i].append(ms)
            if r == a.rounds:
                results.append(m.finish())
    same = all(np.array_equal(results[0][0], c) and results[0][1] == km for c, km in results)
    for v, t in zip(a.variants, times):
        print("%-40s median %.3f ms  min %.3f ms  (%.0f Mbases/s)" % (
            v, float(np.median(t)), float(np.min(t)), R * L / (np.median(t) * 1e-3) / 1e6))
    print("counts identical across variants:", same, " kmers:", results[0][1], " hits:",
          int(results[0][0].astype(np.uint64).sum()))


if __name__ == "__main__":
    main()
