#!/usr/bin/env python3
"""snp-pattern-gen candidate counting on MI355X.

Workload: a synthetic genome with the GRCh38 primary-assembly chromosome
lengths (3.09 Gbases, uniform ACGT, the first 10 kb of every chromosome and a
few 50 kb blocks set to N) generated in HBM; candidates = the ref and alt
k-mers of the 20,920 SNP rows of data/SNP_GRCh38_hg38_wChr.bed (k = 21) cut
from that genome, as snp-pattern-gen's first pass does.

Timed (inputs resident in HBM): one step = the counting kernels in seq_nt4
mode (vc_set_nt4_decode + vc_count_device; chromosomes take the segmented
long-read kernel).

CPU beside it: the REAL reference snp-pattern-gen (oracle/_ref, compiled from
its sources) on a sample -- chr1 of the same genome written as FASTA plus the
chr1 BED rows -- timed as a whole program, and the drop-in GPU CLI on the
same files (end to end, FASTA load included), whose pattern file must be
byte-identical.  Prints one JSON line.
    python tools/spg_bench.py [--steps N] [--warmup W] [--no-cpu]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))

GRCH38 = [("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555),
          ("chr5", 181538259), ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636),
          ("chr9", 138394717), ("chr10", 133797422), ("chr11", 135086622), ("chr12", 133275309),
          ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189), ("chr16", 90338345),
          ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr20", 64444167),
          ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415),
          ("chrM", 16569)]
NT4 = np.full(256, 4, np.uint8)
for _i, _c in enumerate(b"ACGT"):
    NT4[_c] = NT4[_c + 32] = _i


def canonical(codes: np.ndarray, k: int) -> np.ndarray:
    """canonical 2-bit keys of rows of k codes (0..3)"""
    w = (np.uint64(1) << (2 * np.arange(k - 1, -1, -1, dtype=np.uint64)))
    f = (codes.astype(np.uint64) * w).sum(axis=1, dtype=np.uint64)
    r = ((3 - codes[:, ::-1]).astype(np.uint64) * w).sum(axis=1, dtype=np.uint64)
    return np.minimum(f, r)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    import torch
    import vafc
    import vafc_synth as S
    dev = torch.device("cuda", 0)
    k = a.k
    # genome in HBM
    lens = np.array([L for _, L in GRCH38], np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    total = int(lens.sum())
    padded = (total + 15) // 16 * 16 + 16
    g = torch.empty(padded, dtype=torch.uint8, device=dev)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(12345)
    step = 1 << 28
    for s in range(0, padded, step):
        e = min(padded, s + step)
        g[s:e] = lut[torch.randint(0, 4, (e - s,), device=dev, generator=gen, dtype=torch.int64)]
    for o in offs:
        g[int(o):int(o) + 10000] = ord("N")
    for o, L in zip(offs[:5], lens[:5]):
        g[int(o) + int(L) // 2:int(o) + int(L) // 2 + 50000] = ord("N")
    g[total:] = ord("N")
    # candidates: BED pass 1 on this genome
    name_idx = {n: i for i, (n, _) in enumerate(GRCH38)}
    rows = [r for r in S.read_bed(S.default_bed_path()) if r[0] in name_idx]
    f = k // 2
    ok = [r for r in rows if r[1] - f >= 0 and r[1] - f + k <= int(lens[name_idx[r[0]]])]
    starts = torch.tensor([int(offs[name_idx[r[0]]]) + r[1] - f for r in ok], dtype=torch.int64, device=dev)
    win = g[(starts[:, None] + torch.arange(k, device=dev)[None, :])].cpu().numpy()
    codes = NT4[win]
    alt = NT4[np.frombuffer("".join(r[5][0] for r in ok).encode(), np.uint8)]
    good = (codes < 4).all(axis=1) & (alt < 4)
    codes, alt = codes[good], alt[good]
    alt_codes = codes.copy()
    alt_codes[:, f] = alt
    keys = np.unique(np.concatenate([canonical(codes, k), canonical(alt_codes, k)]))
    vals = np.arange(keys.size, dtype=np.uint32)
    n_pat = (keys.size + 1) // 2
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.astype(np.int32)).to(dev)
    m = vafc.KmerMap(k, keys, vals, n_pat, 0)
    m.set_timing(True)
    vafc.lib().vc_set_nt4_decode(m._h, 1)

    def one_step():
        m.reset()
        m.count_device(g.data_ptr(), total, d_offs.data_ptr(), d_lens.data_ptr(), len(GRCH38))

    for _ in range(a.warmup):
        one_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kms = []
    for _ in range(a.steps):
        one_step()
        kms.append(m.kernel_ms())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    counts, km = m.finish()
    cnt = counts[:keys.size]
    res = {
        "metric": "candidate k-mer counting over a GRCh38-sized genome (snp-pattern-gen pass 2), k=%d" % k,
        "value": round(total / dt / 1e6, 1), "unit": "Mbases/sec", "n_gpus": 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "u8",
        "data": "synthetic genome with GRCh38 chromosome lengths (seed 12345) in HBM; candidates from "
                "SNP_GRCh38_hg38_wChr.bed",
        "config": {"workload": "spg: 25 chromosomes, %d bases, %d BED rows, %d candidate keys" % (
            total, len(rows), keys.size), "k": k},
        "count_kernels_ms": round(float(np.median(kms)), 3),
        "kmers_counted": int(km), "candidates_seen": int((cnt > 0).sum()), "unique_ref_candidates": int((cnt == 1).sum()),
        "roofline": {"bound": "hbm", "achieved": round(total / dt / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(total / dt / 8e12, 4), "traffic": None,
                     "note": "algorithmic bytes 1 B/base (the genome read once)"},
    }
    if not a.no_cpu:
        ref = os.path.join(ROOT, "oracle", "_ref", "snp-pattern-gen")
        cli = os.path.join(ROOT, "kmer-cnt_amd", "lib", "snp-pattern-gen")
        with tempfile.TemporaryDirectory() as d:
            i21 = name_idx["chr1"]
            seq = g[int(offs[i21]):int(offs[i21] + lens[i21])].cpu().numpy().tobytes()
            with open(os.path.join(d, "g.fa"), "wb") as fp:
                fp.write(b">chr1\n")
                for s in range(0, len(seq), 60):
                    fp.write(seq[s:s + 60] + b"\n")
            with open(os.path.join(d, "s.bed"), "w") as fp:
                for r in rows:
                    if r[0] == "chr1":
                        fp.write("%s\t%d\t%d\t%s\t%s\t%s\n" % r)
            out = {}
            for tag, binary in (("reference", ref), ("gpu_cli", cli)):
                t = time.perf_counter()
                p = subprocess.run([binary, "-k", str(k), "-b", "s.bed", "-f", "g.fa", "-o", tag + ".txt"], cwd=d,
                                   capture_output=True, text=True, timeout=900)
                wall = time.perf_counter() - t
                assert p.returncode == 0, p.stderr
                out[tag] = (wall, hashlib.md5(open(os.path.join(d, tag + ".txt"), "rb").read()).hexdigest())
            res["cpu_baseline"] = {"value": round(len(seq) / out["reference"][0] / 1e6, 2), "unit": "Mbases/sec",
                                   "cores": 1, "kind": "reference",
                                   "sample": "chr1 of this genome (%d bases) + its BED rows, whole program "
                                             "(FASTA load included), wall %.2f s" % (len(seq), out["reference"][0])}
            res["gpu_cli_same_sample"] = {"value": round(len(seq) / out["gpu_cli"][0] / 1e6, 2),
                                          "unit": "Mbases/sec", "wall_s": round(out["gpu_cli"][0], 3),
                                          "note": "drop-in CLI end to end incl. process start, FASTA load, "
                                                  "device init"}
            res["parity_vs_reference_on_sample"] = out["reference"][1] == out["gpu_cli"][1]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
