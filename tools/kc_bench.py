#!/usr/bin/env python3
"""kc-c4 k-mer histogram on MI355X.

Workload: N synthetic 150 bp reads (default 10M = 1.5 Gbases) sampled from a
synthetic 50 Mb genome (uniform ACGT, seed 12345) with 50 % reverse
complements, 0.5 % substitutions and 0.1 % N, generated in HBM with torch;
k = 31 (kc-c4's default).  About 30x coverage, so the histogram has kc-c4's
usual shape: an error peak at 1 and a coverage peak near 24.

Timed (inputs resident in HBM): one step = vc_reset (table clear) + the
counting kernels over all reads (vc_count_device) + the histogram kernel
(vc_kc_histogram).  `kernel_ms` is the counting kernels alone (HIP events on
the library's stream).

Roofline: random-access bound.  Algorithmic bytes per k-mer = one 16-byte
table slot read and written (32 B; the probe load, the key CAS when the k-mer
is new and the count's atomic add all hit the same slot) + 1 B per base of
input; `achieved` = those bytes / counting-kernel time vs 8 TB/s.

CPU beside it: the REAL reference kc-c4 (oracle/_ref, compiled from its
sources) on a sample (the first `--cpu-reads` reads written as FASTQ), whole
program, at -t 1/4/16, and the drop-in GPU CLI on the same file, whose
stdout must be byte-identical.  Prints one JSON line.
    python tools/kc_bench.py [--reads N] [--steps N] [--warmup W] [--no-cpu]
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


def make_reads(torch, dev, n, L=150, genome_len=50_000_000, seed=12345):
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    comp = torch.zeros(256, dtype=torch.uint8, device=dev)
    for a, b in zip(b"ACGTN", b"TGCAN"):
        comp[a] = b
    g = lut[torch.randint(0, 4, (genome_len,), device=dev, generator=gen)]
    seq = torch.empty(n * L, dtype=torch.uint8, device=dev)
    ar = torch.arange(L, device=dev)
    step = 1 << 22
    for s in range(0, n, step):
        m = min(step, n - s)
        st = torch.randint(0, genome_len - L + 1, (m,), device=dev, generator=gen)
        r = g[st[:, None] + ar[None, :]]
        rev = torch.rand(m, device=dev, generator=gen) < 0.5
        r[rev] = comp[r[rev].flip(1).long()]
        u = torch.rand(m, L, device=dev, generator=gen)
        sub = u < 0.005
        r[sub] = lut[torch.randint(0, 4, (int(sub.sum()),), device=dev, generator=gen)]
        r[(u >= 0.005) & (u < 0.006)] = ord("N")
        seq[s * L:(s + m) * L] = r.reshape(-1)
    offs = torch.arange(n, dtype=torch.int64, device=dev) * L
    lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    return seq, offs, lens


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=31)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--slots", type=int, default=1 << 29)
    ap.add_argument("--cpu-reads", type=int, default=2_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    import torch
    import vafc
    dev = torch.device("cuda", 0)
    L = 150
    seq, offs, lens = make_reads(torch, dev, a.reads, L)
    torch.cuda.synchronize()
    h = vafc.KmerHistogram(a.k, a.slots, 0)
    h.set_timing(True)

    def one_step():
        h.reset()
        h.count_device(seq.data_ptr(), seq.numel(), offs.data_ptr(), lens.data_ptr(), a.reads)
        return h.histogram()

    for _ in range(a.warmup):
        one_step()
    torch.cuda.synchronize()
    kms = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        hist, distinct, kmers = one_step()
        kms.append(h.kernel_ms())
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    h.close()
    bases = a.reads * L
    kern = float(np.median(kms)) * 1e-3
    alg = bases + 32 * kmers
    peak_i = int(np.argmax(hist[2:])) + 2
    res = {
        "metric": "kc-c4 k-mer histogram, Mbases/sec on 150 bp reads, k=%d" % a.k,
        "value": round(bases / dt / 1e6, 1), "unit": "Mbases/sec", "n_gpus": 1, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "u64",
        "data": "synthetic: %d x %d bp reads from a 50 Mb random genome (0.5%% subst, 0.1%% N, 50%% revcomp), "
                "generated in HBM" % (a.reads, L),
        "config": {"workload": "kc-c4: %d reads x %d bp, k=%d, table %d slots" % (a.reads, L, a.k, a.slots),
                   "k": a.k},
        "count_kernels_ms": round(kern * 1e3, 3),
        "kmers_per_sec": round(kmers / kern, 1),
        "kmers": int(kmers), "distinct": int(distinct), "hist_1": int(hist[1]), "coverage_peak": peak_i,
        "roofline": {"bound": "hbm", "achieved": round(alg / kern / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(alg / kern / 8e12, 4), "traffic": None,
                     "note": "algorithmic bytes = 1 B/base + 32 B/k-mer (one 16 B slot read + written)"},
    }
    if not a.no_cpu:
        ref = os.path.join(ROOT, "oracle", "_ref", "kc-c4")
        cli = os.path.join(ROOT, "kmer-cnt_amd", "lib", "kc-c4")
        n = min(a.cpu_reads, a.reads)
        sample = seq[:n * L].cpu().numpy().reshape(n, L)
        with tempfile.TemporaryDirectory() as d:
            fq = os.path.join(d, "s.fq")
            qual = b"I" * L
            with open(fq, "wb") as fp:
                fp.write(b"".join(b"@r%d\n%s\n+\n%s\n" % (i, sample[i].tobytes(), qual) for i in range(n)))
            runs = {}
            for tag, binary, t in (("ref_t1", ref, 1), ("ref_t4", ref, 4), ("ref_t16", ref, 16),
                                   ("gpu_cli", cli, 4)):
                t0 = time.perf_counter()
                p = subprocess.run([binary, "-k", str(a.k), "-t", str(t), fq], capture_output=True, timeout=900)
                wall = time.perf_counter() - t0
                assert p.returncode == 0, p.stderr
                runs[tag] = (wall, hashlib.md5(p.stdout).hexdigest())
        best = min(("ref_t1", "ref_t4", "ref_t16"), key=lambda x: runs[x][0])
        res["cpu_baseline"] = {"value": round(n * L / runs[best][0] / 1e6, 2), "unit": "Mbases/sec",
                               "cores": int(best.split("_t")[1]), "kind": "reference",
                               "sample": "first %d reads as FASTQ, whole program; wall -t1/-t4/-t16 = "
                                         "%.2f/%.2f/%.2f s" % (n, runs["ref_t1"][0], runs["ref_t4"][0],
                                                                runs["ref_t16"][0])}
        res["gpu_cli_same_sample"] = {"value": round(n * L / runs["gpu_cli"][0] / 1e6, 2), "unit": "Mbases/sec",
                                      "wall_s": round(runs["gpu_cli"][0], 3),
                                      "note": "drop-in CLI end to end incl. process start, FASTQ parse, device init"}
        res["parity_vs_reference_on_sample"] = len({v[1] for v in runs.values()}) == 1
    print(json.dumps(res))


if __name__ == "__main__":
    main()
