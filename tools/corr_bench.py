#!/usr/bin/env python3
"""correlation-matrix on the GPU vs the reference.

Workload: N synthetic samples over the GRCh38 panel's row count (20,849 SNPs
by default): genotypes of N/4 individuals, each sampled 4 times at depths
5..40 with 5 % depth-0 rows, VAF rounded to 4 decimals as vaf-counter writes
it.  One step = the full N x N depth-aware Pearson matrix
(correlation-matrix.c:146-162) on the device (kernel time from HIP events; the
host-side staging and the D2H copy are reported separately by wall clock).

CPU baseline: the REAL reference binary (oracle/_ref/correlation-matrix) on
the first --cpu-samples samples written as .vaf files, wall clock of the whole
program (its pair loop dominates), scaled per pair-row; parity: the GPU CLI's
.corr/.tree on that subset are byte-identical to the reference's.

    python tools/corr_bench.py [--samples 1000] [--rows 20849] [--cpu-samples 160]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))


def synth(n, rows, seed=11):
    rng = np.random.default_rng(seed)
    n_ind = max(1, n // 4)
    geno = rng.integers(0, 3, (n_ind, rows))
    vaf = np.zeros((n, rows))
    dep = np.zeros((n, rows), np.int32)
    for s in range(n):
        d = rng.poisson(5 + (s * 7) % 36, rows)
        d[rng.random(rows) < 0.05] = 0
        alt = rng.binomial(d, np.clip(geno[s % n_ind] / 2.0, 0.01, 0.99))
        vaf[s] = np.where(d > 0, np.round(alt / np.maximum(d, 1), 4), 0.0)
        dep[s] = d
    return vaf, dep


def write_vafs(d, vaf, dep):
    paths = []
    for s in range(vaf.shape[0]):
        p = os.path.join(d, "s%04d.vaf" % s)
        with open(p, "w") as f:
            f.write("# Average depth: %.2f\nCHR\tPOS\tRSID\tREF\tALT\tREF_COUNT\tALT_COUNT\tTOTAL_COUNT\tVAF\n"
                    % dep[s].mean())
            f.write("".join("chr1\t%d\trs%d\tA\tC\t0\t0\t%d\t%.4f\n" % (i, i, dep[s, i], vaf[s, i])
                            for i in range(vaf.shape[1])))
        paths.append(p)
    return paths


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=1000)
    ap.add_argument("--rows", type=int, default=20849)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cpu-samples", type=int, default=160)
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first)
    import vafc
    t0 = time.time()
    vaf, dep = synth(a.samples, a.rows)
    sys.stderr.write("synthesized %d x %d in %.1fs\n" % (a.samples, a.rows, time.time() - t0))
    ms, walls = [], []
    corr = None
    for _ in range(a.steps + 1):
        t0 = time.perf_counter()
        corr, k = vafc.correlation_matrix_raw(vaf, dep)
        walls.append(time.perf_counter() - t0)
        ms.append(k)
    ms, walls = ms[1:], walls[1:]
    pairs = a.samples * (a.samples - 1) // 2
    kms = float(np.median(ms))
    gpu_rate = pairs * a.rows / (kms * 1e-3)
    # CPU reference on a bounded subset + parity of the CLI on it
    cpu = None
    ref = os.path.join(ROOT, "oracle", "_ref", "correlation-matrix")
    cli = os.path.join(ROOT, "kmer-cnt_amd", "lib", "correlation-matrix")
    with tempfile.TemporaryDirectory() as d:
        m = min(a.cpu_samples, a.samples)
        paths = write_vafs(d, vaf[:m], dep[:m])
        res = {}
        for tag, b in (("ref", ref), ("gpu", cli)):
            if not os.path.exists(b):
                continue
            t0 = time.perf_counter()
            p = subprocess.run([b, "-t", "-o", os.path.join(d, tag + ".corr")] + paths, capture_output=True,
                               timeout=900)
            w = time.perf_counter() - t0
            assert p.returncode == 0, p.stderr[-500:]
            with open(os.path.join(d, tag + ".corr")) as f, open(os.path.join(d, tag + ".tree")) as g:
                res[tag] = (w, f.read(), g.read())
        if "ref" in res:
            mp = m * (m - 1) // 2
            cpu = {"value": mp * a.rows / res["ref"][0], "unit": "pair-rows/s", "cores": 1, "kind": "reference",
                   "sample": "first %d samples (%d pairs x %d rows), whole program wall %.2f s" % (
                       m, mp, a.rows, res["ref"][0])}
        parity = ("ref" in res and "gpu" in res and res["ref"][1:] == res["gpu"][1:])
        cli_wall = res["gpu"][0] if "gpu" in res else None
    line = {
        "tool": "correlation-matrix", "samples": a.samples, "rows": a.rows, "pairs": pairs,
        "kernel_ms": round(kms, 3), "call_wall_ms": round(float(np.median(walls)) * 1e3, 1),
        "value": round(gpu_rate, 1), "unit": "pair-rows/s (kernel)",
        "fp64_ops_per_valid_pair_row": 10,
        "cpu_baseline": cpu,
        "speedup_kernel_vs_cpu": round(gpu_rate / cpu["value"], 1) if cpu else None,
        "cli_wall_s_on_cpu_sample": round(cli_wall, 3) if cli_wall else None,
        "parity_cli_vs_reference_on_sample": parity,
        "matrix_checksum": float(np.nansum(corr)),
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
