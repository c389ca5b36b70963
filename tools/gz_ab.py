#!/usr/bin/env python3
"""A/B of inflater builds on the GPU box: one synthetic FASTQ (the bench's
reads, pigz-style gzip -1), then each libvafc.so given on the command line
timed in its own process on vc_gz_inflate_parallel at the given thread counts
(best of --reps), in rounds that alternate the libraries.

    python tools/gz_ab.py [--reads 8000000] [--threads 1,16] LIB[:KEY=VAL,...] [...]

(an optional `:KEY=VAL,...` suffix sets environment knobs for that variant)

The first call in a fresh process runs 3-4x slower on the box than later
ones (profiles/r02_gz_first.log; not seen on the build host), so use
--reps >= 2 (best of) or compare like with like.
"""
import argparse
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, time
sys.path.insert(0, os.path.join(%(root)r, "kmer-cnt_amd"))
import vafc
gz = %(gz)r
for th in %(threads)r:
    best = 1e9
    for _ in range(%(reps)d):
        t0 = time.time()
        n = vafc.lib().vc_gz_inflate_parallel(gz.encode(), th, 0, None, 0, None)
        best = min(best, time.time() - t0)
    print("%%s threads %%2d: %%.0f MB/s of text" %% (os.environ["GZAB_NAME"], th, n / best / 1e6), flush=True)
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=8_000_000)
    ap.add_argument("--threads", default="1,16")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("libs", nargs="+")
    a = ap.parse_args()
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))
    import numpy as np
    import torch
    import bench
    import vafc
    import vafc_synth as S
    dev = torch.device("cuda", 0)
    panel = S.grch38_panel()
    tmp = tempfile.mkdtemp(prefix="gzab_")
    R, L = a.reads, 150
    d_seq = torch.empty(R * L, dtype=torch.uint8, device=dev)
    d_offs = torch.empty(R, dtype=torch.int64, device=dev)
    d_lens = torch.empty(R, dtype=torch.int32, device=dev)
    win = torch.from_numpy(panel.windows().reshape(-1)).to(dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(dev)
    vafc.synth_reads(d_seq.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), 0, R, L, S.READ_SEED_R1, 0.01,
                     win.data_ptr(), dos.data_ptr(), panel.n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    fq = os.path.join(tmp, "r.fq")
    gz = fq + ".gz"
    bench.write_fastq_from_device(d_seq, R, L, fq)
    bench.gzip_level1(fq, gz, 16)
    os.unlink(fq)
    print("file: %d reads, %.2f GB gzip" % (R, os.path.getsize(gz) / 1e9), flush=True)
    threads = [int(x) for x in a.threads.split(",")]
    for _ in range(a.rounds):
        for spec in a.libs:
            lib, _, knobs = spec.partition(":")
            env = dict(os.environ, VAFC_LIB=os.path.abspath(lib), GZAB_NAME=spec)
            env.update(kv.split("=", 1) for kv in knobs.split(",") if kv)
            code = CHILD % {"root": ROOT, "gz": gz, "threads": threads, "reps": a.reps}
            subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=600)
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
