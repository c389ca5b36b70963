#!/usr/bin/env python3
"""gzip ingest sweep on the GPU box: the bench's e2e FASTQ (synthetic reads
generated in HBM, written as FASTQ, compressed pigz-style at level 1), then
the drop-in CLI's counting-phase rate at several parse-worker counts
($VAFC_GZ_PARSERS) and the host-only reader (no device) for the same split.

    python tools/gz_sweep.py [--reads 16000000] [--threads 16] [--parsers 1,2,3,4,6]
"""
import argparse
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=16_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--parsers", default="1,2,3,4,6")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--scaling", default="", help="also time the inflater alone at these thread counts")
    ap.add_argument("--variants", default="", help="';'-separated groups of space-separated KEY=VAL env "
                                                   "settings, each timed with the CLI (instead of --parsers); "
                                                   "CLI=path runs another vaf-counter build")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import vafc
    import vafc_synth as S
    dev = torch.device("cuda", 0)
    panel = S.grch38_panel()
    tmp = bench.scratch_dir(args.reads * 330 * 1.3, tempfile.mkdtemp(prefix="gzsweep_"))   # /dev/shm when it fits
    pat = os.path.join(tmp, "p.txt")
    panel.write_patterns(pat, 21)
    R, L = args.reads, 150
    d_seq = torch.empty(R * L, dtype=torch.uint8, device=dev)
    d_offs = torch.empty(R, dtype=torch.int64, device=dev)
    d_lens = torch.empty(R, dtype=torch.int32, device=dev)
    win = torch.from_numpy(panel.windows().reshape(-1)).to(dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(dev)
    torch.cuda.synchronize()
    vafc.synth_reads(d_seq.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), 0, R, L, S.READ_SEED_R1, 0.01,
                     win.data_ptr(), dos.data_ptr(), panel.n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    fq = os.path.join(tmp, "r.fq")
    gz = fq + ".gz"
    bench.write_fastq_from_device(d_seq, R, L, fq)
    bench.gzip_level1(fq, gz, args.threads)
    del d_seq, d_offs, d_lens
    print("file: %d reads, %.2f GB text, %.2f GB gzip" % (R, os.path.getsize(fq) / 1e9, os.path.getsize(gz) / 1e9),
          flush=True)
    os.unlink(fq)
    for v in [x.strip() for x in args.variants.split(";") if x.strip()]:
        env = dict(os.environ, **dict(kv.split("=", 1) for kv in v.split()))
        cli = os.path.abspath(env.pop("CLI", bench.PRODUCT_CLI))   # CLI=path: another build (A/B)
        rs = [bench.cli_run(cli, pat, gz, args.threads, os.path.join(tmp, "o.vaf"), 21, env=env)
              for _ in range(args.reps)]
        print("%-60s CLI %s Mbases/s (process %s s)" % (v, [round(r["mbases"]) for r in rs],
                                                        [round(r["wall"], 2) for r in rs]), flush=True)
    for parsers in ([int(x) for x in args.parsers.split(",")] if not args.variants else []):
        env = dict(os.environ, VAFC_GZ_PARSERS=str(parsers))
        rs = [bench.cli_run(bench.PRODUCT_CLI, pat, gz, args.threads, os.path.join(tmp, "o.vaf"), 21, env=env)
              for _ in range(args.reps)]
        os.environ["VAFC_GZ_PARSERS"] = str(parsers)
        hs = []
        for _ in range(args.reps):
            t0 = time.time()
            st, _ = vafc.scan_file_parallel(gz, 21, 10_000_000, args.threads, 0)
            hs.append(st.bases / (time.time() - t0) / 1e6)
        print("parsers %d: CLI %s Mbases/s (process %s s); host-only reader %s Mbases/s" % (
            parsers, [round(r["mbases"]) for r in rs], [round(r["wall"], 2) for r in rs],
            [round(h) for h in hs]), flush=True)
    t0 = time.time()
    n = vafc.lib().vc_gz_inflate_parallel(gz.encode(), args.threads, 0, None, 0, None)
    print("inflate only: %.0f MB/s of text" % (n / (time.time() - t0) / 1e6), flush=True)
    for th in [int(x) for x in args.scaling.split(",") if x]:
        best = 1e9
        for _ in range(2):
            t0 = time.time()
            n = vafc.lib().vc_gz_inflate_parallel(gz.encode(), th, 0, None, 0, None)
            best = min(best, time.time() - t0)
        print("inflate only, %2d threads: %.0f MB/s of text (%.0f per thread)" % (th, n / best / 1e6, n / best / 1e6 / th),
              flush=True)
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
