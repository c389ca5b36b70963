#!/usr/bin/env python3
"""rocprofv3 kernel + memory-copy trace of the drop-in CLI on the whole C2
stream as plain FASTQ (tools only): writes the workload's reads to /dev/shm as
bench.py's e2e leg does, runs the CLI once untimed, then once under
    rocprofv3 --kernel-trace --memory-copy-trace --stats -d OUTDIR -o p --output-format csv -- vaf-counter ...
and prints the CLI's -v Speed line and the copy / kernel totals.
    python tools/e2e_prof.py OUTDIR [--reads N] [--threads 16]"""
import argparse
import csv
import glob
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--reads", type=int, default=100_000_000)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import vafc
    import vafc_synth as S
    dev = torch.device("cuda", 0)
    panel = S.grch38_panel()
    tmp = tempfile.mkdtemp(prefix="vafc_e2eprof_")
    pat = os.path.join(tmp, "p.txt")
    panel.write_patterns(pat, 21)
    R, L = a.reads, 150
    d_seq = torch.empty(R * L, dtype=torch.uint8, device=dev)
    d_offs = torch.empty(R, dtype=torch.int64, device=dev)
    d_lens = torch.empty(R, dtype=torch.int32, device=dev)
    win = torch.from_numpy(panel.windows().reshape(-1)).to(dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(dev)
    vafc.synth_reads(d_seq.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), 0, R, L, S.READ_SEED_R1, 0.01,
                     win.data_ptr(), dos.data_ptr(), panel.n, 0)
    torch.cuda.synchronize()
    work = bench.scratch_dir(R * (2 * L + 16) * 1.25, tmp)
    fq = os.path.join(work, "c2.fq")
    bench.write_fastq_from_device(d_seq, R, L, fq, threads=a.threads)
    del d_seq, d_offs, d_lens
    torch.cuda.empty_cache()
    cli = os.path.join(ROOT, "kmer-cnt_amd", "lib", "vaf-counter")
    bench.cli_run(cli, pat, fq, a.threads, os.path.join(tmp, "warm.vaf"), 21, timeout=300)
    os.makedirs(a.outdir, exist_ok=True)
    cmd = ["rocprofv3", "--kernel-trace", "--memory-copy-trace", "--stats", "-d", a.outdir, "-o", "p",
           "--output-format", "csv", "--", cli, "-v", "-k", "21", "-t", str(a.threads), "-p", pat,
           "-o", os.path.join(tmp, "prof.vaf"), fq]
    env = dict(os.environ, TMPDIR="/tmp")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
    sys.stdout.write("\n".join(l for l in p.stderr.splitlines() if "Speed" in l or "Total runtime" in l
                               or "K-mer counting" in l) + "\n")
    for name in ("p_kernel_stats.csv", "p_memory_copy_stats.csv"):
        for f in glob.glob(os.path.join(a.outdir, "**", name), recursive=True):
            rows = list(csv.DictReader(open(f)))
            tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e9
            print("%s: %d rows, total %.3f s" % (name, len(rows), tot))
            for r in rows[:4]:
                print("  %s calls %s total %.3f s" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"]) / 1e9))
    os.unlink(fq)
    if work != tmp:
        shutil.rmtree(work, ignore_errors=True)
    shutil.rmtree(tmp, ignore_errors=True)
    return p.returncode


if __name__ == "__main__":
    sys.exit(main())
