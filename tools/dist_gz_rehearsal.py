#!/usr/bin/env python3
"""One gzip FASTQ over torchrun-style ranks on one GPU box (tools only): the
split-gzip path of kmer-cnt_amd/vafc_dist.py (shares of the deflate stream,
vafc_gzip.h) against the same driver at one rank.  Writes --reads reads of the
C2 stream as FASTQ in /dev/shm, gzips it the pigz way at level 1
(bench.gzip_level1), then runs the driver at 1 rank (-t T) and at N ranks
(-t T/N each, gloo, VAFC_REHEARSAL=1: every rank on GPU 0, so the N ranks
share the one box's CPU share), alternately, and prints one JSON object: each
run's counting Speed line (the reference's metric), per-file line and .vaf md5.

    python tools/dist_gz_rehearsal.py [--reads 30000000] [--ranks 2] [--rounds 2]
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))
DRIVER = os.path.join(ROOT, "kmer-cnt_amd", "vafc_dist.py")


def run(n, threads, pat, gzs, out, timeout=600, hold=None, waves=True):
    env = dict(os.environ, VAFC_DIST_BACKEND="gloo", VAFC_REHEARSAL="1")
    if hold is not None:
        env["VAFC_GZ_HOLD"] = str(hold)
    if not waves:
        env["VAFC_GZ_WAVES"] = "0"
    argv = ["-v", "-k", "21", "-t", str(threads), "-p", pat, "-o", out] + list(gzs)
    t0 = time.time()
    if n == 1:
        env.pop("WORLD_SIZE", None)
        p = subprocess.run([sys.executable, DRIVER] + argv, env=env, capture_output=True, text=True, timeout=timeout)
        err, rc = p.stderr, p.returncode
    else:
        import bench
        logf = out + ".err"
        with open(logf, "w") as f:
            port = bench.free_port()
            procs = []
            for r in range(n):
                e = dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                         MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
                procs.append(subprocess.Popen([sys.executable, DRIVER] + argv, env=e, stdout=subprocess.DEVNULL,
                                              stderr=f if r == 0 else subprocess.DEVNULL))
            rc = 0
            for p in procs:
                rc = rc or p.wait(timeout=timeout)
        err = open(logf).read()
    wall = time.time() - t0
    m = re.search(r"Speed:\s+([0-9.]+) Mbases/sec", err)
    per_file = re.findall(r"^\[V::count_fastq_kmers\].*$", err, re.M)
    if rc != 0 or not m:
        raise RuntimeError("driver at %d rank(s) failed (%d): %s" % (n, rc, err[-2000:]))
    return {"mbases": float(m.group(1)), "process_wall_s": round(wall, 2), "per_file": per_file,
            "counting": re.search(r"K-mer counting:\s+([0-9.]+) sec", err).group(1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=30_000_000)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--threads", type=int, default=16, help="reader threads of the box (split over the ranks)")
    ap.add_argument("--files", type=int, default=1, help="the reads as this many gzip files (R1, R2, ...)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import vafc
    import vafc_synth as S
    dev = torch.device("cuda", 0)
    panel = S.grch38_panel()
    tmp = tempfile.mkdtemp(prefix="vafc_gzr_")
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
    work = bench.scratch_dir(R * (2 * L + 16) * 1.5, tmp)
    gzs, gz_bytes, text = [], 0, 0
    per = R // a.files
    for f in range(a.files):
        fq = os.path.join(work, "c2_%d.fq" % f)
        n = per if f + 1 < a.files else R - per * f
        bench.write_fastq_from_device(d_seq[f * per * L:], n, L, fq, threads=a.threads, first=f * per)
        gzs.append(fq + ".gz")
        gz_bytes += bench.gzip_level1(fq, gzs[-1], a.threads)
        text += os.path.getsize(fq)
        os.unlink(fq)
    del d_seq, d_offs, d_lens
    torch.cuda.empty_cache()
    sys.stderr.write("[gzr] %d reads, %.2f GB of text, %.2f GB gzip\n" % (R, text / 1e9, gz_bytes / 1e9))
    out = {"workload": "%dM x %d bp reads of the C2 stream as %d pigz-shaped level-1 gzip FASTQ file(s) (%.2f GB, "
                       "%.2f GB of text) in the page cache; k = 21, the GRCh38 panel" % (R // 10**6, L, a.files,
                                                                                        gz_bytes / 1e9, text / 1e9),
           "box": "one GPU box, %d reader threads in all: 1 rank x %d against %d ranks x %d (gloo, every rank on "
                  "GPU 0)" % (a.threads, a.threads, a.ranks, max(1, a.threads // a.ranks)),
           "runs": {"1": [], str(a.ranks): [], "%d_two_pass" % a.ranks: []}}
    legs = [(1, None, True, "1"), (a.ranks, None, True, str(a.ranks)), (a.ranks, 0, True, "%d_two_pass" % a.ranks)]
    if a.files > 1:   # the files one after another, each split over every rank
        legs.append((a.ranks, None, False, "%d_no_waves" % a.ranks))
        out["runs"]["%d_no_waves" % a.ranks] = []
    md5s = {}
    run(1, a.threads, pat, gzs, os.path.join(tmp, "warm.vaf"))
    for rep in range(a.rounds):
        # N ranks with the scans' chunks held for the count (one inflate pass,
        # the driver's default budget) and with holding off (VAFC_GZ_HOLD=0:
        # every share inflated twice)
        for n, hold, waves, key in legs:
            o = os.path.join(tmp, "r%s.vaf" % key)
            r = run(n, max(1, a.threads // n), pat, gzs, o, hold=hold, waves=waves)
            md5s[key] = bench.md5(o)
            out["runs"][key].append(r)
            sys.stderr.write("[gzr] %s rank(s), round %d: %.1f Mbases/s\n" % (key, rep + 1, r["mbases"]))
    out["vaf_identical"] = len(set(md5s.values())) == 1
    out["note"] = ("held shares: each rank's blind scan keeps its decoded chunks and the count streams them, so a "
                   "share is inflated once; two_pass: the scan's output is dropped and the count inflates the "
                   "share again from its start bit with the known window")
    print(json.dumps(out))
    for gz in gzs:
        os.unlink(gz)
    if work != tmp:
        shutil.rmtree(work, ignore_errors=True)
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
