#!/usr/bin/env python3
"""Fixed costs of the end-to-end pass at N shards, measured on one GPU (tools
only).  The drop-in CLI counts the whole C2 stream (100M
synthetic 150 bp reads as FASTQ in /dev/shm) once with one shard and once with
N shards that all live on device 0 (VAFC_DEVICES=0,0,...), -t 16, and reports
its counting timer split by VAFC_PHASES=1: the reader's pinned-slot allocation
for every shard, the reading and counting of the file, and vc_finish (the last
batches, the shard sum, the copy of the counts).  Prints one JSON object.

    python tools/n8_projection.py [--reads 100000000] [--shards 8] [--runs 3]
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

PHASE = re.compile(r"\[P::main\] shards (\d+) threads (\d+): reserve ([0-9.]+) s, read\+count ([0-9.]+) s, "
                   r"finish ([0-9.]+) s, counting ([0-9.]+) s")


def run(cli, pat, fq, threads, devices, out):
    env = dict(os.environ, VAFC_PHASES="1", VAFC_DEVICES=devices)
    t0 = time.time()
    p = subprocess.run([cli, "-v", "-k", "21", "-t", str(threads), "-p", pat, "-o", out, fq],
                       capture_output=True, text=True, timeout=300, env=env)
    wall = time.time() - t0
    m = PHASE.search(p.stderr)
    sp = re.search(r"Speed:\s+([0-9.]+) Mbases/sec", p.stderr)
    if p.returncode != 0 or not m or not sp:
        raise RuntimeError("CLI failed: %s" % p.stderr[-2000:])
    return {"shards": int(m.group(1)), "reserve_s": float(m.group(3)), "read_count_s": float(m.group(4)),
            "finish_s": float(m.group(5)), "counting_s": float(m.group(6)), "mbases": float(sp.group(1)),
            "process_wall_s": round(wall, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=100_000_000)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import vafc
    import vafc_synth as S
    dev = torch.device("cuda", 0)
    panel = S.grch38_panel()
    tmp = tempfile.mkdtemp(prefix="vafc_n8_")
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
    out = {"workload": "%dM x %d bp reads of the C2 stream as FASTQ (%.2f GB) in %s, -t %d" % (
        R // 1_000_000, L, os.path.getsize(fq) / 1e9, work, a.threads), "runs": {}}
    vafs = {}
    cli = bench.PRODUCT_CLI
    for rep in range(a.runs):
        for n in (1, a.shards):
            key = "shards_%d" % n
            o = os.path.join(tmp, "%s.vaf" % key)
            r = run(cli, pat, fq, a.threads, ",".join(["0"] * n), o)
            out["runs"].setdefault(key, []).append(r)
            vafs[key] = bench.md5(o)
            sys.stderr.write("[n8] %s run %d: %s\n" % (key, rep + 1, json.dumps(r)))
    for key, rs in out["runs"].items():
        med = sorted(rs, key=lambda r: r["counting_s"])[len(rs) // 2]
        out[key] = {k: med[k] for k in ("reserve_s", "read_count_s", "finish_s", "counting_s", "mbases")}
    out["vaf_identical"] = len(set(vafs.values())) == 1
    print(json.dumps(out))
    os.unlink(fq)
    if work != tmp:
        shutil.rmtree(work, ignore_errors=True)
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
