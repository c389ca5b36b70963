#!/usr/bin/env python3
"""Host-only A/B of the two ways a gzip share is counted (tools only; no GPU):
held (vc_gz_share_open keeps the blind scan's decoded chunks, the count
streams them: one inflate pass) against two-pass (vc_gz_share_scan, then
vc_scan_gz_share inflates the share again from its start bit).  The shares of
one file are scanned and counted one after another in this process, each with
--threads threads, and the scan and count phases are timed apart; with
VAFC_GZ_PROFILE=1 the inflater's thread-seconds go to stderr.

    python tools/gz_held_ab.py [--reads 16000000] [--world 2] [--threads 8] [--rounds 2] [--gz FILE]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))


def make_gz(path, reads, threads):
    import bench
    import vafc_synth as S
    fq = path[:-3]
    rng = np.random.default_rng(7)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    with open(fq, "wb") as f:
        for a in range(0, reads, 1_000_000):
            n = min(reads, a + 1_000_000) - a
            f.write(S.fastq_bytes_np(acgt[rng.integers(0, 4, (n, 150), dtype=np.uint8)], a))
    bench.gzip_level1(fq, path, threads)
    text = os.path.getsize(fq)
    os.unlink(fq)
    return text


def one(gz, world, threads, hold):
    import vafc
    import vafc_dist as D
    size = os.path.getsize(gz)
    t0 = time.time()
    rows, ws, hs = [], [], []
    for r in range(world):
        b, e = D.byte_range(size, r, world)
        if hold:
            info, w, h = vafc.gz_share_open(gz, b, e, threads=threads, hold_bytes=hold)
        else:
            (info, w), h = vafc.gz_share_scan(gz, b, e, threads=threads), None
        rows.append((info["start_bit"], info["end_bit"], info["text_len"], info["ok"], info["ended"]))
        ws.append(w)
        hs.append(h)
    t1 = time.time()
    mem = {}
    try:   # how much of the kept text sits on huge pages
        for line in open("/proc/self/smaps_rollup"):
            if line.split(":")[0] in ("Rss", "AnonHugePages"):
                mem[line.split(":")[0]] = int(line.split()[1]) >> 10
    except OSError:
        pass
    assert D.gz_shares_chain(rows)
    wins = D.gz_windows(rows, ws)
    bases, ranges = 0, []
    close_s = 0.0
    profs = []
    for r in range(world):
        if hs[r] is not None:
            st, ri, _, _ = vafc.scan_gz_share_held(hs[r], 21, r == 0, wins[r], rows[r][2], 10_000_000, threads)
            tc = time.time()
            hs[r].close()
            close_s += time.time() - tc
        else:
            st, ri, _, _ = vafc.scan_gz_share(gz, 21, r == 0, rows[r][0], wins[r], rows[r][2], 10_000_000, threads)
        bases += st.bases
        ranges.append((ri.first, ri.next, ri.errs, ri.stopped))
        prof = vafc.ingest_profile()
        profs.append({k: round(prof[k], 3) for k in ("reader_s", "main_wait_s", "submit_s", "parse_thread_s",
                                                    "slot_wait_thread_s", "acquire_thread_s", "read_thread_s",
                                                    "worker_cpu_s", "worker_wall_s", "threads") if k in prof})
    t2 = time.time()
    assert D.chain_holds(ranges)
    return {"scan_s": round(t1 - t0, 3), "count_s": round(t2 - t1, 3), "close_s": round(close_s, 3),
            "bases": int(bases),
            "held": [h is not None for h in hs], "after_scan_mib": mem, "ingest": profs}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=16_000_000)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--hold", type=int, default=32 << 30)
    ap.add_argument("--gz", default=None)
    a = ap.parse_args()
    import bench
    tmp = None
    gz = a.gz
    text = None
    if gz is None:
        tmp = bench.scratch_dir(a.reads * 330 * 1.5, tempfile.mkdtemp(prefix="vafc_gzh_"))
        gz = os.path.join(tmp, "r.fq.gz")
        text = make_gz(gz, a.reads, a.threads)
    thp = {}
    for f in ("enabled", "defrag"):
        try:
            thp[f] = open("/sys/kernel/mm/transparent_hugepage/" + f).read().strip()
        except OSError:
            pass
    out = {"thp": thp, "gz_bytes": os.path.getsize(gz), "text_bytes": text, "world": a.world, "threads": a.threads,
           "two_pass": [], "held": []}
    for _ in range(a.rounds):
        for key, hold in (("two_pass", 0), ("held", a.hold)):
            r = one(gz, a.world, a.threads, hold)
            out[key].append(r)
            sys.stderr.write("[gzh] %s %s\n" % (key, r))
    print(json.dumps(out))
    if tmp:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
