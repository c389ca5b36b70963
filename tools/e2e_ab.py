#!/usr/bin/env python3
"""End-to-end A/B of drop-in CLI builds or settings on the whole C2 stream
(tools only).  Writes the workload's reads as FASTQ in /dev/shm (as bench.py's
e2e leg does), optionally gzip level 1, then runs the variants alternately,
`--rounds` times each, and prints one JSON object with every run's -v Speed
line and each variant's min / median / max / spread.

    python tools/e2e_ab.py [--reads N] [--gzip] [--threads 16] [--rounds 5] \\
        numa=kmer-cnt_amd/lib_ab/numa/vaf-counter nonuma=kmer-cnt_amd/lib_ab/numa/vaf-counter,VAFC_NUMA=0

A variant is NAME=CLI[,KEY=VAL...] (CLI relative to the repository root);
the key T sets that variant's -t instead of --threads.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))


def cpu_stat():
    """cgroup v2 cpu.stat (throttling counters), {} if unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (l.split() for l in f if l.strip())}
    except (OSError, ValueError):
        return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=100_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--gzip", action="store_true", help="pigz-shaped gzip level 1 (bench.py's e2e file)")
    ap.add_argument("--gzip-single", action="store_true",
                    help="one plain zlib level-1 deflate stream (gzip -1's shape: no sync-flushed pieces)")
    ap.add_argument("--bgzf", action="store_true",
                    help="BGZF-shaped gzip (bgzip's layout: independent members of 64 KiB of text, level 1)")
    ap.add_argument("--host-parse", action="store_true",
                    help="also time the parallel reader alone (vc_scan_file_parallel, no GPU) under each variant's env")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import vafc
    import vafc_synth as S
    dev = torch.device("cuda", 0)
    panel = S.grch38_panel()
    tmp = tempfile.mkdtemp(prefix="vafc_e2eab_")
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
    path = fq
    if a.gzip:
        path = fq + ".gz"
        bench.gzip_level1(fq, path, a.threads)
        os.unlink(fq)
    elif a.bgzf:
        import struct
        import zlib
        path = fq + ".gz"
        with open(fq, "rb") as f, open(path, "wb") as g:
            for b in iter(lambda: f.read(65280), b""):
                c = zlib.compressobj(1, zlib.DEFLATED, -15)
                body = c.compress(b) + c.flush()
                # FEXTRA with the BC subfield holding the member size - 1 (SAM spec, BGZF)
                hdr = b"\x1f\x8b\x08\x04" + b"\x00\x00\x00\x00" + b"\x00\xff" + struct.pack("<H", 6) + b"BC" + \
                    struct.pack("<HH", 2, 18 + len(body) + 8 - 1)
                g.write(hdr + body + struct.pack("<II", zlib.crc32(b) & 0xFFFFFFFF, len(b) & 0xFFFFFFFF))
        os.unlink(fq)
    elif a.gzip_single:
        import gzip
        path = fq + ".gz"
        with open(fq, "rb") as f, gzip.GzipFile(path, "wb", compresslevel=1, mtime=0) as g:
            for b in iter(lambda: f.read(16 << 20), b""):
                g.write(b)
        os.unlink(fq)
    specs = []
    for v in a.variants:
        name, rest = v.split("=", 1)
        parts = rest.split(",")
        env = dict(os.environ)
        thr = a.threads
        for kv in parts[1:]:
            k_, val = kv.split("=", 1)
            if k_ == "T":
                thr = int(val)
            else:
                env[k_] = val
        specs.append((name, os.path.join(ROOT, parts[0]), env, thr))
    out = {"workload": "%dM x %d bp reads of the C2 stream, %s, -t %d" % (
        R // 1_000_000, L, "gzip level 1, pigz-shaped" if a.gzip else
        ("gzip level 1, one stream (gzip -1 shape)" if a.gzip_single else
         ("BGZF, 64 KiB members, level 1" if a.bgzf else "plain FASTQ")), a.threads), "runs": {}}
    md5s = {}
    for name, cli, env, thr in specs:   # one untimed pass each: the first pass over a fresh file is slow
        bench.cli_run(cli, pat, path, thr, os.path.join(tmp, "warm.vaf"), 21, env=env, timeout=300)
    for rep in range(a.rounds):
        for name, cli, env, thr in specs:
            o = os.path.join(tmp, name + ".vaf")
            c0 = cpu_stat()
            r = bench.cli_run(cli, pat, path, thr, o, 21, env=env, timeout=300)
            c1 = cpu_stat()
            out["runs"].setdefault(name, []).append(r["mbases"])
            if r.get("diag"):
                out.setdefault("diag", {}).setdefault(name, []).append(r["diag"])
            if c0 and c1:
                out.setdefault("throttled_ms", {}).setdefault(name, []).append(
                    round((c1.get("throttled_usec", 0) - c0.get("throttled_usec", 0)) / 1000, 1))
                out.setdefault("cpu_s", {}).setdefault(name, []).append(
                    round((c1.get("usage_usec", 0) - c0.get("usage_usec", 0)) / 1e6, 2))
            md5s[name] = bench.md5(o)
            sys.stderr.write("[e2e_ab] %s round %d: %.1f Mbases/s\n" % (name, rep + 1, r["mbases"]))
    if a.host_parse:   # the reader alone: pieces parsed into host slots, nothing shipped
        import time
        for rep in range(a.rounds):
            for name, cli, env, thr in specs:
                saved = {k_: os.environ.get(k_) for k_ in env if k_.startswith("VAFC_")}
                for k_ in saved:
                    os.environ[k_] = env[k_]
                t = time.time()
                vafc.scan_file_parallel(path, 21, 10_000_000, threads=thr, piece_bytes=16 << 20)
                dt = time.time() - t
                for k_, v_ in saved.items():
                    if v_ is None:
                        os.environ.pop(k_, None)
                    else:
                        os.environ[k_] = v_
                out.setdefault("host_parse_gbs", {}).setdefault(name, []).append(
                    round(os.path.getsize(path) / dt / 1e9, 2))
    for name, xs in out["runs"].items():
        s = sorted(xs)
        med = s[len(s) // 2]
        out[name] = {"min": s[0], "median": med, "max": s[-1], "spread": round((s[-1] - s[0]) / med, 3)}
    out["vaf_identical"] = len(set(md5s.values())) == 1
    print(json.dumps(out))
    os.unlink(path)
    if work != tmp:
        shutil.rmtree(work, ignore_errors=True)
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
