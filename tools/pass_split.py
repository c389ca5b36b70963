#!/usr/bin/env python3
"""Where the plain C2 pass's time goes, device pass against parse-only (tools
only; GPU box).  Writes the C2 stream (100M x 150 bp, bench.py's generator) as
one FASTQ in /dev/shm, then alternates, for each variant and round:

  parse   the parallel reader alone (vc_scan_file_parallel, no device)
  device  the in-process product pass (vc_count_file_range over the whole
          file, warm pinned slots), as bench.py's headline step
  cli     (--cli) the drop-in CLI binary, fresh process, VAFC_INGEST_PROFILE=1

each with the reader's per-thread split (vc_ingest_profile_ex: pread, slot
copy, guess, worker CPU vs wall), the cgroup's cpu.stat delta (throttling) and
getrusage deltas.  One JSON object on stdout: every pass, and per variant and
leg the medians.

    python tools/pass_split.py [--reads N] [--rounds 5] [--cli] \\
        copy0=VAFC_SLOT_COPY=0 copy2=VAFC_SLOT_COPY=2 t15=VAFC_SLOT_COPY=2,T=15
A variant is NAME=KEY=VAL[,KEY=VAL...]; T sets its thread count.
"""
import argparse
import json
import os
import resource
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))


def cpu_stat():
    """cgroup v2 cpu.stat of this process's cgroup ({} if unreadable)."""
    for d in ("/sys/fs/cgroup",):
        try:
            with open(os.path.join(d, "cpu.stat")) as f:
                return {k: int(v) for k, v in (l.split() for l in f if l.strip())}
        except (OSError, ValueError):
            continue
    return {}


def usage(who):
    r = resource.getrusage(who)
    return {"cpu_s": r.ru_utime + r.ru_stime, "nivcsw": r.ru_nivcsw, "nvcsw": r.ru_nvcsw, "minflt": r.ru_minflt}


def delta(a, b):
    return {k: round(b[k] - a[k], 4) if isinstance(b[k], float) else b[k] - a[k] for k in b if k in a}


def cg_delta(c0, c1):
    if not (c0 and c1):
        return None
    return {"throttled_ms": round((c1.get("throttled_usec", 0) - c0.get("throttled_usec", 0)) / 1e3, 1),
            "nr_throttled": c1.get("nr_throttled", 0) - c0.get("nr_throttled", 0),
            "cg_cpu_s": round((c1.get("usage_usec", 0) - c0.get("usage_usec", 0)) / 1e6, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=100_000_000)
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--piece", type=int, default=32 << 20, help="parse-only piece bytes (the warm device pass: 32 MB)")
    ap.add_argument("--cli", action="store_true")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import vafc
    import vafc_synth as S
    T0 = a.threads or bench.rank_threads(1)
    dev = torch.device("cuda", 0)
    rows = S.read_bed(S.default_bed_path())
    panel = S.make_panel(rows)
    tmp = tempfile.mkdtemp(prefix="vafc_split_")
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
    t = time.time()
    bench.write_fastq_from_device(d_seq, R, L, fq, threads=T0)
    size = os.path.getsize(fq)
    sys.stderr.write("[split] %d reads as FASTQ (%.2f GB) in %.1fs\n" % (R, size / 1e9, time.time() - t))
    del d_seq, d_offs, d_lens
    torch.cuda.empty_cache()
    db = vafc.load_patterns(pat)
    keys, vals, _ = db.keys(21)
    kmap = vafc.KmerMap(21, keys, vals, db.n, 0)
    counts = torch.zeros(2 * db.n, dtype=torch.int32, device=dev)
    tally = torch.zeros(1, dtype=torch.int64, device=dev)
    kmap.bind_outputs(counts.data_ptr(), tally.data_ptr())

    specs = []
    for v in a.variants:
        name, rest = v.split("=", 1)
        env, thr = {}, T0
        for kv in rest.split(","):
            if not kv:
                continue
            k_, val = kv.split("=", 1)
            if k_ == "T":
                thr = int(val)
            else:
                env[k_] = val
        specs.append((name, env, thr))

    def with_env(env, fn):
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            return fn()
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    def timed(fn):
        c0, u0 = cpu_stat(), usage(resource.RUSAGE_SELF)
        t = time.perf_counter()
        fn()
        dt = time.perf_counter() - t
        rec = {"s": round(dt, 4), "text_GBs": round(size / dt / 1e9, 2), "rusage": delta(u0, usage(resource.RUSAGE_SELF)),
               "cgroup": cg_delta(c0, cpu_stat())}
        return rec

    def parse_pass(thr):
        r = timed(lambda: vafc.scan_file_parallel(fq, 21, 10_000_000, thr, a.piece))
        r["reader"] = vafc.ingest_profile()
        return r

    def device_pass(thr):
        def go():
            counts.zero_()
            tally.zero_()
            torch.cuda.synchronize()
            kmap.count_file_range(fq, 0, size, 10_000_000, thr)
        r = timed(go)
        r["reader"] = vafc.ingest_profile()
        r["mbases"] = round(R * L / r["s"] / 1e6, 1)
        return r

    def cli_pass(thr, env):
        e = dict(os.environ, VAFC_INGEST_PROFILE="1", VAFC_PHASES="1", **env)
        c0, u0 = cpu_stat(), usage(resource.RUSAGE_CHILDREN)
        r = bench.cli_run(bench.PRODUCT_CLI, pat, fq, thr, os.path.join(tmp, "cli.vaf"), 21, env=e, timeout=300)
        return {"mbases": r["mbases"], "counting_s": round(R * L / (r["mbases"] * 1e6), 4),
                "process_s": round(r["wall"], 3), "diag": r["diag"],
                "rusage": delta(u0, usage(resource.RUSAGE_CHILDREN)), "cgroup": cg_delta(c0, cpu_stat())}

    out = {"workload": "C2 stream: %dM x %d bp as one FASTQ (%.2f GB) in %s" % (R // 10**6, L, size / 1e9, work),
           "host_cpus": os.cpu_count(), "cpu_share": bench.cpu_share(), "cgroup_cpu_max": bench.cgroup_cpu_max(),
           "parse_piece": a.piece, "passes": []}
    # warm: the first pass over a fresh file is slow; the device pass pins its slots
    for name, env, thr in specs:
        with_env(env, lambda: parse_pass(thr))
        with_env(env, lambda: device_pass(thr))
        with_env(env, lambda: device_pass(thr))
    for rep in range(a.rounds):
        for name, env, thr in specs:
            for leg in ("parse", "device") + (("cli",) if a.cli else ()):
                if leg == "parse":
                    r = with_env(env, lambda: parse_pass(thr))
                elif leg == "device":
                    r = with_env(env, lambda: device_pass(thr))
                else:
                    r = cli_pass(thr, env)
                r.update(variant=name, leg=leg, round=rep, threads=thr)
                out["passes"].append(r)
                rd = r.get("reader", {})
                sys.stderr.write("[split] %s %s r%d: %s s%s\n" % (
                    name, leg, rep, r.get("s", r.get("counting_s")),
                    "" if not rd else " parse %.2f read %.2f copy %.2f cpu %.2f/wall %.2f thr-s; acquire %.2f "
                    "slot-wait %.2f; main wait %.3f submit %.3f" % (
                        rd["parse_thread_s"], rd["read_thread_s"], rd["copy_thread_s"], rd["worker_cpu_s"],
                        rd["worker_wall_s"], rd["acquire_thread_s"], rd["slot_wait_thread_s"], rd["main_wait_s"],
                        rd["submit_s"])))
    med = {}
    for name, env, thr in specs:
        for leg in ("parse", "device", "cli"):
            ps = [p for p in out["passes"] if p["variant"] == name and p["leg"] == leg]
            if not ps:
                continue
            key = "s" if leg != "cli" else "counting_s"
            m = {key: float(np.median([p[key] for p in ps]))}
            if leg != "cli":
                for f in ("parse_thread_s", "read_thread_s", "copy_thread_s", "guess_thread_s", "worker_cpu_s",
                          "worker_wall_s", "acquire_thread_s", "slot_wait_thread_s", "main_wait_s", "submit_s",
                          "main_cpu_s"):
                    m[f] = round(float(np.median([p["reader"][f] for p in ps])), 3)
            m["throttled_ms"] = float(np.median([(p["cgroup"] or {}).get("throttled_ms", 0) for p in ps]))
            med["%s/%s" % (name, leg)] = m
        p_s = med.get("%s/parse" % name, {}).get("s")
        for leg, key in (("device", "s"), ("cli", "counting_s")):
            d = med.get("%s/%s" % (name, leg))
            if d and p_s:
                d["frac_of_parse_only"] = round(p_s / d[key], 3)
    out["median"] = med
    print(json.dumps(out))
    kmap.close()
    os.unlink(fq)
    if work != tmp:
        shutil.rmtree(work, ignore_errors=True)
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
