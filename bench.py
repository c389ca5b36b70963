#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X vaf-counter hot path.

Metric (BASELINE.json): Mbases/sec (+ k-mers/sec) on 150 bp FASTQ, k=21, as
the reference defines it: bases / counting-phase wall clock
(vaf-counter.c:646-651,707), FASTQ parse, PCIe and kernels included.
Workload (configs[1], "C2"): 100M synthetic 150 bp reads against the
SNP_GRCh38_hg38_wChr panel (20,849 ACGT patterns), generated on the device by
the counter-based generator of kmer-cnt_amd/vafc_synth.py and written once as
one 4-line FASTQ file (31.5 GB) into the page cache (/dev/shm).

One step = one pass of the product over the whole file: every rank counts
its byte range of the file (vc_count_file_range, the torchrun driver's split,
kmer-cnt_amd/vafc_dist.py) into its GPU's counts, then ONE all-reduce of the
uint32 counts and the k-mer tally (RCCL with the "nccl" backend).  W untimed
steps, then K timed steps between a barrier + torch.cuda.synchronize() on
both sides; the time is the maximum over ranks.  value = bases of the file x
K / that time.  The file is fixed, so N GPUs split the same work ("scaling":
"strong").  `python bench.py --gpus N` starts N rank processes itself (one per
GPU, before any GPU call) unless it runs under torchrun already, whose
WORLD_SIZE must then equal N.

Also reported:
  steps_detail  per timed step: wall, the slowest rank's counting seconds and
                its reader profile (vc_ingest_profile: main-thread waits,
                H2D submits, parse and slot waits), so a slow step names its
                phase.
  roofline      the counting kernel on HBM-resident reads (1 B
                per base + 8 B per read; the layout's 12 B/read beside it) /
                its HIP-event-timed duration, against 8 TB/s HBM3E; traffic
                from a committed rocprofv3 PMC summary (profiles/pmc_summary.json).
                Its kernel-side Mbases/s is `kernel_value`.
  cpu_baseline  the REAL reference vaf-counter (oracle/_ref, compiled from the
                reference sources) on a bounded sample of the same reads
                written as FASTQ, timed by its own -v "Speed" line; median of
                3 at -t 1 / 4 / 16 / nproc, the best median.
  parity        the product's .vaf on that sample vs the reference's (md5);
                the whole file's counts vs the product's vc_count_device on
                the same HBM reads (self-consistency at full size).
  cli           (N = 1) the drop-in CLI binary on the same file, plain and
                gzip level 1, its own -v Speed line, with a stage roofline.
--config c3 / c4 / c5 (the other BASELINE.json configs) measure the counting
kernel on HBM-resident reads only (value = kernel-side Mbases/s).
"""
import argparse
import hashlib
import json
import mmap
import os
import re
import shutil
import struct
import subprocess
import sys
import tempfile
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
PRODUCT_CLI = os.path.join(ROOT, "kmer-cnt_amd", "lib", "vaf-counter")
REF_CLI = os.path.join(ROOT, "oracle", "_ref", "vaf-counter")
PORT_CLI = os.path.join(ROOT, "oracle", "build", "vaf-counter-oracle")


def log(msg):
    sys.stderr.write("[bench] %s\n" % msg)
    sys.stderr.flush()


def cpu_share(gpus=1):
    """Host threads this process may use: the affinity mask, at most 16 per GPU
    (the GPU box's CPU share; os.cpu_count() there is the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16 * gpus, n))


# What bounds the counting kernel below its HBM roofline (PMC of the closing
# kernels).  Panels of more than 65,536 keys take the
# large-panel path (LDS Bloom filter + L2 second-level filter).
LIMITER_FLANK = ("the roofline is HBM (integer byte work, no MFMA); the kernel runs below it, bound by VALU "
                 "issue: 9.9 VALU per base (2.32 G per C2 launch, about 158 per 16-base chunk-wave, 64 of them "
                 "the flank lookups); an ablation in one process puts 85 % of the time in instruction issue "
                 "(VALU-only variant 4.19 of 4.93 ms), 10 % in the hit path, 4 % in the read loads and 0.6 % in "
                 "the LDS lookups (their bank conflicts, 0.70 of the LDS cycles, hide behind the other waves); "
                 "HBM requests are 1.48x the algorithmic bytes (the waves' live read lines, 4.9 MB per XCD, "
                 "overflow its 4 MB L2 and are fetched again), not the limit; DESIGN.md sections 3.1.1-3.1.2, "
                 "profiles/r05final_c2_pmc_counters.json, profiles/r04c_ablation_time.log")
LIMITER_LARGE_PANEL = ("the roofline is HBM (integer byte work, no MFMA); the large-panel kernel runs far below "
                       "it, bound by VALU issue and the L1 tag rate of its gathers: 9.3 % of windows pass the "
                       "144 KiB LDS Bloom filter (about 6 % is that size's information limit for 200k SNP pairs); "
                       "an ablation puts 57 % of the time in the scan (Bloom lookups at 9 VALU a window), 15 % in "
                       "the hit loop, 10 % in the drains' arithmetic, 15 % in the gathers into the L2-resident "
                       "second-level filter (64 distinct lines per instruction) and 3 % in the exact-table probes; "
                       "21.4 VALU per base (5.01 G per launch), TA busy 3.73 G cycles over 256 CUs; DESIGN.md "
                       "section 3.1.3, profiles/r05v3_c5_pmc_counters.json, profiles/r05ab_abl_time.log")


def cli_run(binary, pat, fq, threads, out, k, env=None, timeout=900):
    """A vaf-counter CLI (reference or drop-in) with -v: its own counting-phase
    Speed line (bases / counting wall clock, vaf-counter.c:707) and k-mer rate."""
    t0 = time.time()
    p = subprocess.run([binary, "-v", "-k", str(k), "-t", str(threads), "-p", pat, "-o", out, fq],
                       capture_output=True, text=True, timeout=timeout, env=env)
    wall = time.time() - t0
    m = re.search(r"Speed:\s+([0-9.]+) Mbases/sec", p.stderr)
    km = re.search(r"K-mer throughput:\s+([0-9.]+) million", p.stderr)
    bases = re.search(r"Bases processed:\s+([0-9]+)", p.stderr)
    if p.returncode != 0 or not m:
        raise RuntimeError("%s failed: %s" % (binary, p.stderr[-2000:]))
    diag = re.findall(r"^\[(?:ingest|P::main)\].*$", p.stderr, re.M)   # VAFC_INGEST_PROFILE / VAFC_PHASES lines
    return {"mbases": float(m.group(1)), "mkmers": float(km.group(1)) if km else None, "wall": wall,
            "bases": int(bases.group(1)) if bases else None, "diag": diag}


def cgroup_cpu_max():
    """The process's cgroup v2 CPU quota ("max 100000" = none), or None."""
    try:
        with open("/proc/self/cgroup") as f:
            rel = f.read().strip().split("::")[-1]
    except (OSError, IndexError):
        rel = ""
    # the cgroup's own directory, or the namespace root (a container's cgroup
    # namespace shows its cgroup as "/" while /proc/self/cgroup names the host path)
    for d in ("/sys/fs/cgroup" + rel, "/sys/fs/cgroup"):
        try:
            with open(os.path.join(d, "cpu.max")) as f:
                return f.read().strip()
        except OSError:
            continue
    return None


def md5(path):
    h = hashlib.md5()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def write_fastq_from_device(d_seq, n, L, path, threads=8, first=0):
    """The first n HBM-resident reads as 4-line FASTQ (@r<i>, qualities 'I');
    records are built by `threads` threads (vafc_synth.fastq_bytes_np, the
    bytes of vafc_synth.fastq_bytes) and written in order."""
    import vafc_synth as S
    step = 500_000

    def piece(a):
        b = min(n, a + step)
        return S.fastq_bytes_np(d_seq[a * L:b * L].cpu().numpy().reshape(b - a, L), first + a)

    with open(path, "wb") as f, ThreadPoolExecutor(max(1, threads)) as ex:
        for blob in ex.map(piece, range(0, n, step)):
            f.write(blob)


def scratch_dir(need_bytes, fallback):
    """/dev/shm (memory-backed: the files are page-cached by construction) when it
    has room for need_bytes with a margin, else `fallback`."""
    try:
        st = os.statvfs("/dev/shm")
        if st.f_bavail * st.f_frsize > 2 * need_bytes:
            return tempfile.mkdtemp(prefix="vafc_e2e_", dir="/dev/shm")
    except OSError:
        pass
    return fallback


def pinned_h2d_gbs(dev, nbytes=1 << 30, reps=5):
    """Host-to-device copy rate from pinned memory (the rate the CLI's staged
    batches can reach): best of `reps` 1 GiB copies timed with HIP events."""
    import torch
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    best = 0.0
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        d.copy_(h, non_blocking=True)
        e1.record()
        e1.synchronize()
        best = max(best, nbytes / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    del h, d
    return best


def vaf_counts(path):
    """(ref, alt) counts of a .vaf file as the interleaved uint32 vector counts[2i], counts[2i+1]."""
    ref, alt = [], []
    with open(path) as f:
        for line in f:
            if line.startswith("#") or line.startswith("CHR\t"):
                continue
            p = line.split("\t")
            ref.append(int(p[5]))
            alt.append(int(p[6]))
    out = np.zeros(2 * len(ref), np.uint32)
    out[0::2] = ref
    out[1::2] = alt
    return out


def gzip_level1(src, dst, threads, chunk=16 << 20):
    """One gzip member of src at zlib level 1, compressed by `threads` threads
    the way pigz does it: 16 MB pieces, each primed with the previous 32 KiB as
    its dictionary and sync-flushed (the last one finished), concatenated into
    one deflate stream; CRC-32 and length trailer over the whole text."""
    import vafc
    size = os.path.getsize(src)
    if size == 0:   # an empty member
        with open(dst, "wb") as g:
            g.write(b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x04\x03" + zlib.compress(b"", 1)[2:-4] +
                    struct.pack("<II", 0, 0))
        return os.path.getsize(dst)
    with open(src, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    try:
        view = memoryview(mm)

        def piece(a):
            b = min(size, a + chunk)
            kw = {"zdict": bytes(view[a - 32768:a])} if a >= 32768 else \
                ({"zdict": bytes(view[:a])} if a else {})
            co = zlib.compressobj(1, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY, **kw)
            return co.compress(view[a:b]) + co.flush(zlib.Z_FINISH if b == size else zlib.Z_SYNC_FLUSH)

        arr = np.frombuffer(mm, np.uint8)
        crc = int(vafc.lib().vc_gz_crc32(0, arr.ctypes.data, size))
        with open(dst, "wb") as g, ThreadPoolExecutor(threads) as ex:
            g.write(b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x04\x03")   # XFL 4 = fastest, OS unix
            for z in ex.map(piece, range(0, size, chunk)):
                g.write(z)
            g.write(struct.pack("<II", crc, size & 0xFFFFFFFF))
        del arr
        view.release()
    finally:
        mm.close()
    return os.path.getsize(dst)


def cli_leg(d_seq, L, k, pat, tmp, n_reads, cpu, devices=None, dev=None, device_vaf=None, kernel_s=None,
            fq=None):
    """The drop-in CLI binary end to end on a page-cached FASTQ of the first
    n_reads HBM reads (plain, gzip), median of VAFC_CLI_RUNS (3) runs each;
    fq: that FASTQ when the caller wrote it already (kept).

    device_vaf: md5 of the .vaf that count_device gives on the same HBM reads
    -- the CLI's .vaf on the file must equal it (a full-size bit-exact check;
    the reference itself is checked on the 2M-read sample).  kernel_s: the
    counting kernels' time for these reads (for the roofline split).
    devices: several GPUs in the one CLI process (VAFC_DEVICES,
    vc_create_multi: pieces dealt round robin, one RCCL reduce)."""
    import vafc
    t = cpu_share(len(devices) if devices else 1)
    est = n_reads * (2 * L + 16)
    own_fq = fq is None
    if own_fq:
        work = scratch_dir(est * 1.25, tmp)
        fq = os.path.join(work, "e2e.fq")
        t0 = time.time()
        write_fastq_from_device(d_seq, n_reads, L, fq, threads=t)
        log("cli: %d reads as FASTQ in %s in %.1fs" % (n_reads, work, time.time() - t0))
    else:
        work = os.path.dirname(fq)
    gz = os.path.join(work, "cli.fq.gz")
    fq_bytes = os.path.getsize(fq)
    t0 = time.time()
    gz_bytes = gzip_level1(fq, gz, t)
    log("cli: gzip level 1 (%.2f GB) in %.1fs" % (gz_bytes / 1e9, time.time() - t0))
    out = {"workload": "%dM x %d bp reads (%.2f Gbases) of this workload as 4-line FASTQ (%.2f GB), "
                       "page-cached (%s); k=%d, same panel" % (
                           n_reads // 1_000_000, L, n_reads * L / 1e9, fq_bytes / 1e9,
                           "tmpfs" if work.startswith("/dev/shm") else "disk", k),
           "reads": n_reads, "threads": t, "host_cpus": os.cpu_count(), "cpu_share": cpu_share(),
           "cgroup_cpu_max": cgroup_cpu_max(),
           "timer": "CLI -v Speed line: bases / counting-phase wall clock (from the first file open, the "
                    "reader's buffer allocation included, to the counts on the host), as the reference's "
                    "vaf-counter.c:646-651,707; process start, HIP init and table upload are outside it, "
                    "as the reference's map creation is; process_wall_s is the whole process"}
    env = dict(os.environ)
    env.pop("VAFC_DEVICES", None)
    env["VAFC_DEVICE"] = os.environ.get("LOCAL_RANK", "0")
    if devices:
        env["VAFC_DEVICES"] = ",".join(str(d) for d in devices)
        out["devices"] = list(devices)
        out["multi_gpu"] = ("one CLI process over %d GPUs: the parallel reader's pieces dealt round robin to "
                            "one shard per GPU, one RCCL reduce of the counts before the .vaf is written"
                            % len(devices))
    vafs = {}
    n_runs = int(os.environ.get("VAFC_CLI_RUNS", "3"))
    for name, path in (("plain", fq), ("gzip", gz)):
        # one untimed run first: the first pass over a freshly written 31.5 GB
        # file ran at half speed or less on every box (profiles/r04c_n8_projection.json,
        # profiles/r04c_numa_ab.json: 7.4 and 14.0 Gbases/s against 15-27 after it)
        cli_run(PRODUCT_CLI, pat, path, t, os.path.join(tmp, "e2e_warm.vaf"), k, env=env, timeout=180)
        runs = []
        for rep in range(n_runs):
            o = os.path.join(tmp, "e2e_%s.vaf" % name)
            # a run takes seconds; a hang (e.g. in a multi-GPU RCCL set-up) ends the
            # leg after 3 minutes instead of holding the whole bench line back
            r = cli_run(PRODUCT_CLI, pat, path, t, o, k, env=env, timeout=180)
            runs.append(r)
            log("cli %s -t %d (run %d): %.1f Mbases/s counting phase, %.2fs process" %
                (name, t, rep + 1, r["mbases"], r["wall"]))
        vafs[name] = md5(o)
        srt = sorted(runs, key=lambda r: r["mbases"])
        med = srt[len(srt) // 2]
        out[name] = {"value": med["mbases"], "unit": "Mbases/sec",
                     "min": srt[0]["mbases"], "median": med["mbases"], "max": srt[-1]["mbases"],
                     "spread": round((srt[-1]["mbases"] - srt[0]["mbases"]) / med["mbases"], 3),
                     "spread_inner": round((srt[-2]["mbases"] - srt[1]["mbases"]) / med["mbases"], 3)
                     if len(srt) >= 4 else None,
                     "counting_s": round(med["bases"] / (med["mbases"] * 1e6), 3) if med["bases"] else None,
                     "process_wall_s": round(med["wall"], 3),
                     "process_mbases": round(med["bases"] / med["wall"] / 1e6, 1) if med["bases"] else None,
                     "kmers_per_sec": med["mkmers"] * 1e6 if med["mkmers"] else None,
                     "runs": [r["mbases"] for r in runs],
                     "runs_note": "after one untimed run; value = median"}
    bases = n_reads * L
    out["gzip"]["format"] = ("one gzip member, zlib level 1 (gzip -1's algorithm), compressed the way pigz "
                             "does (16 MB pieces, 32 KiB dictionary carried, sync-flushed), %.2f GB" % (gz_bytes / 1e9))
    if cpu:
        ref_wall = bases / (cpu["value"] * 1e6)
        for name in ("plain", "gzip"):
            out[name]["vs_cpu_baseline"] = round(out[name]["value"] / cpu["value"], 1)
            out[name]["vs_reference_process_wall"] = round(ref_wall / out[name]["process_wall_s"], 1)
        out["reference_wall_s_est"] = round(ref_wall, 1)
        out["reference_wall_note"] = ("the reference's counting time for these bases at the cpu_baseline rate "
                                      "(its full-file run, about %.0f s, is not repeated here); "
                                      "vs_reference_process_wall = that / the CLI's whole-process wall" % ref_wall)

    # -- roofline of the end-to-end pass: which stage limits it
    try:
        h2d_bytes = bases + 12 * n_reads             # read bytes + u64 offset + u32 length per read
        pin = pinned_h2d_gbs(dev) if dev is not None else None
        st0 = time.time()
        vafc.scan_file_parallel(fq, k, 10_000_000, t, 16 << 20)
        parse_s = time.time() - st0
        st0 = time.time()
        vafc.lib().vc_gz_inflate_parallel(gz.encode(), t, 0, None, 0, None)
        inflate_s = time.time() - st0
        roof = {"h2d_bytes": h2d_bytes, "text_bytes": fq_bytes, "pcie_peak_GBs": 63.0,
                "pinned_h2d_GBs": round(pin, 1) if pin else None,
                "parse_only_s": round(parse_s, 3), "parse_only_GBs": round(fq_bytes / parse_s / 1e9, 2),
                "inflate_only_s": round(inflate_s, 3), "inflate_only_GBs": round(fq_bytes / inflate_s / 1e9, 2),
                "kernel_s": round(kernel_s, 4) if kernel_s else None,
                "note": "per stage: its time for this file at its own ceiling / the CLI's counting wall; the "
                        "stage nearest 1.0 limits the pass (stages overlap: reader threads, PCIe copies and "
                        "kernels run concurrently).  parse_only = the same parallel reader with no device "
                        "(vc_scan_file_parallel, same -t); inflate_only = the parallel inflater alone"}
        for name in ("plain", "gzip"):
            wall = out[name]["counting_s"]
            if not wall:
                continue
            stages = {"h2d": h2d_bytes / ((pin or 63.0) * 1e9) / wall,
                      "parse": parse_s / wall,
                      "kernel": (kernel_s or 0.0) / wall}
            if name == "gzip":
                stages["inflate"] = inflate_s / wall
            roof[name] = {"h2d_GBs": round(h2d_bytes / wall / 1e9, 2),
                          "h2d_frac_of_pcie_peak": round(h2d_bytes / wall / 63e9, 3),
                          "text_GBs": round(fq_bytes / wall / 1e9, 2),
                          "stage_frac": {a: round(b, 3) for a, b in stages.items()},
                          "limiter": max(stages, key=stages.get)}
        out["roofline"] = roof
    except Exception as e:  # never hide the measured line
        log("cli roofline failed: %r" % (e,))
    if device_vaf is not None:
        out["parity_vs_count_device_full_size"] = vafs["plain"] == device_vaf and vafs["gzip"] == device_vaf
        out["parity_full_size_note"] = ("self-consistency, not reference parity: the CLI's .vaf on the whole "
                                        "file (plain and gzip) equals the .vaf from the product's own "
                                        "vc_count_device on the same %d HBM reads; the reference itself is "
                                        "checked on the cpu_baseline sample (parity_vs_reference_on_sample)"
                                        % n_reads)
    if devices:   # the single-device CLI on the same file
        o = os.path.join(tmp, "e2e_1gpu.vaf")
        env1 = dict(env)
        env1.pop("VAFC_DEVICES", None)
        r = cli_run(PRODUCT_CLI, pat, fq, cpu_share(), o, k, env=env1)
        out["single_gpu_same_file"] = {"value": r["mbases"], "unit": "Mbases/sec", "threads": cpu_share()}
        out["parity_vs_single_gpu"] = vafs["plain"] == md5(o) and vafs["gzip"] == vafs["plain"]
    os.unlink(gz)
    if own_fq:
        os.unlink(fq)
        if work != tmp:
            shutil.rmtree(work, ignore_errors=True)
    return out


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(argv, n, script=None):
    """`--gpus N` outside torchrun: N rank processes of this script, one per
    GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1),
    started before this process touches the GPU.  Rank 0 prints the JSON line
    (its stdout is ours).  Returns 0, or the exit status of the first rank to
    fail (the others are then stopped)."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    alive = set(range(n))
    while alive:
        for r in sorted(alive):
            x = procs[r].poll()
            if x is None:
                continue
            alive.discard(r)
            if x != 0 and rc == 0:
                rc = x if x > 0 else 1
                log("rank %d exited with %d: stopping the other ranks" % (r, x))
                for o in alive:
                    procs[o].terminate()
        time.sleep(0.1)
    for p in procs:
        p.wait()
    return rc


def rank_threads(world):
    """Reader threads per rank: the CPU share of one GPU (16 on the GPU pool),
    no more than the affinity mask or the cgroup's CPU quota split over the
    ranks on this node."""
    if os.environ.get("VAFC_BENCH_THREADS"):      # experiments: a fixed count per rank
        return max(1, int(os.environ["VAFC_BENCH_THREADS"]))
    n = cpu_share(1)
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    n = min(n, max(1, aff // world))
    q = cgroup_cpu_max()
    if q and not q.startswith("max"):
        try:
            quota, period = (int(x) for x in q.split()[:2])
            n = min(n, max(1, quota // period // world))
        except ValueError:
            pass
    return max(1, n)


def kernel_leg(kmap, d_seq, d_offs, d_lens, R, L, steps, warmup, world, dist, counts, tally):
    """The counting kernel on HBM-resident reads: `warmup` + `steps` launches
    of vc_count_device over this rank's R reads (N > 1: plus the RCCL
    all-reduce of the counts), all on torch's current stream with no host
    synchronisation inside; returns (wall seconds of the timed launches, max
    over ranks; per-launch kernel ms from HIP events)."""
    import torch
    kmap.bind_outputs(counts.data_ptr(), tally.data_ptr())
    kmap.set_timing(True)
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        counts.zero_()
        tally.zero_()
        kmap.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr(), d_lens.data_ptr(), R, stream)
        if world > 1:
            for x in [dist.all_reduce(counts, async_op=True), dist.all_reduce(tally, async_op=True)]:
                x.wait()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
        kernel_ms.append(kmap.kernel_ms())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=counts.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kmap.set_timing(False)
    return elapsed, kernel_ms


def headline_leg(kmap, fq, k, steps, warmup, rank, world, dist, cpu_group, dev, n_pat):
    """The reference's metric on the whole file, every rank counting its byte
    range (vafc_dist.byte_range, vc_count_file_range) into its GPU, one
    all-reduce per step; W untimed + K timed steps between barriers and
    device synchronisations, time = max over ranks.  Returns the e2e dict
    (rank 0) and the all-reduced counts of the last step (uint32)."""
    import torch
    import vafc
    import vafc_dist as D
    threads = rank_threads(world)
    size = os.path.getsize(fq)
    begin, end = D.byte_range(size, rank, world)
    counts = torch.zeros(2 * n_pat, dtype=torch.int32, device=dev)
    tally = torch.zeros(1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    kmap.bind_outputs(counts.data_ptr(), tally.data_ptr())
    block = 10_000_000            # the reference's default -b

    def step():
        counts.zero_()
        tally.zero_()
        torch.cuda.synchronize()  # the fills (torch's stream) before the count (the map's own stream)
        a = time.perf_counter()
        st, ri = kmap.count_file_range(fq, begin, end, block, threads)   # returns with its stream synced
        c = time.perf_counter() - a
        prof = vafc.ingest_profile()
        if world > 1:
            dist.all_reduce(counts)
            dist.all_reduce(tally)
        torch.cuda.synchronize()
        return st, ri, c, time.perf_counter() - a, prof

    for w in range(warmup):
        st, ri, c, sw, _ = step()
        log("rank %d e2e warmup %d: %.3f s (count %.3f s)" % (rank, w + 1, sw, c))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    rec = []
    t0 = time.perf_counter()
    for _ in range(steps):
        st, ri, c, sw, prof = step()
        rec.append((sw, c, prof))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    bases, seqs, km = int(st.bases), int(st.seqs), int(tally.item())
    info = (int(ri.first), int(ri.next), int(ri.errs), int(ri.stopped))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        v = torch.tensor([bases, seqs], dtype=torch.int64, device=dev)
        dist.all_reduce(v)
        bases, seqs = (int(x) for x in v.tolist())
        infos = [None] * world
        recs = [None] * world
        dist.all_gather_object(infos, info, group=cpu_group)
        dist.all_gather_object(recs, rec, group=cpu_group)
    else:
        infos, recs = [info], [rec]
    final = counts.cpu().numpy().view(np.uint32).copy()
    kmap.bind_outputs(0, 0)
    if rank != 0:
        return None, final
    exact = D.chain_holds(infos)
    per_step = []
    for i in range(steps):
        slow = max(range(world), key=lambda r: recs[r][i][1])
        per_step.append({"ms": round(1e3 * max(recs[r][i][0] for r in range(world)), 1),
                         "count_ms": round(1e3 * recs[slow][i][1], 1), "slowest_rank": slow,
                         "reader": recs[slow][i][2]})
    rates = sorted(bases / (p["ms"] * 1e-3) / 1e6 for p in per_step)
    med = rates[len(rates) // 2]
    e2e = {"value": round(bases * steps / elapsed / 1e6, 1), "unit": "Mbases/sec",
           "kmers_per_sec": round(km * steps / elapsed, 1),
           "bases": bases, "seqs": seqs, "kmers": km, "file_bytes": size, "threads_per_rank": threads,
           "ranks": world, "elapsed_s": round(elapsed, 4),
           "step_mbases": {"min": round(rates[0], 1), "median": round(med, 1), "max": round(rates[-1], 1),
                           "spread": round((rates[-1] - rates[0]) / med, 3)},
           "split_exact": exact, "ranges": [list(x) for x in infos],
           "steps_detail": per_step,
           "timer": "per rank: zero the counts, vc_count_file_range over its byte range (first file open to "
                    "its counts final on the GPU: parse, pinned staging, H2D, kernels), then the all-reduce; "
                    "K steps between barriers, max over ranks -- the reference's counting-phase clock "
                    "(vaf-counter.c:646-651,707) plus the reduction its single process does not need"}
    if not exact:
        log("e2e: the ranks' byte ranges did not chain (%s): counts not exact" % (infos,))
    return e2e, final


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="timed steps (passes over the file; c3-c5: launches)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=None, help="reads per GPU (c2: of the file; c4: in total)")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--f-snp", type=float, default=0.01)
    ap.add_argument("--panel", default="grch38", choices=["grch38", "syn200k"])
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="BASELINE.json configs: c2 (default, the headline: k=21, 100M reads as FASTQ), "
                         "c3 (k=31, 100M pairs = 200M reads of 150 bp), c4 (1B reads in total split over "
                         "the GPUs), c5 (200k-SNP synthetic panel); c3-c5: the kernel on HBM-resident reads")
    ap.add_argument("--kernel-steps", type=int, default=10, help="c2: timed kernel launches for the roofline")
    ap.add_argument("--cpu-reads", type=int, default=2_000_000, help="CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline timings (the parity sample still runs)")
    ap.add_argument("--no-parity", action="store_true", help="skip the live parity sample too")
    ap.add_argument("--no-cli", action="store_true", help="skip the drop-in CLI binary leg (N = 1)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="c2 without the FASTQ file: value = the kernel on HBM-resident reads (profiling runs)")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(sys.argv[1:], args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        log("--gpus %d but WORLD_SIZE is %d: refusing to report one for the other" % (args.gpus, world))
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    strong_kernel = args.config == "c4"
    headline = args.config == "c2" and not args.no_e2e
    if args.config == "c3":
        args.k = 31
        R = 2 * (args.reads or 100_000_000)
    elif args.config == "c4":
        total = args.reads or 1_000_000_000
        base, extra = divmod(total, world)
        R = base + (1 if rank < extra else 0)
    else:
        R = args.reads or 100_000_000
    if args.config == "c5":
        args.panel = "syn200k"

    # stdout carries the one JSON line only: everything else a rank's
    # libraries print there (gloo's "[Gloo] Rank 0 is connected ..." lines)
    # goes to stderr, the line to the saved descriptor
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist
    # one GPU per rank; the modulo only matters for rehearsals with more ranks
    # than GPUs (VAFC_DIST_BACKEND=gloo), never for the driver's N-GPU runs
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = os.environ.get("VAFC_DIST_BACKEND", "nccl")
    cpu_group = None
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        # host-side group: file names, per-step records, and waiting while rank
        # 0 writes the file or runs the reference (a gloo barrier does not keep
        # an RCCL kernel spinning on the GPUs)
        cpu_group = dist.new_group(backend="gloo")
    import vafc
    import vafc_synth as S
    vafc.check_build()   # refuse binaries built from other sources than this tree

    # ---- patterns -> device table (product host path: fscanf loader + table builder)
    rows = S.read_bed(S.default_bed_path()) if args.panel == "grch38" else S.synthetic_bed(200_000)
    panel = S.make_panel(rows)
    tmp = tempfile.mkdtemp(prefix="vafc_bench_%d_" % rank)
    pat = os.path.join(tmp, "patterns.txt")
    panel.write_patterns(pat, args.k)
    db = vafc.load_patterns(pat)
    keys, vals, coll = db.keys(args.k)
    if coll and rank == 0:
        log("%d k-mer collisions in the panel (the reference warns the same)" % coll)
    kmap = vafc.KmerMap(args.k, keys, vals, db.n, local)
    tinfo = kmap.table_info()
    n_pat = db.n

    # ---- synthetic reads, resident in HBM (rank r: reads r*R .. of the stream;
    # c2: the file is rank 0's reads, every rank counts a byte range of it)
    L = args.read_len
    if strong_kernel:
        base, extra = divmod(args.reads or 1_000_000_000, world)
        first = rank * base + min(rank, extra)
    else:
        first = rank * R
    t0 = time.time()
    d_seq = torch.empty(R * L, dtype=torch.uint8, device=dev)
    d_offs = torch.empty(R, dtype=torch.int64, device=dev)
    d_lens = torch.empty(R, dtype=torch.int32, device=dev)
    win = torch.from_numpy(panel.windows().reshape(-1)).to(dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(dev)
    torch.cuda.synchronize()
    vafc.synth_reads(d_seq.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), first, R, L,
                     S.READ_SEED_R1, args.f_snp, win.data_ptr(), dos.data_ptr(), panel.n,
                     torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    log("rank %d: %d reads x %d bp generated in HBM in %.2fs" % (rank, R, L, time.time() - t0))

    # ---- the counting kernel on HBM-resident reads (roofline)
    counts = torch.zeros(2 * n_pat, dtype=torch.int32, device=dev)
    tally = torch.zeros(1, dtype=torch.int64, device=dev)
    k_steps, k_warm = (args.kernel_steps, 2) if headline else (args.steps, args.warmup)
    k_elapsed, kernel_ms = kernel_leg(kmap, d_seq, d_offs, d_lens, R, L, k_steps, k_warm, world, dist, counts, tally)
    reads_total = R
    if world > 1:
        n = torch.tensor([R], dtype=torch.int64, device=dev)
        dist.all_reduce(n)
        reads_total = int(n.item())
    k_value = reads_total * L * k_steps / k_elapsed / 1e6
    k_kmer_rate = int(tally.item()) * k_steps / k_elapsed
    k_ms = float(np.mean(kernel_ms))
    # algorithmic bytes as SURVEY.md section 8(d) defines them: 1 B per base +
    # 8 B per read (one u64 offset, or a u32 offset + length); the kernel's
    # input layout reads 12 B per read (u64 offset + u32 length), reported beside it
    alg_bytes = R * L * 1 + R * 8
    layout_bytes = R * L * 1 + R * 12
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                pj = json.load(f)
            for e in (pj if isinstance(pj, list) else [pj]):
                if (e.get("config", "c2") == args.config and e.get("reads_per_launch", e.get("reads")) == R
                        and e.get("read_len") == L and e.get("k") == args.k):
                    traffic = e.get("hbm_bytes_per_launch")
        except (OSError, ValueError, AttributeError):
            pass

    # ---- live parity on a bounded sample, at every world size: every rank
    # counts the same first n reads of the stream (rank 0's prefix) and the
    # counts are all-reduced, so the result must be N x the reference's counts
    # on that sample (u32, mod 2^32).  Rank 0 runs the reference (and the CPU
    # baseline) on the sample; the other ranks wait on the gloo barrier.
    cpu = None
    parity = None
    n = min(args.cpu_reads, R)
    stream = torch.cuda.current_stream().cuda_stream
    if not args.no_parity and n > 0:
        if first == 0:
            p_seq, p_offs, p_lens = d_seq, d_offs, d_lens
        else:   # rank r > 0: regenerate reads 0 .. n-1 of the stream
            p_seq = torch.empty(n * L, dtype=torch.uint8, device=dev)
            p_offs = torch.empty(n, dtype=torch.int64, device=dev)
            p_lens = torch.empty(n, dtype=torch.int32, device=dev)
            vafc.synth_reads(p_seq.data_ptr(), p_offs.data_ptr(), p_lens.data_ptr(), 0, n, L,
                             S.READ_SEED_R1, args.f_snp, win.data_ptr(), dos.data_ptr(), panel.n, stream)
        par_counts = torch.zeros(2 * n_pat, dtype=torch.int32, device=dev)
        par_tally = torch.zeros(1, dtype=torch.int64, device=dev)
        kmap.bind_outputs(par_counts.data_ptr(), par_tally.data_ptr())
        kmap.count_device(p_seq.data_ptr(), n * L, p_offs.data_ptr(), p_lens.data_ptr(), n, stream)
        torch.cuda.synchronize()
        par_local = par_counts.cpu().numpy().view(np.uint32).copy()
        if world > 1:
            dist.all_reduce(par_counts)
            dist.all_reduce(par_tally)
        torch.cuda.synchronize()
        par = par_counts.cpu().numpy().view(np.uint32).copy()
        log("rank %d: parity sample counted: local sum %d, after the all-reduce %d" % (
            rank, int(par_local.astype(np.uint64).sum()), int(par.astype(np.uint64).sum())))
        kmap.bind_outputs(0, 0)
    if rank == 0 and not args.no_parity and n > 0:
        kind = "reference" if os.path.exists(REF_CLI) else "port"
        binary = REF_CLI if kind == "reference" else PORT_CLI
        try:
            fq = os.path.join(tmp, "sample.fq")
            write_fastq_from_device(d_seq, n, L, fq, threads=cpu_share())
            # -t 1, -t 4, -t <CPU share> and -t nproc, median of
            # 3 each; the best median is the baseline (--no-cpu: one -t 1 run,
            # for parity only).  A thread count whose first run is under half the
            # best median so far is not repeated (it cannot be the best).
            runs = {}
            for t in (sorted({1, 4, cpu_share(), os.cpu_count() or 1}) if not args.no_cpu else []):
                rs = []
                for rep in range(3):
                    r = cli_run(binary, pat, fq, t, os.path.join(tmp, "ref_t%d.vaf" % t), args.k, timeout=600)
                    rs.append(r)
                    log("cpu %s -t %d (run %d): %.2f Mbases/s (%.1fs)" % (kind, t, rep + 1, r["mbases"], r["wall"]))
                    best_so_far = max([x["mbases"] for x in runs.values()] + [0.0])
                    if rep == 0 and r["mbases"] < 0.5 * best_so_far:
                        break
                runs[t] = sorted(rs, key=lambda r: r["mbases"])[len(rs) // 2]
            if args.no_cpu:
                cli_run(binary, pat, fq, 1, os.path.join(tmp, "ref_t1.vaf"), args.k, timeout=600)
            best_t = max(runs, key=lambda t: runs[t]["mbases"]) if runs else None
            cpu = None if not runs else {"value": runs[best_t]["mbases"], "unit": "Mbases/sec",
                   "cores": 2 + best_t if best_t > 1 else 3,
                   "kind": kind,
                   "threads_flag": best_t, "host_cpus": os.cpu_count(), "cpu_share": cpu_share(),
                   "sample": "first %d reads (%d Mbases) of this workload as FASTQ, page-cached; "
                             "reference -v Speed line, median of 3 runs per thread count (1 run where the "
                             "first was under half the best); best of %s; "
                             "cores = threads the best run kept busy: kt_pipeline's 3 workers at -t 1 (kt_for "
                             "runs inline); at -t > 1 the lookup worker waits in kt_for's join while its -t "
                             "threads run, next to the 2 other pipeline workers" % (
                                 n, n * L // 1_000_000,
                                 " / ".join("-t %d (%.2f)" % (t, runs[t]["mbases"]) for t in sorted(runs))),
                   "kmers_per_sec": runs[best_t]["mkmers"] * 1e6 if runs[best_t]["mkmers"] else None}
            ref_vaf = os.path.join(tmp, "ref_t1.vaf")
            if world == 1:   # the product's .vaf on the sample, byte for byte
                gpu_vaf = os.path.join(tmp, "gpu.vaf")
                db.write_vaf(par, gpu_vaf)
                parity = md5(gpu_vaf) == md5(ref_vaf)
            else:            # N ranks counted the sample: N x the reference's counts
                ref = vaf_counts(ref_vaf).astype(np.uint64)
                want = (ref * world) & 0xFFFFFFFF
                parity = bool(np.array_equal(par.astype(np.uint64), want))
                log("parity sample: reference sum %d, x%d = %d; all-reduced sum %d; local rank-0 rows equal to "
                    "the reference: %s; rows differing after the reduce: %d" % (
                        int(ref.sum()), world, int(want.sum()), int(par.astype(np.uint64).sum()),
                        bool(np.array_equal(par_local.astype(np.uint64), ref)),
                        int((par.astype(np.uint64) != want).sum())))
        except Exception as e:  # the baseline must never hide the measured line
            log("cpu baseline failed: %r" % (e,))

    # ---- the headline: the reference's metric on rank 0's reads as one FASTQ
    e2e = cli = None
    full_parity = None
    if headline:
        fq_path = None
        work = None
        if rank == 0:
            work = scratch_dir(R * (2 * L + 16) * 1.25, tmp)
            fq_path = os.path.join(work, "c2.fq")
            t0 = time.time()
            write_fastq_from_device(d_seq, R, L, fq_path, threads=cpu_share())
            log("e2e: %d reads as FASTQ (%.2f GB) in %s in %.1fs" % (R, os.path.getsize(fq_path) / 1e9, work,
                                                                      time.time() - t0))
        if world > 1:
            box = [fq_path]
            dist.broadcast_object_list(box, src=0, group=cpu_group)
            fq_path = box[0]
        e2e, e_counts = headline_leg(kmap, fq_path, args.k, args.steps, args.warmup, rank, world, dist,
                                     cpu_group, dev, n_pat)
        if rank == 0:
            # full-size self-consistency: the file's counts (all ranks' ranges,
            # all-reduced) == vc_count_device over the same HBM reads
            kmap.reset()
            kmap.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr(), d_lens.data_ptr(), R)
            dc, dkm = kmap.finish()
            full_parity = bool(np.array_equal(dc, e_counts)) and e2e["kmers"] == dkm and e2e["split_exact"]
            e2e["parity_vs_count_device_full_size"] = full_parity
            e2e["parity_full_size_note"] = ("self-consistency, not reference parity: the counts of the whole "
                                            "file over %d rank range(s), all-reduced, equal the product's own "
                                            "vc_count_device on the same %d HBM reads; the reference itself "
                                            "is checked on the cpu_baseline sample" % (world, R))
            if cpu:
                e2e["vs_cpu_baseline"] = round(e2e["value"] / cpu["value"], 1)
            if world == 1 and not args.no_cli:
                try:
                    dev_vaf = os.path.join(tmp, "device_e2e.vaf")
                    db.write_vaf(dc, dev_vaf)
                    cli = cli_leg(d_seq, L, args.k, pat, tmp, R, cpu, dev=dev, device_vaf=md5(dev_vaf),
                                  kernel_s=k_ms * 1e-3, fq=fq_path)
                except Exception as e:
                    log("cli leg failed: %r" % (e,))
            os.unlink(fq_path)
            if work != tmp:
                shutil.rmtree(work, ignore_errors=True)
        if world > 1:
            dist.barrier(group=cpu_group)
    elif world > 1:
        dist.barrier(group=cpu_group)

    if rank == 0:
        data_src = "SNP_GRCh38_hg38_wChr.bed" if args.panel == "grch38" else "a 200k-row synthetic BED"
        kernel_obj = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": "vc_count_reads_kernel (+ vc_count_long_kernel, empty here)",
            "limiter": (LIMITER_LARGE_PANEL if tinfo["n_keys"] > 65536 else LIMITER_FLANK),
            "kernel_ms": round(k_ms, 4),
            "kernel_launches": k_steps,
            "kernel_value": round(k_value, 1),
            "kernel_value_unit": "Mbases/sec on HBM-resident reads (no FASTQ parse, no PCIe)",
            "kernel_kmers_per_sec": round(k_kmer_rate, 1),
            "alg_bytes_per_launch": alg_bytes,
            "alg_bytes_rule": "SURVEY.md 8(d): 1 B/base + 8 B/read",
            "layout_bytes_per_launch": layout_bytes,
            "frac_layout": round(layout_bytes / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        }
        if headline:
            value, unit = e2e["value"], "Mbases/sec"
            ms_step = e2e["elapsed_s"] / args.steps * 1e3
            kmer_rate = e2e["kmers_per_sec"]
            data = ("synthetic (counter-based generator, seed 42; patterns from %s, flanks seed 12345), written "
                    "once as one 4-line FASTQ into the page cache; value = the reference's metric over the whole "
                    "file (bases / counting wall, vaf-counter.c:646-651,707): parse, pinned staging, PCIe, "
                    "kernels and the all-reduce inside every step; the kernel alone on HBM-resident reads is "
                    "roofline.kernel_value" % data_src)
            workload = ("C2: %dM x %d bp reads as one FASTQ (%.2f GB, page cache), k=%d, %s panel (%d patterns, "
                        "%d keys), f_snp=%g; %d rank(s), each counting a byte range of the file" % (
                            R // 1_000_000, L, e2e["file_bytes"] / 1e9, args.k, args.panel, n_pat,
                            tinfo["n_keys"], args.f_snp, world))
            scaling = "strong"
            parallelism = ("dp%d (byte ranges of the file per rank, RCCL all-reduce of uint32 counts + u64 tally)"
                           % world)
        else:
            value, unit = round(k_value, 1), "Mbases/sec"
            ms_step = k_elapsed / k_steps * 1e3
            kmer_rate = k_kmer_rate
            data = ("synthetic (counter-based generator, seed 42; patterns from %s, flanks seed 12345), resident "
                    "in HBM: value is the kernel on HBM-resident reads (no FASTQ parse, no PCIe)" % data_src)
            workload = ("%s: %s x %d bp reads%s, k=%d, %s panel (%d patterns, %d keys), f_snp=%g, HBM-resident"
                        % (args.config.upper(), "%gM" % (reads_total / 1e6) if strong_kernel else
                           "%dM" % (R // 1_000_000), L, " in total over the GPUs" if strong_kernel else " per GPU",
                           args.k, args.panel, n_pat, tinfo["n_keys"], args.f_snp))
            scaling = "strong" if strong_kernel else "weak"
            parallelism = "dp%d (reads sharded per rank, RCCL all-reduce of uint32 counts + u64 tally)" % world
        line = {
            "metric": "Mbases/sec (+ k-mers/sec) on %d bp FASTQ, k=%d" % (L, args.k),
            "value": value,
            "unit": unit,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": data,
            "config": {"workload": workload, "reads_per_gpu": R, "reads_total": reads_total, "read_len": L,
                       "k": args.k, "patterns": n_pat, "filter_bytes": tinfo["filter_bytes"],
                       "table_slots": tinfo["slots"], "parallelism": parallelism},
            "kmers_per_sec": round(kmer_rate, 1),
            "roofline": kernel_obj,
            "cpu_baseline": cpu,
            "vs_cpu_baseline": round(value / cpu["value"], 1) if cpu and headline else None,
            "parity_vs_reference_on_sample": parity,
            "parity_note": ("the product's .vaf on the first %d reads == the reference's (md5)" % n if world == 1 else
                            "all %d ranks count the first %d reads of the stream, %s all-reduce; == %d x the "
                            "reference's counts on that sample (u32)"
                            % (world, n, "RCCL" if backend == "nccl" else backend, world)),
            "parity_full_size": full_parity,
            "build_id": vafc.tree_build_id(),
            "e2e": e2e,
            "cli": cli,
        }
        os.write(out_fd, (json.dumps(line) + "\n").encode())
    kmap.close()
    shutil.rmtree(tmp, ignore_errors=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
