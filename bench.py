#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X vaf-counter hot path.

Metric (BASELINE.json): Mbases/sec (+ k-mers/sec) on 150 bp FASTQ, as the
reference defines it: bases / counting-phase wall clock
(vaf-counter.c:646-651,707), FASTQ parse, PCIe and kernels included.
Workloads (BASELINE.json configs), synthetic reads generated on the device by
the counter-based generator of kmer-cnt_amd/vafc_synth.py and written once as
4-line FASTQ into the page cache (/dev/shm):
  c2 (default, configs[1])  k=21, 100M x 150 bp reads, one file, the
                            SNP_GRCh38_hg38_wChr panel (20,849 patterns)
  c3 (configs[2])           k=31, 100M pairs: R1 and R2 as two files
                            (seeds 42 / 43), counted in argv order
  c5 (configs[4])           k=21, 100M reads, one file, 200k-SNP synthetic panel
  c4 (configs[3])           1B reads split over the GPUs: the counting kernel
                            on HBM-resident reads only (315 GB of FASTQ)

One step = one pass of the product over the workload's files: every rank
counts its byte range of each file (vc_count_file_range, the torchrun
driver's split, kmer-cnt_amd/vafc_dist.py) into its GPU's counts, then ONE
all-reduce of the uint32 counts and the k-mer tally (RCCL with the "nccl"
backend).  W untimed steps, then K timed steps between a barrier +
torch.cuda.synchronize() on both sides; the time is the maximum over ranks.
value = bases of the files x K / that time ("value_kind": "e2e_file").  The
files are fixed, so N GPUs split the same work ("scaling": "strong").
`python bench.py --gpus N` starts N rank processes itself (one per GPU,
before any GPU call) unless it runs under torchrun already, whose WORLD_SIZE
must then equal N; more ranks than visible GPUs is refused (exit 2).

The JSON line is kept under 4 KB; the verbose record (every step's reader
profile, every CLI run's diagnostics, notes) goes to --detail (default: a
file in the temp directory, named on stderr).  Also in the line:
  roofline      the counting kernel on HBM-resident reads (1 B
                per base + 8 B per read) / its HIP-event-timed duration, against
                8 TB/s HBM3E; traffic from a committed rocprofv3 PMC summary
                (profiles/pmc_summary.json).  kernel_value = its Mbases/s.
  cpu_baseline  the REAL reference vaf-counter (oracle/_ref, compiled from the
                reference sources) on a bounded sample of the same reads
                written as FASTQ, timed by its own -v "Speed" line; median of
                3 at -t 1 / 4 / 16 / nproc, the best median.
  parity_*      the product's .vaf on that sample vs the reference's (md5);
                the whole workload's counts vs the product's vc_count_device
                on the same HBM reads (self-consistency at full size).  Both
                also go to stderr as one "[bench] parity ..." line.
  cli           (N = 1) the drop-in CLI binary on the same files, plain and
                gzip level 1, its own -v Speed line, each run's reader phases
                (VAFC_INGEST_PROFILE), cgroup throttling and CPU seconds.
"""
import argparse
import hashlib
import json
import mmap
import os
import re
import resource
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
from vafc_dist import rank_device  # noqa: E402  (one GPU per rank; refuses more ranks than GPUs)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
PRODUCT_CLI = os.path.join(ROOT, "kmer-cnt_amd", "lib", "vaf-counter")
REF_CLI = os.path.join(ROOT, "oracle", "_ref", "vaf-counter")
PORT_CLI = os.path.join(ROOT, "oracle", "build", "vaf-counter-oracle")
LINE_BYTES_MAX = 4096      # the JSON line's size bound (tests/test_bench_helpers.py)


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
# kernels; the full account is in DESIGN.md section 3.1).  Panels of more than
# 65,536 keys take the large-panel path (LDS Bloom filter + L2 second-level filter).
LIMITER_FLANK = ("VALU issue (9.9 VALU/base; HBM requests 1.48x the algorithmic bytes); DESIGN.md 3.1.1-3.1.2")
LIMITER_LARGE_PANEL = ("VALU issue + L1 tag rate of the second-level filter gathers (LDS Bloom pass rate, "
                       "21.4 VALU/base); DESIGN.md 3.1.3")


def cgroup_dir():
    """The process's cgroup v2 directory, or the namespace root."""
    try:
        with open("/proc/self/cgroup") as f:
            rel = f.read().strip().split("::")[-1]
    except (OSError, IndexError):
        rel = ""
    # the cgroup's own directory, or the namespace root (a container's cgroup
    # namespace shows its cgroup as "/" while /proc/self/cgroup names the host path)
    for d in ("/sys/fs/cgroup" + rel, "/sys/fs/cgroup"):
        if os.path.exists(os.path.join(d, "cpu.stat")):
            return d
    return None


def cgroup_cpu_max():
    """The process's cgroup v2 CPU quota ("max 100000" = none), or None."""
    d = cgroup_dir()
    try:
        with open(os.path.join(d or "/sys/fs/cgroup", "cpu.max")) as f:
            return f.read().strip()
    except OSError:
        return None


def cgroup_cpu_stat():
    """cgroup v2 cpu.stat counters ({} if unreadable)."""
    d = cgroup_dir()
    try:
        with open(os.path.join(d or "/sys/fs/cgroup", "cpu.stat")) as f:
            return {k: int(v) for k, v in (l.split() for l in f if l.strip())}
    except (OSError, ValueError):
        return {}


INGEST_LINE = re.compile(
    r"\[ingest\] (\d+) pieces, (\d+) threads: total ([0-9.]+) s; main: wait ([0-9.]+) submit ([0-9.]+) "
    r"reparse ([0-9.]+) cpu ([0-9.]+); workers: parse ([0-9.]+) slot-wait ([0-9.]+) acquire ([0-9.]+) "
    r"\(thread-seconds\); parse split: read ([0-9.]+) \(([0-9.]+) GB\) copy ([0-9.]+) \(([0-9.]+) GB, mode (\d)\) "
    r"guess ([0-9.]+); workers cpu ([0-9.]+) of wall ([0-9.]+)")


def parse_ingest_line(line):
    """The reader's VAFC_INGEST_PROFILE line (vafc_ingest.cpp) as the compact
    dict the bench line carries, or None."""
    m = INGEST_LINE.search(line)
    if not m:
        return None
    g = [float(x) for x in m.groups()]
    return {"total": g[2], "main_wait": g[3], "submit": g[4], "parse": g[7], "slot_wait": g[8],
            "acquire": g[9], "read": g[10], "copy": g[12], "cpu": g[16], "wall": g[17]}


def reader_compact(p):
    """vafc.ingest_profile() in the bench line's compact form (thread-seconds)."""
    if not p:
        return None
    return {"total": p["reader_s"], "main_wait": p["main_wait_s"], "submit": p["submit_s"],
            "parse": p["parse_thread_s"], "slot_wait": p["slot_wait_thread_s"], "acquire": p["acquire_thread_s"],
            "read": p["read_thread_s"], "copy": p["copy_thread_s"], "cpu": p["worker_cpu_s"],
            "wall": p["worker_wall_s"], "main_cpu": p["main_cpu_s"]}


def cli_run(binary, pat, fqs, threads, out, k, env=None, timeout=900):
    """A vaf-counter CLI (reference or drop-in) with -v over one file or a list
    of files (argv order): its own counting-phase Speed line (bases / counting
    wall clock, vaf-counter.c:707) and k-mer rate; the child's CPU seconds and
    the cgroup's throttling over the run."""
    if isinstance(fqs, str):
        fqs = [fqs]
    c0 = cgroup_cpu_stat()
    u0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    t0 = time.time()
    p = subprocess.run([binary, "-v", "-k", str(k), "-t", str(threads), "-p", pat, "-o", out] + list(fqs),
                       capture_output=True, text=True, timeout=timeout, env=env)
    wall = time.time() - t0
    u1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    c1 = cgroup_cpu_stat()
    m = re.search(r"Speed:\s+([0-9.]+) Mbases/sec", p.stderr)
    km = re.search(r"K-mer throughput:\s+([0-9.]+) million", p.stderr)
    bases = re.search(r"Bases processed:\s+([0-9]+)", p.stderr)
    if p.returncode != 0 or not m:
        raise RuntimeError("%s failed: %s" % (binary, p.stderr[-2000:]))
    diag = re.findall(r"^\[(?:ingest|P::main)\].*$", p.stderr, re.M)   # VAFC_INGEST_PROFILE / VAFC_PHASES lines
    return {"mbases": float(m.group(1)), "mkmers": float(km.group(1)) if km else None, "wall": wall,
            "bases": int(bases.group(1)) if bases else None, "diag": diag,
            "cpu_s": round((u1.ru_utime + u1.ru_stime) - (u0.ru_utime + u0.ru_stime), 3),
            "throttled_ms": round((c1.get("throttled_usec", 0) - c0.get("throttled_usec", 0)) / 1e3, 1)
            if c0 and c1 else None}


def md5(path):
    h = hashlib.md5()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def write_fastq_from_device(d_seq, n, L, path, threads=8, first=0):
    """The first n HBM-resident reads of d_seq as 4-line FASTQ (@r<first+i>,
    qualities 'I'); records are built by `threads` threads
    (vafc_synth.fastq_bytes_np, the bytes of vafc_synth.fastq_bytes) and
    written in order."""
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


def cli_leg(fqs, n_reads, L, k, pat, tmp, cpu, dev=None, device_vaf=None, kernel_s=None, detail=None):
    """The drop-in CLI binary end to end on the page-cached FASTQ files `fqs`
    (argv order; plain, then gzip level 1 of each), median of VAFC_CLI_RUNS (3)
    runs each after one untimed run, every run with the reader's profile
    (VAFC_INGEST_PROFILE), its CPU seconds and the cgroup's throttling.

    device_vaf: md5 of the .vaf that count_device gives on the same HBM reads
    -- the CLI's .vaf on the files must equal it (a full-size bit-exact check;
    the reference itself is checked on the sample).  kernel_s: the counting
    kernels' time for these reads (for the stage split).  detail: a dict that
    receives the verbose record."""
    import vafc
    t = cpu_share()
    gzs = [fq + ".gz" for fq in fqs]
    t0 = time.time()
    gz_bytes = sum(gzip_level1(fq, gz, t) for fq, gz in zip(fqs, gzs))
    fq_bytes = sum(os.path.getsize(fq) for fq in fqs)
    log("cli: gzip level 1 (%.2f GB) in %.1fs" % (gz_bytes / 1e9, time.time() - t0))
    out = {"threads": t}
    det = {"timer": "CLI -v Speed line: bases / counting-phase wall clock (from the first file open, the reader's "
                    "buffer allocation included, to the counts on the host), as the reference's "
                    "vaf-counter.c:646-651,707; process start, HIP init and table upload are outside it",
           "gzip_format": "one gzip member per file, zlib level 1 compressed the way pigz does (16 MB pieces, "
                          "32 KiB dictionary carried, sync-flushed), %.2f GB" % (gz_bytes / 1e9),
           "host_cpus": os.cpu_count(), "cgroup_cpu_max": cgroup_cpu_max(), "runs": {}}
    env = dict(os.environ, VAFC_INGEST_PROFILE="1", VAFC_PHASES="1")
    env.pop("VAFC_DEVICES", None)
    env["VAFC_DEVICE"] = os.environ.get("LOCAL_RANK", "0")
    vafs = {}
    n_runs = int(os.environ.get("VAFC_CLI_RUNS", "3"))
    for name, paths in (("plain", fqs), ("gzip", gzs)):
        # one untimed run first: the first pass over a freshly written 31.5 GB
        # file ran at half speed or less on every box (profiles/r04c_n8_projection.json)
        cli_run(PRODUCT_CLI, pat, paths, t, os.path.join(tmp, "e2e_warm.vaf"), k, env=env, timeout=180)
        runs = []
        for rep in range(n_runs):
            o = os.path.join(tmp, "e2e_%s.vaf" % name)
            # a run takes seconds; a hang ends the leg after 3 minutes
            r = cli_run(PRODUCT_CLI, pat, paths, t, o, k, env=env, timeout=180)
            runs.append(r)
            log("cli %s -t %d (run %d): %.1f Mbases/s counting phase, %.2fs process, throttled %s ms" %
                (name, t, rep + 1, r["mbases"], r["wall"], r["throttled_ms"]))
        vafs[name] = md5(o)
        srt = sorted(runs, key=lambda r: r["mbases"])
        med = srt[len(srt) // 2]
        # the reader's phases of each run (summed over the files of the run),
        # as one list per phase, runs in order
        fields = ("total", "parse", "read", "copy", "cpu", "wall", "acquire", "main_wait")
        ingest = {f: [] for f in fields}
        for r in runs:
            ps = [x for x in (parse_ingest_line(l) for l in r["diag"]) if x]
            for f in fields:
                ingest[f].append(round(sum(x[f] for x in ps), 2) if ps else None)
        out[name] = {"value": med["mbases"],
                     "runs": [r["mbases"] for r in runs],
                     "counting_s": round(med["bases"] / (med["mbases"] * 1e6), 3) if med["bases"] else None,
                     "process_s": round(med["wall"], 3),
                     "throttled_ms": [r["throttled_ms"] for r in runs],
                     "cpu_s": [r["cpu_s"] for r in runs],
                     "reader": ingest}
        det["runs"][name] = [{"mbases": r["mbases"], "wall": round(r["wall"], 3), "diag": r["diag"],
                              "cpu_s": r["cpu_s"], "throttled_ms": r["throttled_ms"]} for r in runs]
    bases = n_reads * L
    if cpu:
        for name in ("plain", "gzip"):
            out[name]["vs_cpu_baseline"] = round(out[name]["value"] / cpu["value"], 1)
    # -- the stages of the end-to-end pass: which one limits it
    try:
        h2d_bytes = bases + 12 * n_reads             # read bytes + u64 offset + u32 length per read
        pin = pinned_h2d_gbs(dev) if dev is not None else None
        st0 = time.time()
        for fq in fqs:
            vafc.scan_file_parallel(fq, k, 10_000_000, t, 16 << 20)
        parse_s = time.time() - st0
        st0 = time.time()
        for gz in gzs:
            vafc.lib().vc_gz_inflate_parallel(gz.encode(), t, 0, None, 0, None)
        inflate_s = time.time() - st0
        out["parse_only_s"] = round(parse_s, 3)
        out["inflate_only_s"] = round(inflate_s, 3)
        for name in ("plain", "gzip"):
            wall = out[name]["counting_s"]
            if wall:
                out[name]["frac_of_parse_only"] = round(parse_s / wall, 3)
                if name == "gzip":
                    out[name]["frac_of_inflate_only"] = round(inflate_s / wall, 3)
        det["stages"] = {"h2d_bytes": h2d_bytes, "text_bytes": fq_bytes, "pinned_h2d_GBs": round(pin, 1) if pin else None,
                         "parse_only_GBs": round(fq_bytes / parse_s / 1e9, 2),
                         "inflate_only_GBs": round(fq_bytes / inflate_s / 1e9, 2),
                         "kernel_s": round(kernel_s, 4) if kernel_s else None,
                         "note": "parse_only = the same parallel reader with no device (vc_scan_file_parallel, "
                                 "same -t, 16 MB pieces as the CLI's first pass); inflate_only = the parallel "
                                 "inflater alone; frac_of_parse_only = parse_only_s / the CLI's counting wall"}
    except Exception as e:  # never hide the measured line
        log("cli stages failed: %r" % (e,))
    if device_vaf is not None:
        out["parity_vs_count_device"] = vafs["plain"] == device_vaf and vafs["gzip"] == device_vaf
    for gz in gzs:
        os.unlink(gz)
    if detail is not None:
        detail.update(det)
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


def headline_leg(kmap, fqs, steps, warmup, rank, world, dist, cpu_group, dev, n_pat, detail=None):
    """The reference's metric on the workload's files, every rank counting its
    byte range of each file (vafc_dist.byte_range, vc_count_file_range; files
    in argv order) into its GPU, one all-reduce per step; W untimed + K timed
    steps between barriers and device synchronisations, time = max over ranks.
    Returns the e2e dict (rank 0; None elsewhere) and the all-reduced counts
    of the last step (uint32).  The ranges of every file must chain (vafc_dist
    falls back to a whole-file count when they do not); if they did not,
    `value` is null: no headline from inexact counts."""
    import torch
    import vafc
    import vafc_dist as D
    threads = rank_threads(world)
    sizes = [os.path.getsize(fq) for fq in fqs]
    ranges = [D.byte_range(s, rank, world) for s in sizes]
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
        sts, ris, profs = [], [], []
        for fq, (begin, end) in zip(fqs, ranges):
            st, ri = kmap.count_file_range(fq, begin, end, block, threads)   # returns with its stream synced
            sts.append(st)
            ris.append(ri)
            profs.append(vafc.ingest_profile())
        c = time.perf_counter() - a
        if world > 1:
            dist.all_reduce(counts)
            dist.all_reduce(tally)
        torch.cuda.synchronize()
        return sts, ris, c, time.perf_counter() - a, profs

    for w in range(warmup):
        _, _, c, sw, _ = step()
        log("rank %d e2e warmup %d: %.3f s (count %.3f s)" % (rank, w + 1, sw, c))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    rec = []
    t0 = time.perf_counter()
    for _ in range(steps):
        sts, ris, c, sw, profs = step()
        rec.append((sw, c, profs))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    bases = sum(int(st.bases) for st in sts)
    seqs = sum(int(st.seqs) for st in sts)
    km = int(tally.item())
    info = [(int(ri.first), int(ri.next), int(ri.errs), int(ri.stopped)) for ri in ris]
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
    # per file: the ranks' ranges in rank order must chain
    exact = all(D.chain_holds([infos[r][f] for r in range(world)]) for f in range(len(fqs)))
    step_ms, count_ms, slow = [], [], []
    for i in range(steps):
        s = max(range(world), key=lambda r: recs[r][i][1])
        step_ms.append(round(1e3 * max(recs[r][i][0] for r in range(world)), 1))
        count_ms.append(round(1e3 * recs[s][i][1], 1))
        slow.append(s)
    rates = sorted(bases / (ms * 1e-3) / 1e6 for ms in step_ms)
    med = rates[len(rates) // 2]
    i_slow = max(range(steps), key=lambda i: step_ms[i])
    i_fast = min(range(steps), key=lambda i: step_ms[i])

    def reader_of(i):   # the slowest rank's reader in step i, summed over the files
        ps = [reader_compact(p) for p in recs[slow[i]][i][2]]
        return {k: round(sum(p[k] for p in ps), 2) for k in ps[0]} if ps and ps[0] else None

    e2e = {"value": round(bases * steps / elapsed / 1e6, 1) if exact else None,
           "kmers_per_sec": round(km * steps / elapsed, 1),
           "bases": bases, "seqs": seqs, "kmers": km, "file_bytes": sum(sizes), "files": len(fqs),
           "threads_per_rank": threads, "ranks": world, "elapsed_s": round(elapsed, 4),
           "step_ms": step_ms, "count_ms": count_ms,
           "step_mbases": {"min": round(rates[0], 1), "median": round(med, 1), "max": round(rates[-1], 1),
                           "spread": round((rates[-1] - rates[0]) / med, 3)},
           "reader_slowest_step": reader_of(i_slow), "reader_fastest_step": reader_of(i_fast),
           "split_exact": exact}
    if detail is not None:
        detail["steps"] = [{"ms": step_ms[i], "count_ms": count_ms[i], "slowest_rank": slow[i],
                            "reader": recs[slow[i]][i][2]} for i in range(steps)]
        detail["ranges"] = infos
        detail["timer"] = ("per rank: zero the counts, vc_count_file_range over its byte range of each file (first "
                           "file open to its counts final on the GPU: parse, pinned staging, H2D, kernels), then the "
                           "all-reduce; K steps between barriers, max over ranks -- the reference's counting-phase "
                           "clock (vaf-counter.c:646-651,707) plus the reduction its single process does not need")
    if not exact:
        log("e2e: the ranks' byte ranges did not chain (%s): counts not exact, value withheld" % (infos,))
    return e2e, final


CONFIGS = {
    # name: (k, reads per file of this rank's stream, read seeds of the files, panel)
    "c2": (21, 100_000_000, None, "grch38"),
    "c3": (31, 100_000_000, "pair", "grch38"),
    "c4": (21, None, None, "grch38"),
    "c5": (21, 100_000_000, None, "syn200k"),
}


def assemble_line(a):
    """The one JSON line from the measured pieces (dict `a`); everything here
    must stay within LINE_BYTES_MAX bytes (tests/test_bench_helpers.py), the
    parity booleans last."""
    e2e, cli, cpu = a.get("e2e"), a.get("cli"), a.get("cpu")
    headline = e2e is not None
    line = {
        "metric": "Mbases/sec (+ k-mers/sec) on %d bp FASTQ, k=%d" % (a["L"], a["k"]),
        "value": e2e["value"] if headline else round(a["k_value"], 1),
        "unit": "Mbases/sec",
        "value_kind": "e2e_file" if headline else "kernel_hbm",
        "n_gpus": a["world"],
        "steps": a["steps"],
        "warmup": a["warmup"],
        "ms_per_step": round((e2e["elapsed_s"] / a["steps"] if headline else a["k_elapsed"] / a["k_steps"]) * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if (headline or a["config"] == "c4") else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("synthetic: counter-based generator (seed 42%s), %s panel; %s" % (
            ", R2 seed 43" if a["config"] == "c3" else "", a["panel_src"],
            "4-line FASTQ in the page cache, value = bases / counting wall (vaf-counter.c:707)" if headline else
            "reads resident in HBM, value = the kernel alone")),
        "config": {"workload": a["workload"], "reads_per_gpu": a["R"], "reads_total": a["reads_total"],
                   "read_len": a["L"], "k": a["k"], "patterns": a["n_pat"], "files": a["n_files"],
                   "parallelism": a["parallelism"]},
        "kmers_per_sec": e2e["kmers_per_sec"] if headline else round(a["k_kmer_rate"], 1),
        "roofline": {"bound": "hbm", "achieved": round(a["achieved"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(a["achieved"] / HBM_PEAK_GBS, 4), "traffic": a["traffic"],
                     "kernel": "vc_count_reads_kernel", "kernel_ms": round(a["k_ms"], 4),
                     "kernel_launches": a["k_steps"], "kernel_value": round(a["k_value"], 1),
                     "alg_bytes_per_launch": a["alg_bytes"], "alg_bytes_rule": "SURVEY.md 8(d): 1 B/base + 8 B/read",
                     "limiter": a["limiter"]},
        "cpu_baseline": cpu,
        "vs_cpu_baseline": round(e2e["value"] / cpu["value"], 1) if cpu and headline and e2e["value"] else None,
        "e2e": e2e,
        "cli": cli,
        "build_id": a["build_id"],
        "detail": a.get("detail_path"),
        "parity_vs_reference_on_sample": a["parity"],
        "parity_full_size": a["full_parity"],
    }
    return line


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="timed steps (passes over the files; c4: launches)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=None,
                    help="reads per file (c2/c5; c3: per mate file; c4: in total over the GPUs)")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--k", type=int, default=None, help="k (default: the config's)")
    ap.add_argument("--f-snp", type=float, default=0.01)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS),
                    help="BASELINE.json configs: c2 (default, the headline: k=21, 100M reads, one FASTQ), c3 "
                         "(k=31, 100M pairs as R1 + R2 FASTQ), c4 (1B reads in total over the GPUs, kernel on "
                         "HBM-resident reads), c5 (200k-SNP synthetic panel, 100M reads, one FASTQ)")
    ap.add_argument("--kernel-steps", type=int, default=10, help="e2e configs: timed kernel launches for the roofline")
    ap.add_argument("--cpu-reads", type=int, default=2_000_000, help="CPU baseline sample (reads, over all files)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline timings (the parity sample still runs)")
    ap.add_argument("--no-parity", action="store_true", help="skip the live parity sample too")
    ap.add_argument("--no-cli", action="store_true", help="skip the drop-in CLI binary leg (N = 1)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="no FASTQ files: value = the kernel on HBM-resident reads (profiling runs)")
    ap.add_argument("--detail", default=None, help="where the verbose record goes (JSON)")
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
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    k_cfg, per_file, pairing, panel_name = CONFIGS[args.config]
    k = args.k or k_cfg
    strong_kernel = args.config == "c4"
    headline = not strong_kernel and not args.no_e2e
    if strong_kernel:
        total = args.reads or 1_000_000_000
        base, extra = divmod(total, world)
        R = base + (1 if rank < extra else 0)
        first = rank * base + min(rank, extra)
        parts = [(None, first, R)]
    else:
        n_file = args.reads or per_file
        # this rank's reads: file f's reads first_f .. (rank 0's are the files)
        seeds = [None, "R2"] if pairing == "pair" else [None]
        parts = [(s, rank * n_file, n_file) for s in seeds]
        R = n_file * len(seeds)

    # stdout carries the one JSON line only: everything else a rank's
    # libraries print there (gloo's "[Gloo] Rank 0 is connected ..." lines)
    # goes to stderr, the line to the saved descriptor
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist
    backend = os.environ.get("VAFC_DIST_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    dev_idx = rank_device(local, local_world, n_dev, backend, os.environ.get("VAFC_REHEARSAL") == "1")
    if dev_idx is None:
        log("local rank %d of %d but %d GPU(s) visible: one GPU per rank (a gloo rehearsal on fewer GPUs needs "
            "VAFC_DIST_BACKEND=gloo VAFC_REHEARSAL=1)" % (local, local_world, n_dev))
        sys.exit(2)
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    cpu_group = None
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        # host-side group: file names, per-step records, and waiting while rank
        # 0 writes the files or runs the reference (a gloo barrier does not keep
        # an RCCL kernel spinning on the GPUs)
        cpu_group = dist.new_group(backend="gloo")
    import vafc
    import vafc_synth as S
    vafc.check_build()   # refuse binaries built from other sources than this tree
    detail = {"argv": sys.argv[1:]}

    # ---- patterns -> device table (product host path: fscanf loader + table builder)
    rows = S.read_bed(S.default_bed_path()) if panel_name == "grch38" else S.synthetic_bed(200_000)
    panel = S.make_panel(rows)
    tmp = tempfile.mkdtemp(prefix="vafc_bench_%d_" % rank)
    pat = os.path.join(tmp, "patterns.txt")
    panel.write_patterns(pat, k)
    db = vafc.load_patterns(pat)
    keys, vals, coll = db.keys(k)
    if coll and rank == 0:
        log("%d k-mer collisions in the panel (the reference warns the same)" % coll)
    kmap = vafc.KmerMap(k, keys, vals, db.n, dev_idx)
    tinfo = kmap.table_info()
    n_pat = db.n

    # ---- synthetic reads, resident in HBM: the parts one after another, the
    # offsets absolute in d_seq (c3: R1 then R2, 100M each)
    L = args.read_len
    t0 = time.time()
    d_seq = torch.empty(R * L, dtype=torch.uint8, device=dev)
    d_offs = torch.empty(R, dtype=torch.int64, device=dev)
    d_lens = torch.empty(R, dtype=torch.int32, device=dev)
    win = torch.from_numpy(panel.windows().reshape(-1)).to(dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(dev)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream().cuda_stream

    def seed_of(s):
        return S.READ_SEED_R2 if s == "R2" else S.READ_SEED_R1

    def gen(seq, offs, lens, plist):
        at = 0
        for s, f0, n in plist:
            vafc.synth_reads(seq[at * L:].data_ptr(), offs[at:].data_ptr(), lens[at:].data_ptr(), f0, n, L,
                             seed_of(s), args.f_snp, win.data_ptr(), dos.data_ptr(), panel.n, stream)
            if at:
                offs[at:at + n] += at * L
            at += n

    gen(d_seq, d_offs, d_lens, parts)
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
    # 8 B per read (one u64 offset, or a u32 offset + length)
    alg_bytes = R * L * 1 + R * 8
    achieved = alg_bytes / (k_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                pj = json.load(f)
            for e in (pj if isinstance(pj, list) else [pj]):
                if (e.get("config", "c2") == args.config and e.get("reads_per_launch", e.get("reads")) == R
                        and e.get("read_len") == L and e.get("k") == k):
                    traffic = e.get("hbm_bytes_per_launch")
        except (OSError, ValueError, AttributeError):
            pass
    detail["kernel_ms"] = kernel_ms

    # ---- live parity on a bounded sample, at every world size: every rank
    # counts the same first reads of rank 0's files (an equal share of each
    # file) and the counts are all-reduced, so the result must be N x the
    # reference's counts on that sample (u32, mod 2^32).  Rank 0 runs the
    # reference (and the CPU baseline) on the sample; the other ranks wait.
    cpu = None
    parity = None
    n_files = len(parts)
    n_each = min(args.cpu_reads, R) // n_files
    sample_parts = [(s, 0, n_each) for s, _, _ in parts] if not strong_kernel else [(None, 0, n_each)]
    if not args.no_parity and n_each > 0:
        p_seq = torch.empty(n_files * n_each * L, dtype=torch.uint8, device=dev)
        p_offs = torch.empty(n_files * n_each, dtype=torch.int64, device=dev)
        p_lens = torch.empty(n_files * n_each, dtype=torch.int32, device=dev)
        gen(p_seq, p_offs, p_lens, sample_parts)
        par_counts = torch.zeros(2 * n_pat, dtype=torch.int32, device=dev)
        par_tally = torch.zeros(1, dtype=torch.int64, device=dev)
        kmap.bind_outputs(par_counts.data_ptr(), par_tally.data_ptr())
        kmap.count_device(p_seq.data_ptr(), p_seq.numel(), p_offs.data_ptr(), p_lens.data_ptr(), n_files * n_each,
                          stream)
        torch.cuda.synchronize()
        par_local = par_counts.cpu().numpy().view(np.uint32).copy()
        if world > 1:
            dist.all_reduce(par_counts)
            dist.all_reduce(par_tally)
        torch.cuda.synchronize()
        par = par_counts.cpu().numpy().view(np.uint32).copy()
        kmap.bind_outputs(0, 0)
    if rank == 0 and not args.no_parity and n_each > 0:
        kind = "reference" if os.path.exists(REF_CLI) else "port"
        binary = REF_CLI if kind == "reference" else PORT_CLI
        try:
            sfq = []
            for f in range(n_files):
                path = os.path.join(tmp, "sample_%d.fq" % (f + 1))
                write_fastq_from_device(p_seq[f * n_each * L:], n_each, L, path, threads=cpu_share())
                sfq.append(path)
            # -t 1, -t 4, -t <CPU share> and -t nproc, median of
            # 3 each; the best median is the baseline (--no-cpu: one -t 1 run,
            # for parity only).  A thread count whose first run is under half the
            # best median so far is not repeated (it cannot be the best).
            runs = {}
            for t in (sorted({1, 4, cpu_share(), os.cpu_count() or 1}) if not args.no_cpu else []):
                rs = []
                for rep in range(3):
                    r = cli_run(binary, pat, sfq, t, os.path.join(tmp, "ref_t%d.vaf" % t), k, timeout=600)
                    rs.append(r)
                    log("cpu %s -t %d (run %d): %.2f Mbases/s (%.1fs)" % (kind, t, rep + 1, r["mbases"], r["wall"]))
                    best_so_far = max([x["mbases"] for x in runs.values()] + [0.0])
                    if rep == 0 and r["mbases"] < 0.5 * best_so_far:
                        break
                runs[t] = sorted(rs, key=lambda r: r["mbases"])[len(rs) // 2]
            if args.no_cpu:
                cli_run(binary, pat, sfq, 1, os.path.join(tmp, "ref_t1.vaf"), k, timeout=600)
            best_t = max(runs, key=lambda t: runs[t]["mbases"]) if runs else None
            if runs:
                cpu = {"value": runs[best_t]["mbases"], "unit": "Mbases/sec",
                       # threads the best run kept busy: kt_pipeline's 3 workers at -t 1
                       # (kt_for runs inline); at -t > 1 the lookup worker waits in
                       # kt_for's join while its -t threads run, beside 2 pipeline workers
                       "cores": 2 + best_t if best_t > 1 else 3,
                       "kind": kind, "threads_flag": best_t, "host_cpus": os.cpu_count(), "cpu_share": cpu_share(),
                       "by_threads": {str(t): runs[t]["mbases"] for t in sorted(runs)},
                       "sample": "first %d reads of each of %d file(s) (%d Mbases), reference -v Speed, median of 3 "
                                 "per -t" % (n_each, n_files, n_files * n_each * L // 1_000_000)}
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
    if not args.no_parity and n_each > 0:
        del p_seq, p_offs, p_lens

    # ---- the headline: the reference's metric on rank 0's reads as FASTQ files
    e2e = cli = None
    full_parity = None
    if headline:
        fq_paths = None
        work = None
        if rank == 0:
            work = scratch_dir(R * (2 * L + 16) * 1.25, tmp)
            fq_paths = []
            at = 0
            for f, (s, f0, n) in enumerate(parts):
                path = os.path.join(work, "%s_%d.fq" % (args.config, f + 1))
                t0 = time.time()
                write_fastq_from_device(d_seq[at * L:], n, L, path, threads=cpu_share(), first=f0)
                log("e2e: file %d: %d reads as FASTQ (%.2f GB) in %s in %.1fs" % (
                    f + 1, n, os.path.getsize(path) / 1e9, work, time.time() - t0))
                fq_paths.append(path)
                at += n
        if world > 1:
            box = [fq_paths]
            dist.broadcast_object_list(box, src=0, group=cpu_group)
            fq_paths = box[0]
        e2e_detail = {}
        e2e, e_counts = headline_leg(kmap, fq_paths, args.steps, args.warmup, rank, world, dist, cpu_group, dev,
                                     n_pat, detail=e2e_detail)
        if rank == 0:
            detail["e2e"] = e2e_detail
            # full-size self-consistency: the files' counts (all ranks' ranges,
            # all-reduced) == vc_count_device over the same HBM reads
            kmap.reset()
            kmap.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr(), d_lens.data_ptr(), R)
            dc, dkm = kmap.finish()
            full_parity = bool(np.array_equal(dc, e_counts)) and e2e["kmers"] == dkm and e2e["split_exact"]
            detail["parity_full_size_note"] = (
                "self-consistency, not reference parity: the counts of the whole files over %d rank range(s), "
                "all-reduced, equal the product's own vc_count_device on the same %d HBM reads; the reference "
                "itself is checked on the cpu_baseline sample" % (world, R))
            if world == 1 and not args.no_cli:
                try:
                    dev_vaf = os.path.join(tmp, "device_e2e.vaf")
                    db.write_vaf(dc, dev_vaf)
                    cli_detail = {}
                    cli = cli_leg(fq_paths, R, L, k, pat, tmp, cpu, dev=dev, device_vaf=md5(dev_vaf),
                                  kernel_s=k_ms * 1e-3, detail=cli_detail)
                    detail["cli"] = cli_detail
                except Exception as e:
                    log("cli leg failed: %r" % (e,))
            for path in fq_paths:
                os.unlink(path)
            if work != tmp:
                shutil.rmtree(work, ignore_errors=True)
        if world > 1:
            dist.barrier(group=cpu_group)
    elif world > 1:
        dist.barrier(group=cpu_group)

    if rank == 0:
        log("parity sample=%s full_size=%s cli_vs_count_device=%s" % (
            parity, full_parity, (cli or {}).get("parity_vs_count_device")))
        detail_path = args.detail or os.path.join(tempfile.gettempdir(), "vafc_bench_detail_%d.json" % os.getpid())
        try:
            with open(detail_path, "w") as f:
                json.dump(detail, f)
            log("detail record: %s" % detail_path)
        except OSError as e:
            log("detail record not written: %r" % (e,))
            detail_path = None
        if headline:
            workload = ("%s: %d file(s) of %dM x %d bp reads (%.2f GB, page cache), k=%d, %s panel (%d patterns, "
                        "%d keys), f_snp=%g; %d rank(s), byte ranges of each file" % (
                            args.config.upper(), n_files, R // n_files // 1_000_000, L, e2e["file_bytes"] / 1e9, k,
                            panel_name, n_pat, tinfo["n_keys"], args.f_snp, world))
            parallelism = "dp%d (byte ranges per rank, RCCL all-reduce of u32 counts + u64 tally)" % world
        else:
            workload = ("%s: %s x %d bp reads%s, k=%d, %s panel (%d patterns, %d keys), HBM-resident"
                        % (args.config.upper(), "%gM" % (reads_total / 1e6) if strong_kernel else
                           "%dM" % (R // 1_000_000), L, " over the GPUs" if strong_kernel else " per GPU",
                           k, panel_name, n_pat, tinfo["n_keys"]))
            parallelism = "dp%d (reads per rank, RCCL all-reduce of u32 counts + u64 tally)" % world
        line = assemble_line({
            "L": L, "k": k, "world": world, "steps": args.steps, "warmup": args.warmup, "config": args.config,
            "e2e": e2e, "cli": cli, "cpu": cpu, "k_value": k_value, "k_elapsed": k_elapsed, "k_steps": k_steps,
            "k_kmer_rate": k_kmer_rate, "k_ms": k_ms, "achieved": achieved, "traffic": traffic,
            "alg_bytes": alg_bytes, "panel_src": "SNP_GRCh38_hg38_wChr.bed" if panel_name == "grch38" else
            "200k-row synthetic", "workload": workload, "R": R, "reads_total": reads_total, "n_pat": n_pat,
            "n_files": n_files, "parallelism": parallelism,
            "limiter": LIMITER_LARGE_PANEL if tinfo["n_keys"] > 65536 else LIMITER_FLANK,
            "build_id": vafc.tree_build_id(), "detail_path": detail_path, "parity": parity,
            "full_parity": full_parity})
        text = json.dumps(line)
        if len(text) > LINE_BYTES_MAX:
            log("the line is %d bytes (bound %d)" % (len(text), LINE_BYTES_MAX))
        os.write(out_fd, (text + "\n").encode())
    kmap.close()
    shutil.rmtree(tmp, ignore_errors=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
