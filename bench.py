#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X vaf-counter hot path.

Metric (BASELINE.json): Mbases/sec (+ k-mers/sec) on 150 bp FASTQ, k=21.
Workload (configs[1], "C2"): per GPU 100M synthetic 150 bp reads against the
SNP_GRCh38_hg38_wChr panel (20,849 ACGT patterns), generated on the device by
the same counter-based generator as kmer-cnt_amd/vafc_synth.py, resident in
HBM before the timed region.  --config c3 (k = 31, 100M pairs), c5 (200k-SNP
panel) and c4 (1B reads in total, split over the ranks: strong scaling) are
the other BASELINE.json configs.

One step = one pass of the hot path over the whole batch: zero the counts,
decode + extract + filter + probe + count every read (vc_count_device), and --
with N > 1 -- the RCCL all-reduce of the uint32 count vector and the k-mer
tally (torch.distributed "nccl" backend), all enqueued on one stream with no
host synchronisation inside the step.  `value` is kernel-side throughput on
HBM-resident reads; it excludes FASTQ parsing and PCIe.

Also reported:
  roofline      the counting kernels' algorithmic bytes (1 B/base
                + 8 B/read; the layout's 12 B/read beside it) / their event-timed duration,
                against 8 TB/s HBM3E; traffic from a committed rocprofv3 PMC
                summary of this workload (profiles/pmc_summary.json) if present.
  cpu_baseline  the REAL reference vaf-counter (oracle/_ref, compiled from the
                reference sources) on a bounded sample of the same reads written
                as FASTQ, timed by its own -v "Speed" line; median of 3 at
                -t 1 / 4 / 16 / nproc, the best median.
  parity        the product's .vaf on that sample vs the reference's (md5).
  e2e           the metric as the reference defines it (bases / counting-phase
                wall clock, vaf-counter.c:646-651,707): the drop-in CLI on a
                page-cached 16M-read FASTQ written on the box, plain and
                gzip level 1, parse + PCIe + kernels + reduce included; the
                reference on the same file for .vaf parity.
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
                 "HBM requests are 1.47x the algorithmic bytes (the waves' live read lines, 4.9 MB per XCD, "
                 "overflow its 4 MB L2 and are fetched again), not the limit; DESIGN.md sections 3.1.1-3.1.2, "
                 "profiles/r04j_final_c2_pmc_counters.json, profiles/r04c_ablation_time.log")
LIMITER_LARGE_PANEL = ("the roofline is HBM (integer byte work, no MFMA); the large-panel kernel runs far below "
                       "it, bound by VALU issue and the texture-address (TA) rate of its gathers: 9.3 % of "
                       "windows pass the 144 KiB LDS Bloom filter (about 6 % is that size's information limit "
                       "for 200k SNP pairs), each pass is a hit-loop trip and one lane of a random gather into "
                       "the L2-resident second-level filter; 23.6 VALU per base (5.5 G per launch, ~0.8 of the "
                       "kernel time at ~4 cycles each), TA busy ~0.5 of the cycles (3.66 G over 256 CUs); "
                       "DESIGN.md section 3.1 (large panels), profiles/r04j_final_c5_pmc_counters.json")


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


def e2e_leg(d_seq, L, k, pat, tmp, n_reads, cpu, devices=None, dev=None, device_vaf=None, kernel_s=None):
    """The drop-in CLI end to end on a page-cached FASTQ of the first n_reads
    HBM reads (plain, gzip), median of 3 runs each.

    device_vaf: md5 of the .vaf that count_device gives on the same HBM reads
    -- the CLI's .vaf on the file must equal it (a full-size bit-exact check;
    the reference itself is checked on the 2M-read sample).  kernel_s: the
    counting kernels' time for these reads (for the roofline split).
    devices: several GPUs in the one CLI process (VAFC_DEVICES,
    vc_create_multi: pieces dealt round robin, one RCCL reduce)."""
    import vafc
    t = cpu_share(len(devices) if devices else 1)
    est = n_reads * (2 * L + 16)
    work = scratch_dir(est * 1.25, tmp)
    fq = os.path.join(work, "e2e.fq")
    gz = fq + ".gz"
    t0 = time.time()
    write_fastq_from_device(d_seq, n_reads, L, fq, threads=t)
    fq_bytes = os.path.getsize(fq)
    log("e2e: %d reads as FASTQ (%.2f GB) in %s in %.1fs" % (n_reads, fq_bytes / 1e9, work, time.time() - t0))
    t0 = time.time()
    gz_bytes = gzip_level1(fq, gz, t)
    log("e2e: gzip level 1 (%.2f GB) in %.1fs" % (gz_bytes / 1e9, time.time() - t0))
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
    n_runs = int(os.environ.get("VAFC_E2E_RUNS", "5"))
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
            log("e2e %s -t %d (run %d): %.1f Mbases/s counting phase, %.2fs process" %
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
        log("e2e roofline failed: %r" % (e,))
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
    for f in (fq, gz):
        os.unlink(f)
    if work != tmp:
        shutil.rmtree(work, ignore_errors=True)
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=None, help="reads per GPU (c4: in total)")
    ap.add_argument("--read-len", type=int, default=150)
    ap.add_argument("--k", type=int, default=21)
    ap.add_argument("--f-snp", type=float, default=0.01)
    ap.add_argument("--panel", default="grch38", choices=["grch38", "syn200k"])
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"],
                    help="BASELINE.json configs: c2 (default, the headline: k=21, 100M reads per GPU), "
                         "c3 (k=31, 100M pairs = 200M reads of 150 bp), c4 (1B reads in total split over "
                         "the GPUs: strong scaling), c5 (200k-SNP synthetic panel)")
    ap.add_argument("--cpu-reads", type=int, default=2_000_000, help="CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline timings (the parity sample still runs)")
    ap.add_argument("--no-parity", action="store_true", help="skip the live parity sample too")
    ap.add_argument("--e2e-reads", type=int, default=None,
                    help="reads of the end-to-end FASTQ (default: all of the workload's reads on rank 0)")
    ap.add_argument("--no-e2e", action="store_true")
    args = ap.parse_args()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    strong = args.config == "c4"
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

    import torch
    import torch.distributed as dist
    # one GPU per rank; the modulo only matters for rehearsals with more ranks
    # than GPUs (VAFC_DIST_BACKEND=gloo), never for the driver's N-GPU runs
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # Every torch op and every vafc launch of this process run on torch's
    # default stream: its handle 0 is HIP's null stream, which vc_count_device
    # takes as such (include/vafc.h; the round-3 ABI read 0 as the counter's
    # own stream, and a zero-fill on torch's default stream raced with the
    # count, profiles/r03_rank1_parity_race.log).
    if world > 1:
        backend = os.environ.get("VAFC_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        # host-side group for waiting while rank 0 runs the e2e leg on every
        # GPU (a gloo barrier does not keep an RCCL kernel spinning on them)
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
    kmap = vafc.create_combined_kmer_map(db, args.k, device=local)
    tinfo = kmap.table_info()
    n_pat = db.n

    # ---- synthetic reads, resident in HBM (rank r: reads r*R0 .. of the stream)
    L = args.read_len
    if strong:
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

    counts = torch.zeros(2 * n_pat, dtype=torch.int32, device=dev)
    tally = torch.zeros(1, dtype=torch.int64, device=dev)
    kmap.bind_outputs(counts.data_ptr(), tally.data_ptr())
    kmap.set_timing(True)
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        # everything on torch's current stream: zero, count, then the RCCL
        # all-reduces (their stream waits on this one) -- no host sync
        counts.zero_()
        tally.zero_()
        kmap.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr(), d_lens.data_ptr(), R, stream)
        if world > 1:
            w = [dist.all_reduce(counts, async_op=True), dist.all_reduce(tally, async_op=True)]
            for x in w:
                x.wait()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kernel_ms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        kernel_ms.append(kmap.kernel_ms())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    reads_total = R
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        n = torch.tensor([R], dtype=torch.int64, device=dev)
        dist.all_reduce(n)
        reads_total = int(n.item())

    kmers_total = int(tally.item())           # after the all-reduce: all ranks' k-mers
    bases_total = reads_total * L
    ms_step = elapsed / args.steps * 1e3
    value = bases_total * args.steps / elapsed / 1e6
    kmer_rate = kmers_total * args.steps / elapsed

    # ---- roofline of the counting kernels (this rank's launch).  Algorithmic
    # bytes as SURVEY.md section 8(d) defines them: 1 B per base + 8 B per read
    # (one u64 offset, or a u32 offset + length).  The kernel's input layout
    # reads 12 B per read (u64 offset + u32 length); that figure is reported
    # beside it (layout_bytes_per_launch, frac_layout).
    k_ms = float(np.mean(kernel_ms))
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
    e2e = None
    n = min(args.cpu_reads, R)
    if not args.no_parity and n > 0:
        if first == 0:
            p_seq, p_offs, p_lens = d_seq, d_offs, d_lens
        else:   # rank r > 0: regenerate reads 0 .. n-1 of the stream
            p_seq = torch.empty(n * L, dtype=torch.uint8, device=dev)
            p_offs = torch.empty(n, dtype=torch.int64, device=dev)
            p_lens = torch.empty(n, dtype=torch.int32, device=dev)
            vafc.synth_reads(p_seq.data_ptr(), p_offs.data_ptr(), p_lens.data_ptr(), 0, n, L,
                             S.READ_SEED_R1, args.f_snp, win.data_ptr(), dos.data_ptr(), panel.n,
                             torch.cuda.current_stream().cuda_stream)
        par_counts = torch.zeros(2 * n_pat, dtype=torch.int32, device=dev)
        par_tally = torch.zeros(1, dtype=torch.int64, device=dev)
        kmap.bind_outputs(par_counts.data_ptr(), par_tally.data_ptr())
        kmap.set_timing(False)
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
    if rank == 0 and not args.no_e2e and args.config == "c2":
        # the reference's own metric on this workload's reads (all R of rank 0's
        # reads by default); N > 1: one CLI process over all N GPUs (the other
        # ranks wait at the barrier below)
        try:
            ne = min(args.e2e_reads or R, R)
            kmap.set_timing(True)
            kmap.reset()
            kmap.count_device(d_seq.data_ptr(), ne * L, d_offs.data_ptr(), d_lens.data_ptr(), ne)
            ec, _ = kmap.finish()
            e_ks = kmap.kernel_ms() * 1e-3
            dev_vaf = os.path.join(tmp, "device_e2e.vaf")
            db.write_vaf(ec, dev_vaf)
            e2e = e2e_leg(d_seq, L, args.k, pat, tmp, ne, cpu,
                          devices=[r % max(torch.cuda.device_count(), 1) for r in range(world)] if world > 1
                          else None, dev=dev, device_vaf=md5(dev_vaf), kernel_s=e_ks / world)
        except Exception as e:
            log("e2e leg failed: %r" % (e,))
    if world > 1:
        dist.barrier(group=cpu_group)

    if rank == 0:
        line = {
            "metric": "Mbases/sec (+ k-mers/sec) on %d bp FASTQ, k=%d" % (L, args.k),
            "value": round(value, 1),
            "unit": "Mbases/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (counter-based generator, seed 42; patterns from %s, flanks seed 12345), "
                    "resident in HBM: value is kernel-side throughput (no FASTQ parse, no PCIe); the "
                    "reference's end-to-end metric is the e2e object" % (
                        "SNP_GRCh38_hg38_wChr.bed" if args.panel == "grch38" else "a 200k-row synthetic BED"),
            "config": {
                "workload": "%s: %s x %d bp reads%s, k=%d, %s panel (%d patterns, %d keys), f_snp=%g"
                            % (args.config.upper(), "%gM" % (reads_total / 1e6) if strong else "%dM" % (R // 1_000_000),
                               L, " in total over the GPUs" if strong else " per GPU", args.k, args.panel, n_pat,
                               tinfo["n_keys"], args.f_snp),
                "reads_per_gpu": R, "reads_total": reads_total, "read_len": L, "k": args.k, "patterns": n_pat,
                "filter_bytes": tinfo["filter_bytes"], "table_slots": tinfo["slots"],
                "parallelism": "dp%d (reads sharded per rank, RCCL all-reduce of uint32 counts + u64 tally)" % world,
            },
            "kmers_per_sec": round(kmer_rate, 1),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "vc_count_reads_kernel (+ vc_count_long_kernel, empty here)",
                "limiter": (LIMITER_LARGE_PANEL if tinfo["n_keys"] > 65536 else LIMITER_FLANK),
                "kernel_ms": round(k_ms, 4),
                "alg_bytes_per_launch": alg_bytes,
                "alg_bytes_rule": "SURVEY.md 8(d): 1 B/base + 8 B/read",
                "layout_bytes_per_launch": layout_bytes,
                "frac_layout": round(layout_bytes / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            },
            "cpu_baseline": cpu,
            "parity_vs_reference_on_sample": parity,
            "parity_note": ("the product's .vaf on the first %d reads == the reference's (md5)" % n if world == 1 else
                            "all %d ranks count the first %d reads of the stream, %s all-reduce; == %d x the "
                            "reference's counts on that sample (u32)"
                            % (world, n, "RCCL" if os.environ.get("VAFC_DIST_BACKEND", "nccl") == "nccl" else
                               os.environ.get("VAFC_DIST_BACKEND"), world)),
            "build_id": vafc.tree_build_id(),
            "e2e": e2e,
        }
        print(json.dumps(line), flush=True)
    kmap.close()
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
