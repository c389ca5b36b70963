#!/usr/bin/env python3
"""Collect rocprofv3 PMC counters for the counting kernel, one pass per group.

Run on the GPU box:  python tools/pmc.py OUTDIR [bench args...]
Each pass is a separate `rocprofv3 --kernel-trace --pmc ... -- python3 bench.py`
(no sys/runtime tracing with --pmc).  Writes OUTDIR/pmc_counters.json with the
per-dispatch average of each counter for vc_count_reads_kernel, plus derived
numbers (HBM bytes per launch with gfx950's FETCH_SIZE x2 correction).
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES",
    "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT",
    "SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE",
    "FETCH_SIZE",
    "WRITE_SIZE",
    "TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum",
    "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum",
]
# diagnosis passes (python tools/pmc.py OUTDIR --set diag [bench args...])
DIAG = [
    "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_ANY",
    "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY",
    "SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL",
    "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM",
    "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES",
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU",
]
KERNEL = "vc_count_reads_kernel"


def main():
    out = os.path.abspath(sys.argv[1])
    rest = sys.argv[2:]
    passes = PASSES
    if rest[:2] == ["--set", "diag"]:
        passes, rest = DIAG, rest[2:]
    elif rest[:2] == ["--set", "insts"]:      # instruction mix only (one pass)
        passes, rest = PASSES[:1], rest[2:]
    bench_args = rest or ["--steps", "2", "--warmup", "1", "--no-cpu"]
    os.makedirs(out, exist_ok=True)
    acc = {}
    for i, group in enumerate(passes):
        d = os.path.join(out, "pass%d" % i)
        cmd = ["rocprofv3", "--kernel-trace", "--pmc"] + group.split() + [
            "-d", d, "-o", "p", "--output-format", "csv", "--",
            "python3", os.path.join(ROOT, "bench.py")] + bench_args
        r = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True, timeout=900)
        with open(os.path.join(out, "pass%d.log" % i), "w") as f:
            f.write(r.stdout[-20000:] + "\n---\n" + r.stderr[-20000:])
        if r.returncode != 0:
            print("pass %d failed (rc %d)" % (i, r.returncode), flush=True)
            continue
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        vals = {}
        for fn in files:
            with open(fn) as f:
                for row in csv.DictReader(f):
                    if KERNEL not in row.get("Kernel_Name", ""):
                        continue
                    key = (row["Counter_Name"])
                    vals.setdefault(key, {}).setdefault(row.get("Dispatch_Id", "0"), 0.0)
                    vals[key][row.get("Dispatch_Id", "0")] += float(row["Counter_Value"])
        for name, per in vals.items():
            acc[name] = sum(per.values()) / max(len(per), 1)
        print("pass %d ok: %s" % (i, ", ".join("%s=%.4g" % (n, acc[n]) for n in group.split() if n in acc)),
              flush=True)
    derived = {}
    if "FETCH_SIZE" in acc:
        derived["hbm_read_bytes_per_launch"] = acc["FETCH_SIZE"] * 1024 * 2   # gfx950: FETCH_SIZE reads 1/2
    if "WRITE_SIZE" in acc:
        derived["hbm_write_bytes_per_launch"] = acc["WRITE_SIZE"] * 1024
    if derived:
        derived["hbm_bytes_per_launch"] = sum(derived.values())
    with open(os.path.join(out, "pmc_counters.json"), "w") as f:
        json.dump({"kernel": KERNEL, "bench_args": bench_args, "counters": acc, "derived": derived}, f, indent=1)
    # the summary bench.py reads for roofline.traffic (same workload only)
    if "hbm_bytes_per_launch" in derived:
        cfg = bench_args[bench_args.index("--config") + 1] if "--config" in bench_args else "c2"
        summ = {"kernel": KERNEL, "config": cfg, "reads": _arg(bench_args, "--reads", 100_000_000),
                "read_len": _arg(bench_args, "--read-len", 150), "k": 31 if cfg == "c3" else _arg(bench_args, "--k", 21),
                "hbm_bytes_per_launch": derived["hbm_bytes_per_launch"],
                "hbm_read_bytes_per_launch": derived.get("hbm_read_bytes_per_launch"),
                "hbm_write_bytes_per_launch": derived.get("hbm_write_bytes_per_launch"),
                "fetch_size_kib_raw": acc.get("FETCH_SIZE"),
                "correction": "read bytes = FETCH_SIZE x 1024 x 2 (gfx950 tallies 128-B requests at 64 B)",
                "counters": acc}
        with open(os.path.join(out, "pmc_summary.json"), "w") as f:
            json.dump(summ, f, indent=1)
    print(json.dumps(derived))


def _arg(args, name, default):
    return int(args[args.index(name) + 1]) if name in args else default


if __name__ == "__main__":
    main()
