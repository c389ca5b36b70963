#!/usr/bin/env python3
"""Per-launch durations of one kernel from a rocprofv3 kernel trace (tools
only): the average over every call (what --stats reports, warm-up launches
included) and over the last STEPS calls (the bench's timed launches, what
its HIP-event kernel_ms measures).
    python tools/trace_avg.py p_kernel_trace.csv vc_count_reads_kernel 10 [MIN_GRID] > out.json
MIN_GRID (optional): only launches whose Grid_Size (threads) is at least
that -- in the default bench command, the kernel leg's launches over 100M
HBM-resident reads (256 blocks) apart from the e2e passes' per-piece ones."""
import csv
import json
import sys


def main():
    path, name, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    min_grid = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]
            and int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0) >= min_grid]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    out = {"trace": path, "kernel": rows[0]["Kernel_Name"] if rows else name, "calls": len(d),
           "durations_ms": [round(x, 4) for x in d],
           "avg_all_ms": round(sum(d) / len(d), 4) if d else None,
           "min_grid": min_grid,
           "timed_steps": steps,
           "avg_timed_ms": round(sum(d[-steps:]) / min(steps, len(d)), 4) if d else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
