#!/usr/bin/env python3
"""Per-variant PMC counts of an ablation run (tools/gpu_run.sh abl): the
rocprofv3 counter CSV of `tools/ab.py --rounds 1 V1 V2 ...` lists the counting
kernel's dispatches round by round, variant by variant; this averages each
counter per variant.
    python tools/abl_pmc_summary.py gpurun_out/TAG_abl_pmc/p_counter_collection.csv "V1 V2 ..." > out.json
"""
import collections
import csv
import json
import sys


def main():
    path, variants = sys.argv[1], sys.argv[2].split()
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if "vc_count_reads_kernel" not in r["Kernel_Name"]:
            continue
        d = per.setdefault(int(r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = {v: collections.defaultdict(list) for v in variants}
    for i, (_, c) in enumerate(per.items()):
        for k, x in c.items():
            out[variants[i % len(variants)]][k].append(x)
    res = {v: {k: sum(x) / len(x) for k, x in sorted(d.items())} for v, d in out.items()}
    json.dump({"source": path, "dispatches": len(per), "per_variant_mean": res}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
