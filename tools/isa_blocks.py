#!/usr/bin/env python3
"""Per-basic-block instruction counts of one kernel in a hipcc -S listing
(tools only): python tools/isa_blocks.py file.s KERNEL_SUBSTRING [top N]."""
import re
import sys


def blocks(path, name):
    txt = open(path).read().split("\n")
    start = next(i for i, l in enumerate(txt) if re.match(r"^_Z\w*%s\w*:" % name, l))
    out, cur, lab = [], [], "entry"
    for l in txt[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            out.append((lab, cur))
            cur, lab = [], m.group(1)
            continue
        t = l.strip().split()
        if t and not t[0].startswith((".", ";")):
            cur.append(t[0])
    out.append((lab, cur))
    return out


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    bl = blocks(path, name)
    tot = {}
    for _, ins in bl:
        for i in ins:
            tot[i] = tot.get(i, 0) + 1
    print("blocks %d, instructions %d, VALU %d" % (len(bl), sum(tot.values()),
                                                   sum(v for k, v in tot.items() if k.startswith("v_"))))
    for lab, ins in sorted(bl, key=lambda b: -len(b[1]))[:top]:
        v = sum(1 for i in ins if i.startswith("v_"))
        ds = sum(1 for i in ins if i.startswith("ds_"))
        gl = sum(1 for i in ins if i.startswith(("global_", "buffer_")))
        print("%-16s total %4d  VALU %4d  DS %3d  VMEM %3d" % (lab, len(ins), v, ds, gl))


if __name__ == "__main__":
    main()
