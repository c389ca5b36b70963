#!/usr/bin/env python3
"""Golden fixtures for yak-count from the REAL
reference binary oracle/_ref/yak-count (compiled by `make -C oracle` from
/root/reference/yak-count.c with its Makefile:31-32 flags).  Run in the build
container after make_golden_kc.py:

    python tests/golden/make_golden_yak.py

Inputs are the kc fixtures of tests/golden/kc/ plus two read sets written to
tests/golden/yak/ (r1.fq, r2.fq: different reads of one genome, so the
two-file Bloom-filter mode keeps k-mers by file 1's filter and counts them in
file 2).  Cases cover: no filter (default), a filter with one file, two
files, filters small enough for many false positives (one 512-bit block per
sub-table), a filter too small to be created (-b below -p + 9), -H 1/8/32,
-p 12, -K small, gzip, an empty file, k = 1/5/21/31.  manifest.json: per case
the argv, exit code, md5 of stdout, the last stderr line and the non-zero
histogram rows.
"""
import hashlib
import json
import os
import shutil
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "yak")
KC = os.path.join(HERE, "kc")
REF = os.path.join(ROOT, "oracle", "_ref", "yak-count")

COMP = bytes.maketrans(b"ACGTacgt", b"TGCAtgca")


def rc(s: bytes) -> bytes:
    return s.translate(COMP)[::-1]


def reads_fq(rng, g, n, L, tag):
    out = []
    for i in range(n):
        s = int(rng.integers(0, len(g) - L + 1))
        r = bytearray(g[s:s + L])
        if rng.random() < 0.5:
            r = bytearray(rc(bytes(r)))
        for j in range(L):
            if rng.random() < 0.01:
                r[j] = b"ACGT"[int(rng.integers(0, 4))]
        out.append(b"@%s%d\n%s\n+\n%s\n" % (tag, i, bytes(r), b"I" * L))
    return b"".join(out)


CASES = [
    ("nobf_k31", [], ["cov.fq"]),
    ("nobf_k21", ["-k", "21"], ["cov.fq"]),
    ("nobf_k1", ["-k", "1"], ["cov.fq"]),
    ("nobf_k5_weird", ["-k", "5"], ["weird.fa"]),
    ("nobf_k21_weird", ["-k", "21"], ["weird.fa"]),
    ("nobf_k21_long", ["-k", "21"], ["long.fa"]),
    ("nobf_gz", ["-k", "21"], ["cov.fq.gz"]),
    ("nobf_K1", ["-k", "21", "-K", "1"], ["badqual.fq"]),
    ("nobf_badqual", ["-k", "21"], ["badqual.fq"]),
    ("nobf_p12", ["-k", "21", "-p", "12"], ["cov.fq"]),
    ("nobf_two_files_ignored", ["-k", "21"], ["r1.fq", "r2.fq"]),
    ("bf24_one", ["-k", "21", "-b", "24"], ["cov.fq"]),
    ("bf24_two", ["-k", "21", "-b", "24"], ["r1.fq", "r2.fq"]),
    ("bf19_two_fp", ["-k", "21", "-b", "19"], ["r1.fq", "r2.fq"]),
    ("bf20_two_fp_H1", ["-k", "21", "-b", "20", "-H", "1"], ["r1.fq", "r2.fq"]),
    ("bf20_two_fp_H8", ["-k", "21", "-b", "20", "-H", "8"], ["r1.fq", "r2.fq"]),
    ("bf19_two_fp_H32", ["-k", "21", "-b", "19", "-H", "32"], ["r1.fq", "r2.fq"]),
    ("bf21_two_p12", ["-k", "21", "-b", "21", "-p", "12"], ["r1.fq", "r2.fq"]),
    ("bf19_two_k31", ["-b", "19"], ["r1.fq", "r2.fq"]),
    ("bf19_two_k5", ["-k", "5", "-b", "19"], ["r1.fq", "r2.fq"]),
    ("bf19_two_K1000", ["-k", "21", "-b", "19", "-K", "1000"], ["r1.fq", "r2.fq"]),
    ("bf14_too_small", ["-k", "21", "-b", "14"], ["r1.fq", "r2.fq"]),
    ("bf20_H0", ["-k", "21", "-b", "20", "-H", "0"], ["r1.fq", "r2.fq"]),
    ("bf19_reversed", ["-k", "21", "-b", "19"], ["r2.fq", "r1.fq"]),
    ("bf22_weird", ["-k", "15", "-b", "22"], ["weird.fa", "long.fa"]),
    ("bf22_empty2", ["-k", "21", "-b", "22"], ["r1.fq", "empty.fq"]),
    ("nobf_empty", ["-k", "21"], ["empty.fq"]),
    ("usage", [], []),
    ("p_too_small", ["-p", "9"], ["cov.fq"]),
]


def main():
    if not os.path.exists(REF):
        raise SystemExit("build the reference first: make -C oracle")
    if os.path.isdir(OUT):
        shutil.rmtree(OUT)
    os.makedirs(OUT)
    rng = np.random.default_rng(77)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    g = acgt[rng.integers(0, 4, 20000)].tobytes()
    with open(os.path.join(OUT, "r1.fq"), "wb") as f:
        f.write(reads_fq(rng, g, 1500, 150, b"a"))
    with open(os.path.join(OUT, "r2.fq"), "wb") as f:
        f.write(reads_fq(rng, g, 1500, 150, b"b"))
    manifest = []
    for name, opts, inputs in CASES:
        argv = list(opts) + [os.path.join("..", "kc", x) if not x.startswith("r") else x for x in inputs]
        p = subprocess.run([REF] + argv, cwd=OUT, capture_output=True)
        hist = {}
        for line in p.stdout.decode().splitlines():
            i, c = line.split("\t")
            if int(c):
                hist[i] = int(c)
        err = p.stderr.decode().splitlines()
        manifest.append({"name": name, "argv": argv, "rc": p.returncode,
                         "stdout_md5": hashlib.md5(p.stdout).hexdigest(),
                         "stdout_lines": len(p.stdout.decode().splitlines()),
                         "stderr_last": err[-1] if err else "",
                         "stderr": p.stderr.decode() if p.returncode else None, "hist": hist})
        print(name, p.returncode, len(hist), err[-1] if err else "")
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
