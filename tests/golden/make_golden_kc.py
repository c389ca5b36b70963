#!/usr/bin/env python3
"""Golden fixtures for kc-c4 from the REAL reference
binary oracle/_ref/kc-c4 (compiled by `make -C oracle` from
/root/reference/kc-c4.c with its Makefile:28-29 flags).  Run in the build
container:

    python tests/golden/make_golden_kc.py

Writes tests/golden/kc/: small inputs (FASTQ from a short repetitive genome so
counts span 1..255 and beyond, poly-A runs past the 10-bit saturation, N and
IUPAC bytes, lower case, raw code bytes 0..3, CRLF, multi-line FASTA with
records longer than the device's one-lane limit, reads shorter than k, gzip,
an empty file, truncated qualities that end blocks early) and manifest.json:
per case the argv, exit code, md5 of stdout and the non-zero histogram rows.
"""
import gzip
import hashlib
import json
import os
import shutil
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "kc")
REF = os.path.join(ROOT, "oracle", "_ref", "kc-c4")

COMP = bytes.maketrans(b"ACGTacgt", b"TGCAtgca")


def rc(s: bytes) -> bytes:
    return s.translate(COMP)[::-1]


def fastq(reads, nl=b"\n"):
    out = []
    for i, r in enumerate(reads):
        out.append(b"@r%d%s%s%s+%s%s%s" % (i, nl, r, nl, nl, b"I" * len(r), nl))
    return b"".join(out)


def fasta(recs, width=60, nl=b"\n"):
    out = []
    for i, r in enumerate(recs):
        out.append(b">s%d desc%s" % (i, nl))
        for j in range(0, len(r), width):
            out.append(r[j:j + width] + nl)
        if not r:
            out.append(nl)
    return b"".join(out)


def sample_reads(rng, genome: bytes, n, L):
    reads = []
    for _ in range(n):
        s = int(rng.integers(0, len(genome) - L + 1))
        r = bytearray(genome[s:s + L])
        if rng.random() < 0.5:
            r = bytearray(rc(bytes(r)))
        for j in range(L):   # 1 % substitutions
            if rng.random() < 0.01:
                r[j] = b"ACGT"[int(rng.integers(0, 4))]
        reads.append(bytes(r))
    return reads


def make_inputs(rng):
    acgt = np.frombuffer(b"ACGT", np.uint8)
    g = acgt[rng.integers(0, 4, 3000)].tobytes()
    files = {}
    # coverage ~150x over a 3 kb genome: counts up to a few hundred
    files["cov.fq"] = fastq(sample_reads(rng, g, 3000, 150))
    # poly-A/poly-C runs beyond 1023 occurrences, plus N/IUPAC/lower case/raw codes
    weird = []
    weird.append(b"A" * 1500)
    weird.append(b"C" * 700 + b"N" + b"G" * 700)
    weird.append(bytes(g[:200]).lower() + b"NNNN" + g[200:400])
    weird.append(g[400:500] + b"RYSWKM" + g[500:600] + b"U" * 40 + b"u" * 30)
    weird.append(bytes([0, 1, 2, 3] * 30) + g[600:700])
    weird.append(g[700:710])           # shorter than most k
    weird.append(b"")                  # empty record
    weird.append(g[710:1000] + b"." + g[1000:1200] + b"-" + g[1200:1300])
    files["weird.fa"] = fasta(weird)
    # CRLF FASTQ
    files["crlf.fq"] = fastq(sample_reads(rng, g, 200, 120), nl=b"\r\n")
    # long multi-line FASTA records (device segments long reads)
    long_recs = [acgt[rng.integers(0, 4, 20000)].tobytes(), g * 4,
                 acgt[rng.integers(0, 4, 5000)].tobytes() + b"N" * 10 + g[:5000],
                 acgt[rng.integers(0, 4, 4097)].tobytes(), acgt[rng.integers(0, 4, 4096)].tobytes()]
    files["long.fa"] = fasta(long_recs, width=70)
    # gzip of the coverage set
    files["cov.fq.gz"] = gzip.compress(files["cov.fq"], 6)
    # an empty file
    files["empty.fq"] = b""
    # FASTQ with truncated qualities: kseq_read returns -2 and the block ends
    rs = sample_reads(rng, g, 60, 100)
    parts = []
    for i, r in enumerate(rs):
        q = b"I" * (len(r) if i % 7 else len(r) // 2)
        if i % 7 == 0 and i:
            parts.append(b"@t%d\n%s\n+\n%s\n@u%d\n" % (i, r, q, i))  # short qual, then header
        else:
            parts.append(b"@t%d\n%s\n+\n%s\n" % (i, r, q))
    files["badqual.fq"] = b"".join(parts)
    # mixed lengths 1..300
    mixed = [acgt[rng.integers(0, 4, int(rng.integers(1, 301)))].tobytes() for _ in range(400)]
    files["mixed.fq"] = fastq(mixed)
    return files


CASES = [
    ("cov_k21", ["-k", "21"], "cov.fq"),
    ("cov_k31", [], "cov.fq"),
    ("cov_k11", ["-k", "11"], "cov.fq"),
    ("cov_k5", ["-k", "5"], "cov.fq"),
    ("cov_k1", ["-k", "1"], "cov.fq"),
    ("cov_k16_p12", ["-k", "16", "-p", "12"], "cov.fq"),
    ("cov_gz_k21", ["-k", "21"], "cov.fq.gz"),
    ("cov_b1_k21", ["-k", "21", "-b", "1"], "cov.fq"),
    ("weird_k21", ["-k", "21"], "weird.fa"),
    ("weird_k5", ["-k", "5"], "weird.fa"),
    ("weird_k31", [], "weird.fa"),
    ("crlf_k21", ["-k", "21"], "crlf.fq"),
    ("long_k21", ["-k", "21"], "long.fa"),
    ("long_k31_b5000", ["-b", "5000"], "long.fa"),
    ("empty_k21", ["-k", "21"], "empty.fq"),
    ("badqual_k21", ["-k", "21"], "badqual.fq"),
    ("badqual_b1_k21", ["-k", "21", "-b", "1"], "badqual.fq"),
    ("mixed_k25", ["-k", "25"], "mixed.fq"),
    ("mixed_k7_t1", ["-k", "7", "-t", "1"], "mixed.fq"),
    ("usage", [], None),
    ("p_too_small", ["-p", "8"], "cov.fq"),
]


def main():
    if not os.path.exists(REF):
        raise SystemExit("build the reference first: make -C oracle")
    if os.path.isdir(OUT):
        shutil.rmtree(OUT)
    os.makedirs(OUT)
    rng = np.random.default_rng(2024)
    for name, data in make_inputs(rng).items():
        with open(os.path.join(OUT, name), "wb") as f:
            f.write(data)
    manifest = []
    for name, opts, inp in CASES:
        argv = list(opts) + ([inp] if inp else [])
        p = subprocess.run([REF] + argv, cwd=OUT, capture_output=True)
        hist = {}
        for line in p.stdout.decode().splitlines():
            i, c = line.split("\t")
            if int(c):
                hist[i] = int(c)
        manifest.append({"name": name, "argv": argv, "rc": p.returncode,
                         "stdout_md5": hashlib.md5(p.stdout).hexdigest(),
                         "stdout_lines": len(p.stdout.decode().splitlines()),
                         "stderr": p.stderr.decode(), "hist": hist})
        print(name, p.returncode, len(hist))
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
