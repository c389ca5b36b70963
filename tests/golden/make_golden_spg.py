#!/usr/bin/env python3
"""Golden fixtures for snp-pattern-gen from the REAL
reference binary oracle/_ref/snp-pattern-gen (compiled by `make -C oracle`
from /root/reference/snp-pattern-gen.c).  Run in the build container:

    python tests/golden/make_golden_spg.py

Writes tests/golden/spg/: small genomes (FASTA, multi-line, CRLF, gzip,
soft-masked, N runs, IUPAC codes, repeated and reverse-complemented segments,
planted alt k-mers, a duplicated chromosome name), BED files (edge positions,
missing chromosomes, non-ACGT alleles, duplicate rows, a row with an extra
column), and manifest.json: per case the argv, exit code, stderr text and the
md5 of the output pattern file.
"""
import gzip
import hashlib
import json
import os
import shutil
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "spg")
REF = os.path.join(ROOT, "oracle", "_ref", "snp-pattern-gen")

COMP = bytes.maketrans(b"ACGTacgt", b"TGCAtgca")


def rc(s: bytes) -> bytes:
    return s.translate(COMP)[::-1]


def wrap(seq: bytes, width: int, nl: bytes = b"\n") -> bytes:
    return nl.join(seq[i:i + width] for i in range(0, len(seq), width)) + nl


def make_genome(rng):
    """dict name -> bytearray, plus the list of (chrom, pos) SNP sites."""
    acgt = np.frombuffer(b"ACGT", np.uint8)
    chroms = {}
    for name, L in (("chr1", 12000), ("chr2", 30000), ("chrX", 8000), ("chrM", 500)):
        chroms[name] = bytearray(acgt[rng.integers(0, 4, L)].tobytes())
    c1, c2, cx = chroms["chr1"], chroms["chr2"], chroms["chrX"]
    # repeats: a forward copy and a reverse-complement copy (ref k-mers there occur twice)
    c2[5000:5300] = c1[1000:1300]
    cx[100:300] = rc(bytes(c1[2000:2200]))
    c2[20000:20400] = c2[10000:10400]            # intra-chromosome repeat
    # soft-masking, N runs, IUPAC codes
    cx[3000:4500] = bytes(cx[3000:4500]).lower()
    c1[7000:7100] = b"N" * 100
    c2[15000:15030] = b"n" * 30
    for pos, ch in ((8100, b"S"), (8200, b"W"), (8300, b"D"), (8400, b"R"), (8500, b"Y"), (8600, b"M")):
        c1[pos:pos + 1] = ch
    return chroms


def snp_rows(chroms, rng):
    rows = []
    names = ["chr1", "chr2", "chrX", "chrM"]
    for i in range(400):
        ch = names[int(rng.integers(0, 4))]
        L = len(chroms[ch])
        pos = int(rng.integers(0, L))
        ref = chr(chroms[ch][pos]).upper()
        alt = "ACGT"[(("ACGT".find(ref) if ref in "ACGT" else 0) + int(rng.integers(1, 4))) % 4]
        rows.append((ch, pos, ref, alt))
    # repeats (ref k-mer not unique), N/IUPAC neighbourhoods, edges
    for pos in (1100, 1150, 2100, 7095, 7150, 8100, 8205, 8300, 10100):
        rows.append(("chr1", pos, "A", "G"))
    for pos in (5100, 10200, 20200, 15010, 0, 3, 10, 29989, 29990, 29999):
        rows.append(("chr2", pos, "C", "T"))
    for pos in (150, 3500, 4499, 7990):
        rows.append(("chrX", pos, "G", "A"))
    rows.append(("chrZ", 100, "A", "C"))        # missing chromosome
    rows.append(("chr1", 500, "A", "N"))        # non-ACGT alt
    rows.append(("chr1", 600, "A", "a"))        # lowercase alt
    rows.append(("chr1", 700, "A", "U"))        # U encodes like T
    rows.append(("chr1", 900, "A", "G"))
    rows.append(("chr1", 900, "A", "G"))        # duplicate row
    return rows


def plant_alts(chroms, rows, k_values):
    """Copy the alt k-mer of some SNPs elsewhere (alt present -> SNP dropped)."""
    c2 = chroms["chr2"]
    at = 25000
    for ch, pos, ref, alt in rows[:40:4]:
        for k in k_values:
            f = k // 2
            s = pos - f
            if s < 0 or s + k > len(chroms[ch]) or alt not in "ACGT":
                continue
            w = bytearray(chroms[ch][s:s + k])
            w[f:f + 1] = alt.encode()
            if at + k < 29900:
                c2[at:at + k] = bytes(w) if (at // 7) % 2 else rc(bytes(w))
                at += k + 3


def write_bed(path, rows, extra_col_at=None):
    with open(path, "w") as f:
        for i, (ch, pos, ref, alt) in enumerate(rows):
            extra = "\tEXTRA" if i == extra_col_at else ""
            f.write("%s\t%d\t%d\trs%d\t%s\t%s%s\n" % (ch, pos, pos + 1, 1000 + i, ref, alt, extra))


def main():
    assert os.path.exists(REF), "build the reference first: make -C oracle"
    if os.path.isdir(OUT):
        shutil.rmtree(OUT)
    os.makedirs(OUT)
    rng = np.random.default_rng(2024)
    chroms = make_genome(rng)
    rows = snp_rows(chroms, rng)
    plant_alts(chroms, rows, (5, 11, 21, 31))
    # genome files
    with open(os.path.join(OUT, "g1.fa"), "wb") as f:
        for name in ("chr1", "chr2", "chrX", "chrM"):
            hdr = b">" + name.encode() + (b" assembled test chromosome" if name == "chr2" else b"")
            f.write(hdr + b"\n" + wrap(bytes(chroms[name]), 60 if name != "chrX" else 80))
        f.write(b">chr2 duplicate name, never used\n" + wrap(b"ACGT" * 50, 60))
    with open(os.path.join(OUT, "g1.fa"), "rb") as f:
        data = f.read()
    with gzip.open(os.path.join(OUT, "g1.fa.gz"), "wb", compresslevel=6) as f:
        f.write(data)
    with open(os.path.join(OUT, "g2_crlf.fa"), "wb") as f:       # CRLF, blank lines, empty record
        f.write(b">empty\r\n")
        f.write(b">chr1\r\n" + wrap(bytes(chroms["chr1"][:6000]), 70, b"\r\n") + b"\r\n")
        f.write(b">chrM\r\n" + wrap(bytes(chroms["chrM"]), 50, b"\r\n"))
    with open(os.path.join(OUT, "g3_oneline.fa"), "wb") as f:     # unwrapped sequences
        for name in ("chrX", "chr1"):
            f.write(b">" + name.encode() + b"\n" + bytes(chroms[name]) + b"\n")
    write_bed(os.path.join(OUT, "snps.bed"), rows)
    write_bed(os.path.join(OUT, "snps_extra_col.bed"), rows[:60], extra_col_at=20)
    open(os.path.join(OUT, "empty.bed"), "w").close()

    cases = []

    def case(name, argv):
        d = tempfile.mkdtemp()
        for fn in os.listdir(OUT):
            if not fn.endswith(".json"):
                shutil.copy(os.path.join(OUT, fn), d)
        p = subprocess.run([REF] + argv, cwd=d, capture_output=True, text=True, timeout=300)
        out = os.path.join(d, "out.txt")
        entry = {"name": name, "argv": argv, "exit": p.returncode, "stderr": p.stderr,
                 "out_md5": hashlib.md5(open(out, "rb").read()).hexdigest() if os.path.exists(out) else None,
                 "out_lines": sum(1 for _ in open(out)) if os.path.exists(out) else None}
        cases.append(entry)
        shutil.rmtree(d)

    for k in (21, 31, 11, 9, 7, 5, 3, 1, 15, 25, 29):
        case("g1_k%d" % k, ["-k", str(k), "-b", "snps.bed", "-f", "g1.fa", "-o", "out.txt"])
    case("g1_default_k", ["-b", "snps.bed", "-f", "g1.fa", "-o", "out.txt"])
    case("g1_gz_k21", ["-k", "21", "-b", "snps.bed", "-f", "g1.fa.gz", "-o", "out.txt"])
    case("g2_crlf_k21", ["-k", "21", "-b", "snps.bed", "-f", "g2_crlf.fa", "-o", "out.txt"])
    case("g2_crlf_k11", ["-k", "11", "-b", "snps.bed", "-f", "g2_crlf.fa", "-o", "out.txt"])
    case("g3_oneline_k21", ["-k", "21", "-b", "snps.bed", "-f", "g3_oneline.fa", "-o", "out.txt"])
    case("extra_col_k21", ["-k", "21", "-b", "snps_extra_col.bed", "-f", "g1.fa", "-o", "out.txt"])
    case("empty_bed", ["-k", "21", "-b", "empty.bed", "-f", "g1.fa", "-o", "out.txt"])
    case("options_reordered", ["-o", "out.txt", "-f", "g1.fa", "-k", "13", "-b", "snps.bed"])
    case("even_k", ["-k", "20", "-b", "snps.bed", "-f", "g1.fa", "-o", "out.txt"])
    case("usage", ["-k", "21", "-b", "snps.bed"])
    case("missing_fasta", ["-k", "21", "-b", "snps.bed", "-f", "nope.fa", "-o", "out.txt"])
    case("missing_bed", ["-k", "21", "-b", "nope.bed", "-f", "g1.fa", "-o", "out.txt"])
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_spg.py", "reference": "oracle/_ref/snp-pattern-gen",
                   "cases": cases}, f, indent=1)
    for c in cases:
        print("%-20s exit %d lines %s" % (c["name"], c["exit"], c["out_lines"]))


if __name__ == "__main__":
    main()
