"""Synthetic workload for the vaf-counter hot path (SURVEY.md §8(d) "Synthetic inputs").

The container has no hg38 FASTA and there is no network, so the pattern set and
the reads are synthesised:

* **Patterns.** For each BED row (``chr start end rsid ref alt``, the format of
  ``SNP/*.bed``), random 150-base left/right flanks L, R are drawn from a
  counter-based RNG with seed 12345.  ``ref_kmer = L[-k//2:] + REF + R[:k-1-k//2]``
  and ``alt_kmer`` likewise with ALT -- the SNP sits at index ``k//2`` exactly as
  ``extract_snp_kmer`` places it (snp-pattern-gen.c:193-217).  Rows whose alleles
  are not single ACGT bases are dropped, as snp-pattern-gen would
  (snp-pattern-gen.c:280,340).  Each SNP also gets a genotype dosage g in {0,1,2}.
* **Reads.** ``read_len`` bp.  With probability ``f_snp`` a read is cut from a
  random SNP's 301-bp window ``L + allele + R`` (allele = ALT with probability
  g/2, start uniform in 0..151); otherwise it is uniform random background.  Then
  0.1% of bases become ``N``, 0.5% are substituted, and half of the reads are
  reverse-complemented.  FASTQ records are ``@r<i>``, quality all ``I``.

Every random draw is ``h64(seed, i, j)`` -- a splitmix64 finaliser of a linear
combination of (seed, item, draw index) -- so any read can be generated
independently of the others.  The HIP generator behind ``vc_synth_reads``
(``csrc/vafc_synth.hip``) evaluates the same function and produces the same
bytes; ``tests/test_gpu_parity.py`` checks that.
"""
from __future__ import annotations

import gzip
import os
from dataclasses import dataclass

import numpy as np

M64 = (1 << 64) - 1
G_SEED = np.uint64(0x9E3779B97F4A7C15)
G_ITEM = np.uint64(0xD1B54A32D192ED03)
G_DRAW = np.uint64(0xABC98388FB8FAC03)
MIX1 = np.uint64(0xBF58476D1CE4E5B9)
MIX2 = np.uint64(0x94D049BB133111EB)

PANEL_SEED = 12345
FLANK = 150
WIN = 2 * FLANK + 1
READ_SEED_R1 = 42
READ_SEED_R2 = 43

# event thresholds on the high 32 bits of a per-base draw
THR_N = np.uint64(int(0.001 * (1 << 32)))
THR_SUB = np.uint64(int(0.006 * (1 << 32)))   # N band + 0.5% substitution band

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
COMP = np.zeros(256, dtype=np.uint8)
COMP[:] = np.arange(256, dtype=np.uint8)
for a, b in (b"AT", b"TA", b"CG", b"GC"):
    COMP[a] = b


def h64(seed, item, draw):
    """splitmix64 finaliser of seed*G_SEED + item*G_ITEM + draw*G_DRAW (mod 2^64)."""
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) * G_SEED + np.asarray(item, dtype=np.uint64) * G_ITEM
             + np.asarray(draw, dtype=np.uint64) * G_DRAW)
        z = z ^ (z >> np.uint64(30))
        z = z * MIX1
        z = z ^ (z >> np.uint64(27))
        z = z * MIX2
        z = z ^ (z >> np.uint64(31))
    return z


# --------------------------------------------------------------------------
# SNP panel
# --------------------------------------------------------------------------

@dataclass
class Panel:
    chrom: list
    start: np.ndarray
    end: np.ndarray
    rsid: list
    ref: np.ndarray        # uint8 ASCII
    alt: np.ndarray        # uint8 ASCII
    left: np.ndarray       # [n, 150] uint8 ASCII
    right: np.ndarray      # [n, 150] uint8 ASCII
    dosage: np.ndarray     # [n] int (0,1,2)

    @property
    def n(self) -> int:
        return len(self.chrom)

    def kmers(self, k: int):
        """(ref_kmer, alt_kmer) ASCII arrays [n, k]."""
        a = k // 2
        b = k - 1 - a
        lft = self.left[:, FLANK - a:] if a else self.left[:, :0]
        rgt = self.right[:, :b]
        ref = np.concatenate([lft, self.ref[:, None], rgt], axis=1)
        alt = np.concatenate([lft, self.alt[:, None], rgt], axis=1)
        return ref, alt

    def windows(self):
        """[n, 2, 301] ASCII windows (allele 0 = REF, 1 = ALT)."""
        w = np.empty((self.n, 2, WIN), dtype=np.uint8)
        for al, base in ((0, self.ref), (1, self.alt)):
            w[:, al, :FLANK] = self.left
            w[:, al, FLANK] = base
            w[:, al, FLANK + 1:] = self.right
        return w

    def write_patterns(self, path: str, k: int) -> None:
        """patterns.txt in the snp-pattern-gen output format (snp-pattern-gen.c:351-353)."""
        ref, alt = self.kmers(k)
        with open(path, "w") as fp:
            for i in range(self.n):
                fp.write("%s\t%d\t%d\t%s\t%c\t%c\t%s\t%s\n" % (
                    self.chrom[i], self.start[i], self.end[i], self.rsid[i],
                    chr(self.ref[i]), chr(self.alt[i]),
                    ref[i].tobytes().decode("latin-1"), alt[i].tobytes().decode("latin-1")))


def read_bed(path: str):
    """BED rows as (chr, start, end, rsid, ref, alt) strings; .gz accepted."""
    op = gzip.open if path.endswith(".gz") else open
    rows = []
    with op(path, "rt") as fp:
        for line in fp:
            f = line.split()
            if len(f) >= 6:
                rows.append((f[0], int(f[1]), int(f[2]), f[3], f[4], f[5]))
    return rows


def synthetic_bed(n: int, seed: int = 777):
    """C5's synthetic panel: chr1-22 uniform, pos uniform, ref != alt uniform."""
    idx = np.arange(n, dtype=np.uint64)
    r0 = h64(seed, idx, 0)
    r1 = h64(seed, idx, 1)
    chrom = (r0 >> np.uint64(32)) % np.uint64(22) + np.uint64(1)
    pos = (r1 >> np.uint64(32)) % np.uint64(240_000_000) + np.uint64(10_000)
    ref = (r0 & np.uint64(3)).astype(np.int64)
    alt = (ref + 1 + ((r1 & np.uint64(0xFFFF)) % np.uint64(3)).astype(np.int64)) % 4
    return [("chr%d" % int(chrom[i]), int(pos[i]), int(pos[i]) + 1, "rs_syn%d" % i,
             "ACGT"[ref[i]], "ACGT"[alt[i]]) for i in range(n)]


def make_panel(rows, seed: int = PANEL_SEED) -> Panel:
    keep = [r for r in rows if len(r[4]) == 1 and len(r[5]) == 1
            and r[4] in "ACGT" and r[5] in "ACGT"]
    n = len(keep)
    idx = np.arange(n, dtype=np.uint64)[:, None]
    q = np.arange(FLANK, dtype=np.uint64)[None, :]
    left = ACGT[(h64(seed, idx, 1000 + q) & np.uint64(3)).astype(np.int64)]
    right = ACGT[(h64(seed, idx, 2000 + q) & np.uint64(3)).astype(np.int64)]
    dosage = ((h64(seed, np.arange(n, dtype=np.uint64), 999) >> np.uint64(32))
              % np.uint64(3)).astype(np.int64)
    return Panel(
        chrom=[r[0] for r in keep],
        start=np.array([r[1] for r in keep], dtype=np.int64),
        end=np.array([r[2] for r in keep], dtype=np.int64),
        rsid=[r[3] for r in keep],
        ref=np.frombuffer("".join(r[4] for r in keep).encode(), dtype=np.uint8).copy(),
        alt=np.frombuffer("".join(r[5] for r in keep).encode(), dtype=np.uint8).copy(),
        left=left.reshape(n, FLANK), right=right.reshape(n, FLANK), dosage=dosage)


def default_bed_path() -> str:
    here = os.path.dirname(os.path.abspath(__file__))
    return os.path.join(os.path.dirname(here), "data", "SNP_GRCh38_hg38_wChr.bed.gz")


def grch38_panel() -> Panel:
    return make_panel(read_bed(default_bed_path()))


# --------------------------------------------------------------------------
# Reads
# --------------------------------------------------------------------------

def f_snp_threshold(f_snp: float) -> np.uint64:
    return np.uint64(min(int(round(f_snp * (1 << 32))), 1 << 32))


def gen_reads(panel: Panel, n_reads: int, first: int = 0, seed: int = READ_SEED_R1,
              f_snp: float = 0.01, read_len: int = 150) -> np.ndarray:
    """Reads first..first+n_reads-1 as a [n_reads, read_len] uint8 ASCII array."""
    assert 1 <= read_len <= WIN
    ii = np.arange(first, first + n_reads, dtype=np.uint64)
    thr = f_snp_threshold(f_snp)
    r0 = h64(seed, ii, 0)
    r1 = h64(seed, ii, 1)
    r2 = h64(seed, ii, 2)
    r3 = h64(seed, ii, 3)
    n_snp = np.uint64(max(panel.n, 1))
    is_snp = ((r0 >> np.uint64(32)) < thr) & (panel.n > 0)
    snp = (((r1 >> np.uint64(32)) * n_snp) >> np.uint64(32)).astype(np.int64)
    g = panel.dosage[snp] if panel.n else np.zeros(n_reads, dtype=np.int64)
    alt = (g == 2) | ((g == 1) & ((r1 & np.uint64(1)) == 1))
    n_start = np.uint64(WIN - read_len + 1)
    start = (((r2 >> np.uint64(32)) * n_start) >> np.uint64(32)).astype(np.int64)
    rc = (r3 & np.uint64(1)) == 1

    p = np.arange(read_len, dtype=np.uint64)[None, :]
    r = h64(seed, ii[:, None], np.uint64(16) + p)
    base = (r & np.uint64(3)).astype(np.int64)
    if panel.n:
        w = panel.windows()
        codes = np.full(256, 0, dtype=np.int64)
        codes[ord("C")], codes[ord("G")], codes[ord("T")] = 1, 2, 3
        sel = np.nonzero(is_snp)[0]
        if len(sel):
            cols = start[sel, None] + np.arange(read_len)[None, :]
            base[sel] = codes[w[snp[sel], alt[sel].astype(np.int64)][np.arange(len(sel))[:, None], cols]]
    u = r >> np.uint64(32)
    sub = ((r >> np.uint64(2)) & np.uint64(0xFFFF)) % np.uint64(3)
    is_sub = (u >= THR_N) & (u < THR_SUB)
    base = np.where(is_sub, (base + 1 + sub.astype(np.int64)) & 3, base)
    out = ACGT[base]
    out[u < THR_N] = ord("N")
    if rc.any():
        out[rc] = COMP[out[rc][:, ::-1]]
    return out


def fastq_bytes(reads: np.ndarray, first: int = 0) -> bytes:
    """4-line FASTQ, names @r<i>, quality all 'I'."""
    n, L = reads.shape
    qual = b"I" * L
    parts = []
    for i in range(n):
        parts.append(b"@r%d\n" % (first + i))
        parts.append(reads[i].tobytes())
        parts.append(b"\n+\n")
        parts.append(qual)
        parts.append(b"\n")
    return b"".join(parts)


def fastq_bytes_np(reads: np.ndarray, first: int = 0) -> bytes:
    """fastq_bytes(reads, first) built with array operations (the same bytes):
    records whose read numbers have the same digit count have the same length,
    so each such run is one 2-D byte array filled column by column."""
    n, L = reads.shape
    out = []
    i = 0
    while i < n:
        d = len(str(first + i))
        j = min(n, 10 ** d - first)           # first index with d + 1 digits
        m = j - i
        tpl = np.frombuffer(b"@r" + b"0" * d + b"\n" + b"A" * L + b"\n+\n" + b"I" * L + b"\n", np.uint8)
        rec = np.tile(tpl, (m, 1))
        num = np.arange(first + i, first + j, dtype=np.int64)
        for c in range(d - 1, -1, -1):        # digits, least significant first
            num, dig = np.divmod(num, 10)
            rec[:, 2 + c] += dig.astype(np.uint8)
        rec[:, 3 + d:3 + d + L] = reads[i:j]
        out.append(rec.tobytes())
        i = j
    return b"".join(out)


def write_fastq(path: str, panel: Panel, n_reads: int, seed: int = READ_SEED_R1,
                f_snp: float = 0.01, read_len: int = 150, chunk: int = 200_000) -> None:
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "wb") as fp:
        for first in range(0, n_reads, chunk):
            m = min(chunk, n_reads - first)
            fp.write(fastq_bytes(gen_reads(panel, m, first, seed, f_snp, read_len), first))


def pack_reads(reads) -> tuple:
    """list of bytes / 2-D array -> (seq uint8, offs uint64, lens uint32), packed back to back."""
    if isinstance(reads, np.ndarray) and reads.ndim == 2:
        n, L = reads.shape
        return (np.ascontiguousarray(reads).reshape(-1),
                np.arange(n, dtype=np.uint64) * np.uint64(L),
                np.full(n, L, dtype=np.uint32))
    lens = np.array([len(r) for r in reads], dtype=np.uint32)
    offs = np.zeros(len(reads), dtype=np.uint64)
    if len(reads) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    seq = np.frombuffer(b"".join(bytes(r) for r in reads), dtype=np.uint8).copy()
    return seq, offs, lens
