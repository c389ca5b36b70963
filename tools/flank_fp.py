#!/usr/bin/env python3
"""Pass rate of the flank-bitmap prefilter (vafc_common.h vc_flank_mark,
VC_FLANK_DIST) on the benchmark panel, CPU only (tools, not tests).

The bitmap is the exact 2^20-bit set of the 10-mers of every key and of its
reverse complement that end at the test distances before the key's last base;
a window passes iff its own 10-mers at those distances are all set.  Two
forms: the round-2 one (first and last ten bases, distances 0 and k - 10) and
the four-test one of the kernels (distances VC_FLANK_DIST(k, 0..3)).  Each is
queried with 4M uniform random k-mers and with the valid windows of 200k
benchmark reads (C2's generator: 1 % of reads drawn over a SNP, so some
passes are true hits; "true" = windows that are keys).
    python tools/flank_fp.py [--extra | --sampled]
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))
import vafc  # noqa: E402
import vafc_synth as S  # noqa: E402

M = np.uint64((1 << 20) - 1)


def revcomp(x, K):
    r = np.zeros_like(x)
    for _ in range(K):
        r = (r << np.uint64(2)) | (np.uint64(3) - (x & np.uint64(3)))
        x = x >> np.uint64(2)
    return r


def dists(K, tests):
    if tests == 2:
        return (0, K - 10)
    return tuple((t * (K - 10) + 1) // 3 for t in range(4))   # VC_FLANK_DIST


def read_windows(reads, K):
    """Forward k-mers of the valid windows of reads (uint8 ASCII rows)."""
    lut = np.full(256, 4, np.int64)
    for c, v in zip(b"ACGT", range(4)):
        lut[c] = v
    codes = lut[reads]
    bad = codes == 4
    cz = np.where(bad, 0, codes).astype(np.uint64)
    n, L = codes.shape
    mk = np.uint64((1 << (2 * K)) - 1) if K < 32 else np.uint64(-1)
    acc = np.zeros(n, np.uint64)
    out = []
    run = np.zeros(n, np.int64)
    for p in range(L):
        acc = ((acc << np.uint64(2)) | cz[:, p]) & mk
        run = np.where(bad[:, p], 0, run + 1)
        if p >= K - 1:
            out.append(acc[run >= K])
    return np.concatenate(out)


def main():
    panel = S.make_panel(S.read_bed(S.default_bed_path()))
    reads = S.gen_reads(panel, 200_000)
    for K in (21, 25, 31):
        d = tempfile.mkdtemp()
        pat = os.path.join(d, "p.txt")
        panel.write_patterns(pat, K)
        keys, _, _ = vafc.load_patterns(pat).keys(K)
        keys = np.unique(np.asarray(keys, dtype=np.uint64))
        allk = np.concatenate([keys, revcomp(keys, K)])
        q = np.random.default_rng(1).integers(0, 1 << (2 * K), size=4_000_000, dtype=np.uint64)
        win = read_windows(reads, K)
        true = np.isin(win, allk).mean()
        for tests in (2, 4):
            ds = dists(K, tests)
            bm = np.zeros(1 << 20, bool)
            for dd in ds:
                bm[(allk >> np.uint64(2 * dd)) & M] = True

            def passes(x):
                ok = np.ones(x.size, bool)
                for dd in ds:
                    ok &= bm[(x >> np.uint64(2 * dd)) & M]
                return ok.mean()
            print("k=%d tests=%d distances=%s keys %d density %.4f random %.4f%% reads %.4f%% (true hits %.4f%%)"
                  % (K, tests, ds, len(keys), bm.mean(), 100 * passes(q), 100 * passes(win), 100 * true))


def extra_tests():
    """Round 4: more than four tests over the same bitmap (k = 21, on the
    benchmark reads): every set is closed under d -> k - 10 - d, so the
    bitmap stays closed under reverse complement."""
    panel = S.make_panel(S.read_bed(S.default_bed_path()))
    reads = S.gen_reads(panel, 200_000)
    K = 21
    d = tempfile.mkdtemp()
    pat = os.path.join(d, "p.txt")
    panel.write_patterns(pat, K)
    keys, _, _ = vafc.load_patterns(pat).keys(K)
    keys = np.unique(np.asarray(keys, dtype=np.uint64))
    allk = np.concatenate([keys, revcomp(keys, K)])
    win = read_windows(reads, K)
    for ds in [(0, 4, 7, 11), (0, 3, 8, 11), (0, 2, 4, 7, 9, 11), (0, 2, 5, 6, 9, 11), (0, 1, 3, 8, 10, 11),
               (0, 3, 5, 6, 8, 11)]:
        bm = np.zeros(1 << 20, bool)
        for dd in ds:
            bm[(allk >> np.uint64(2 * dd)) & M] = True
        ok = np.ones(win.size, bool)
        for dd in ds:
            ok &= bm[(win >> np.uint64(2 * dd)) & M]
        print("k=21 distances=%s density %.3f reads %.4f%%" % (ds, bm.mean(), 100 * ok.mean()))




def sampled_tests():
    """Round 5: a content-sampled flank filter.  Each
    10-mer is 'sampled' iff a hash of it is 0 mod s (the same rule on the read
    and on the key, so a key's sampled 10-mers are its window's); S holds the
    sampled 10-mers of every key orientation; a window passes iff every
    sampled 10-mer inside it is in S -- and a window with none inside must
    pass (nothing to test).  Prints the pass rate on the benchmark reads and
    the share of windows with no sampled 10-mer, per s."""
    panel = S.make_panel(S.read_bed(S.default_bed_path()))
    reads = S.gen_reads(panel, 200_000)
    K = 21
    d = tempfile.mkdtemp()
    pat = os.path.join(d, "p.txt")
    panel.write_patterns(pat, K)
    keys, _, _ = vafc.load_patterns(pat).keys(K)
    keys = np.unique(np.asarray(keys, dtype=np.uint64))
    allk = np.concatenate([keys, revcomp(keys, K)])
    win = read_windows(reads, K)

    def h(v):
        return ((v * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(40)) & np.uint64(0xFFFFFF)

    for s in (2, 3, 4, 6):
        bm = np.zeros(1 << 20, bool)
        for dd in range(K - 9):
            v = (allk >> np.uint64(2 * dd)) & M
            sel = (h(v) % np.uint64(s)) == 0
            bm[v[sel]] = True
        ok = np.ones(win.size, bool)
        nsamp = np.zeros(win.size, np.int64)
        for dd in range(K - 9):
            v = (win >> np.uint64(2 * dd)) & M
            sel = (h(v) % np.uint64(s)) == 0
            nsamp += sel
            ok &= ~sel | bm[v]
        print("k=21 sampled 1/%d: density %.3f, windows with no sampled 10-mer %.3f%%, pass %.4f%%" % (
            s, bm.mean(), 100 * (nsamp == 0).mean(), 100 * ok.mean()))


if __name__ == "__main__":
    if "--extra" in sys.argv:
        extra_tests()
    elif "--sampled" in sys.argv:
        sampled_tests()
    else:
        main()
