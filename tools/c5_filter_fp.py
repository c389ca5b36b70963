#!/usr/bin/env python3
"""False-positive rate of the large-panel LDS Bloom filter (CPU only): the
200k-SNP C5 panel's k = 21 keys, 1M uniform random 21-mers, for the 128 KiB
power-of-two filter (word = product bits 5..19, vafc_common.h vc_filter_word)
and the multiply-high-scaled filter of vc_big_word at several sizes.
    python tools/c5_filter_fp.py
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import filter_fp as FF  # noqa: E402

K = 21
M32, M24, M20 = np.uint64(0xFFFFFFFF), np.uint64(0xFFFFFF), np.uint64(0xFFFFF)


def strands(ks):
    return FF.lo(ks), FF.lo(FF.revcomp(ks))


def mask(fl, rl):
    return (np.uint32(1) << (fl & np.uint32(31))) | (np.uint32(1) << (rl & np.uint32(31)))


def word_pow2(fl, rl, nwords):
    pr = ((fl.astype(np.uint64) & M24) * (rl.astype(np.uint64) & M24)) & M32
    return ((pr >> np.uint64(5)) & np.uint64(nwords - 1)).astype(np.int64)


def word_big(fl, rl, nwords):
    p = ((fl.astype(np.uint64) & M20) * (rl.astype(np.uint64) & M20)) & M32
    return ((p * np.uint64(nwords)) >> np.uint64(32)).astype(np.int64)


def fp_unaligned(keys, q, nwords):
    """The 32 bits at byte offset (p * (4 nwords - 3)) >> 32 of the filter,
    any alignment (no address mask in the kernel).  Tried in round 5: fewer
    false positives, but unaligned LDS dword reads made the C5 kernel 2.15x
    slower (profiles/r05n_ab_unaligned_lds.log), so not kept."""
    nb = 4 * nwords
    F = np.zeros(nb + 8, np.uint8)

    def off(fl, rl):
        p = ((fl.astype(np.uint64) & M20) * (rl.astype(np.uint64) & M20)) & M32
        return ((p * np.uint64(nb - 3)) >> np.uint64(32)).astype(np.int64)

    fl, rl = strands(keys)
    b = off(fl, rl)
    for s in (fl, rl):
        g = 8 * b + (s & np.uint32(31)).astype(np.int64)
        np.bitwise_or.at(F, g >> 3, (np.uint8(1) << (g & 7).astype(np.uint8)))
    qf, qr = strands(q)
    qb = off(qf, qr)
    ok = np.ones(len(q), bool)
    for s in (qf, qr):
        g = 8 * qb + (s & np.uint32(31)).astype(np.int64)
        ok &= ((F[g >> 3] >> (g & 7).astype(np.uint8)) & 1) == 1
    return float(np.mean(ok))


def fp(keys, q, word, nwords):
    F = np.zeros(nwords, np.uint32)
    fl, rl = strands(keys)
    np.bitwise_or.at(F, word(fl, rl, nwords), mask(fl, rl))
    qf, qr = strands(q)
    qm = mask(qf, qr)
    return float(np.mean((F[word(qf, qr, nwords)] & qm) == qm))


def main():
    import vafc
    import vafc_synth as S
    panel = S.make_panel(S.synthetic_bed(200_000))
    d = tempfile.mkdtemp()
    pat = os.path.join(d, "p.txt")
    panel.write_patterns(pat, K)
    keys, _, _ = vafc.load_patterns(pat).keys(K)
    keys = np.unique(np.asarray(keys, dtype=np.uint64))
    q = np.random.default_rng(1).integers(0, 1 << (2 * K), size=1_000_000, dtype=np.uint64)
    print("keys %d" % len(keys))
    print("128 KiB, power of two (vc_filter_word):  FP %.4f" % fp(keys, q, word_pow2, 32768))
    for kib_words in (32768, 34816, 36860):
        print("%6.2f KiB, multiply-high (vc_big_word): FP %.4f" % (kib_words / 256, fp(keys, q, word_big, kib_words)))
    print("%6.2f KiB, any byte offset (not kept):     FP %.4f" % (36860 / 256, fp_unaligned(keys, q, 36860)))


if __name__ == "__main__":
    main()
