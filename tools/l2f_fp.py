#!/usr/bin/env python3
"""False-positive rate of the second-level filter (large panels, CPU only).

Builds the 2nd-level filter as vc_create does for the 200k-SNP synthetic panel
(C5, k = 21, ~400k keys, 2^19 words) with two key hashes and queries 2M
uniform random 21-mers:
  canon   word / bits from vc_hash / vc_hash2 of the canonical k-mer (round 1:
          the drain reverse-complements every queued k-mer and hashes it)
  strands word / bits from a symmetric mix of the two strands' low 32 bits,
          (flo, rlo), which the scan already has (round 2's form)
  l2s     round 5's form of the same (vafc_common.h vc_l2s_hash*, -DVC_BIG_SYMQ)
    python tools/l2f_fp.py
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))

K = 21
U32 = np.uint64(0xFFFFFFFF)


def revcomp(x):
    r = np.zeros_like(x)
    for _ in range(K):
        r = (r << np.uint64(2)) | (np.uint64(3) - (x & np.uint64(3)))
        x = x >> np.uint64(2)
    return r


def m32(x):
    return (np.asarray(x, np.uint64) & U32).astype(np.uint32)


def vc_hash(key):
    lo, hi = m32(key), m32(key >> np.uint64(32))
    x = lo ^ (hi * np.uint32(0x9E3779B1))
    x ^= x >> np.uint32(16)
    return x * np.uint32(0x85EBCA77)


def vc_hash2(key):
    return (m32(key >> np.uint64(17)) ^ m32(key)) * np.uint32(0x9E3779B1)


def mask3(h2):
    one = np.uint32(1)
    return (one << (h2 & np.uint32(31))) | (one << ((h2 >> np.uint32(5)) & np.uint32(31))) | \
           (one << ((h2 >> np.uint32(10)) & np.uint32(31)))


def canon_filter(keys, l2bits):
    return vc_hash(keys) >> np.uint32(32 - l2bits), mask3(vc_hash2(keys))


def strands_filter(keys, l2bits):
    """vafc_common.h vc_l2f_word / vc_l2f_mask on (flo, rlo): a 64-bit product
    of the two strands (each XORed with the same constant: symmetric), its
    halves folded and multiplied."""
    c = np.uint64(0x9E3779B9)
    fl = (keys & U32) ^ c
    rl = (revcomp(keys) & U32) ^ c
    p = fl * rl                                            # exact: both < 2^32
    hi, lo = m32(p >> np.uint64(32)), m32(p)
    w = (hi ^ lo) * np.uint32(0x85EBCA77)
    b = (hi + (lo ^ (lo >> np.uint32(15)))) * np.uint32(0xC2B2AE35)
    return w >> np.uint32(32 - l2bits), mask3(b >> np.uint32(17))


def l2s_filter(keys, l2bits):
    """vafc_common.h vc_l2s_hash / vc_l2s_hash2 (round 5, -DVC_BIG_SYMQ): two
    multiplies of the strands' low words, summed / XORed, then mixed."""
    m = np.uint32(0x9E3779B1)
    u, v = m32(keys) * m, m32(revcomp(keys)) * m
    x = u + v
    x ^= x >> np.uint32(15)
    x = x * np.uint32(0x85EBCA77)
    y = u ^ v
    y ^= y >> np.uint32(13)
    y = y * np.uint32(0xC2B2AE3D)
    return x >> np.uint32(32 - l2bits), mask3(y)


def fp(fn, keys, q, l2bits):
    words = np.zeros(1 << l2bits, np.uint32)
    w, m = fn(keys, l2bits)
    np.bitwise_or.at(words, w, m)
    wq, mq = fn(q, l2bits)
    return float(((words[wq] & mq) == mq).mean())


def main():
    import vafc
    import vafc_synth as S
    panel = S.make_panel(S.synthetic_bed(200_000))
    d = tempfile.mkdtemp()
    pat = os.path.join(d, "p.txt")
    panel.write_patterns(pat, K)
    keys, _, _ = vafc.load_patterns(pat).keys(K)
    keys = np.unique(np.asarray(keys, dtype=np.uint64))
    l2bits = 12
    while l2bits < 19 and (32 << l2bits) < 40 * keys.size:
        l2bits += 1
    q = np.random.default_rng(1).integers(0, 1 << (2 * K), size=2_000_000, dtype=np.uint64)
    q = np.minimum(q, revcomp(q))
    print("%d keys, 2^%d words (%.1f bits per key)" % (keys.size, l2bits, 32 * (1 << l2bits) / keys.size))
    for name, fn in (("canon", canon_filter), ("strands", strands_filter), ("l2s", l2s_filter)):
        print("%-8s FP %.4f %%" % (name, 100 * fp(fn, keys, q, l2bits)))


if __name__ == "__main__":
    main()
