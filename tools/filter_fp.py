#!/usr/bin/env python3
"""False-positive rate of the LDS prefilter on the benchmark panel (CPU only).

Builds the filter exactly as vc_create does (vafc_common.h) for the GRCh38
panel's k=21 keys and queries 2M uniform random 21-mers.  Also evaluates the
earlier word indices: the sum of the strands (constant at the centre base of
an odd k: fwd and revcomp add to 3 there) and the product's top bits (which
separate a SNP's ref and alt k-mers, doubling the filter load).
    python tools/filter_fp.py
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))

K, WBITS = 21, 15
M32, M24 = np.uint64(0xFFFFFFFF), np.uint64(0xFFFFFF)


def revcomp(x):
    r = np.zeros_like(x)
    for _ in range(K):
        r = (r << np.uint64(2)) | (np.uint64(3) - (x & np.uint64(3)))
        x = x >> np.uint64(2)
    return r


def lo(x):
    return (x & M32).astype(np.uint32)


def product_filter(ks, lo_bit=5):   # vafc_common.h: vc_filter_word / vc_filter_mask (k=21: lo 5)
    fl, rl = lo(ks), lo(revcomp(ks))
    pr = ((fl.astype(np.uint64) & M24) * (rl.astype(np.uint64) & M24)) & M32
    w = ((pr >> np.uint64(lo_bit)) & np.uint64((1 << WBITS) - 1)).astype(np.uint32)
    m = (np.uint32(1) << (fl & np.uint32(31))) | (np.uint32(1) << (rl & np.uint32(31)))
    return w, m


def sum_filter(ks):           # kernel v6: word and bits from lo32(fwd) + lo32(rc)
    fx = ((lo(ks).astype(np.uint64) + lo(revcomp(ks))) & M32).astype(np.uint32)
    w = (fx >> np.uint32(5)) & np.uint32((1 << WBITS) - 1)
    m = (np.uint32(1) << (fx & np.uint32(31))) | (np.uint32(1) << ((fx >> np.uint32(20)) & np.uint32(31)))
    return w, m


def main():
    import vafc
    import vafc_synth as S
    panel = S.make_panel(S.read_bed(S.default_bed_path()))
    d = tempfile.mkdtemp()
    pat = os.path.join(d, "p.txt")
    panel.write_patterns(pat, K)
    keys, _, _ = vafc.load_patterns(pat).keys(K)
    keys = np.unique(np.asarray(keys, dtype=np.uint64))
    q = np.random.default_rng(1).integers(0, 1 << (2 * K), size=2_000_000, dtype=np.uint64)
    for name, fn in (("product, bits 5..19 (current: centre base excluded)", product_filter),
                     ("product, bits 17..31 (v7)", lambda ks: product_filter(ks, 32 - WBITS)),
                     ("sum (v6)", sum_filter)):
        F = np.zeros(1 << WBITS, dtype=np.uint32)
        w, m = fn(keys)
        np.bitwise_or.at(F, w, m)
        qw, qm = fn(q)
        fp = float(np.mean((F[qw] & qm) == qm))
        print("%-52s keys %d  words used %5d / %d  FP %.4f" % (name, len(keys), np.count_nonzero(F), 1 << WBITS, fp))


if __name__ == "__main__":
    main()
