"""The CPU oracle (oracle/vafc_oracle.c) against the reference's golden vectors.

The goldens were produced by the REAL reference (oracle/_ref/vaf-counter and
oracle/_ref/ref_kmer_dump, compiled from /root/reference) by
tests/golden/make_golden.py.  This pins the oracle before it is used to check
the HIP path.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, ORACLE_CLI, REF_CLI, run_cli

import json

with open(os.path.join(GOLDEN, "manifest.json")) as _f:
    CASE_NAMES = [c["name"] for c in json.load(_f)["cases"]]


@pytest.mark.parametrize("name", CASE_NAMES)
def test_oracle_cli_matches_reference(name, manifest, synth_dir, tmp_path):
    entry = next(c for c in manifest["cases"] if c["name"] == name)
    rc, stats, data, err = run_cli(ORACLE_CLI, entry, synth_dir, tmp_path)
    assert rc == entry["exit"]
    if entry["vaf_md5"] is not None:
        assert hashlib.md5(data).hexdigest() == entry["vaf_md5"]
        for key in ("bases", "seqs", "kmers"):
            assert stats.get(key) == entry["stats"].get(key), key
    assert ("collisions detected" in err) == entry["collision_warning"]


@pytest.mark.parametrize("k", [1, 5, 15, 16, 17, 21, 31])
def test_oracle_kmers_match_reference_extract(k):
    import oracle as O
    z = np.load(os.path.join(GOLDEN, "kmers_k%d.npz" % k))
    seq, lens, counts, digests = z["seq"], z["lens"], z["counts"], z["digests"]
    pos = 0
    for i, L in enumerate(lens):
        read = seq[pos:pos + L].tobytes()
        pos += int(L)
        km = O.read_kmers(k, read).astype("<u8")
        assert km.size == counts[i], (k, i)
        assert hashlib.md5(km.tobytes()).digest() == digests[i].tobytes(), (k, i)


def test_decode_quirk_examples():
    """nibble LUT on the first 16*floor(len/16) bytes, seq_nt4_table after."""
    import oracle as O
    s = b"ASATSASTTACGTACG"                 # len 16: all head -> S decodes as C (nibble 3)
    assert list(O.decode(s)[:4]) == [0, 1, 0, 3]
    s = b"A" * 38 + b"S" + b"A"             # S at position 38 of 40 (tail) -> invalid
    assert O.decode(s)[38] == 4
    assert O.decode(bytes([0xC1]) + b"A" * 15)[0] == 0      # 0xC1 in the head -> A
    assert O.decode(b"Q" + b"A" * 15)[0] == 0               # Q -> A
    assert O.decode(b"A" * 16 + b"Q")[16] == 4              # Q in the tail -> invalid
    tail = O.decode(b"A" * 16 + bytes([0, 1, 2, 3]))
    assert list(tail[16:]) == [0, 1, 2, 3]                  # raw 0..3 in the tail
    head = O.decode(bytes([0, 1, 2, 3]) + b"A" * 12)
    assert list(head[:4]) == [4, 0, 4, 1]                   # nibble LUT in the head


@pytest.mark.skipif(not os.path.exists(REF_CLI), reason="reference binary not built")
def test_reference_binary_still_matches_manifest(manifest, synth_dir, tmp_path):
    """The committed goldens are reproducible by the reference built here."""
    for entry in manifest["cases"][:6]:
        rc, stats, data, _ = run_cli(REF_CLI, entry, synth_dir, tmp_path)
        assert rc == entry["exit"]
        if entry["vaf_md5"]:
            assert hashlib.md5(data).hexdigest() == entry["vaf_md5"]
