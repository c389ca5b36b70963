"""Gzip shapes of the synthetic C1 reads for the split-gzip tests (round 6):
built from c1_10k.fq in a directory, by tests/golden/make_golden_gz.py (which
runs the reference on them) and again at test time by conftest.synth_dir
(whose md5 check pins them).  Python's zlib at level 1 with mtime 0 is
deterministic.

  c1_10k_multi.fq.gz     three gzip members, cut at byte offsets that fall
                         inside records (as `cat a.gz b.gz c.gz`)
  c1_10k_trailing.fq.gz  one member followed by 3 KiB of non-gzip bytes
                         (gzread ignores them)
  c1_10k_badcrc.fq.gz    three members, the middle one's CRC-32 trailer wrong
                         (gzread's output around a failed check depends on its
                         buffers, so no reference golden: the tests compare
                         the split driver with the whole-file one)
"""
import gzip
import os
import random

VARIANTS = ("c1_10k_multi.fq.gz", "c1_10k_trailing.fq.gz", "c1_10k_badcrc.fq.gz")


def _member(data: bytes) -> bytes:
    return gzip.compress(data, compresslevel=1, mtime=0)


def make(d: str) -> None:
    with open(os.path.join(d, "c1_10k.fq"), "rb") as f:
        text = f.read()
    cuts = [0, len(text) // 3 + 17, 2 * len(text) // 3 + 101, len(text)]
    members = [_member(text[a:b]) for a, b in zip(cuts, cuts[1:])]
    with open(os.path.join(d, "c1_10k_multi.fq.gz"), "wb") as f:
        f.write(b"".join(members))
    rnd = random.Random(5)
    junk = bytes(rnd.randrange(256) for _ in range(3072))
    with open(os.path.join(d, "c1_10k_trailing.fq.gz"), "wb") as f:
        f.write(_member(text) + b"\x00" + junk)
    bad = bytearray(members[1])
    bad[-8] ^= 0x5A            # the CRC-32 of the middle member
    with open(os.path.join(d, "c1_10k_badcrc.fq.gz"), "wb") as f:
        f.write(members[0] + bytes(bad) + members[2])
