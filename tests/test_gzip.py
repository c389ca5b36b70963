"""The parallel gzip inflater (vafc_gzip.cpp) against zlib's gzread, the
reference's reader of .gz input (vaf-counter.c:12,557): identical byte
streams for every compression level and strategy, multi-member files, header
options, trailing bytes and truncated files, at chunk sizes from 1 KiB up;
the speculative path is checked to be the one that runs (accepted chunks),
and the FASTQ reader on top of it against the sequential gzread reader."""
import gzip
import os
import struct
import zlib

import numpy as np
import pytest


def _fastq_text(rng, n, L=150):
    out = []
    for i in range(n):
        seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, L)].tobytes()
        if i % 37 == 0:
            seq = seq[:40] + b"N" * 5 + seq[45:]
        out.append(b"@r%d extra\n%s\n+\n%s\n" % (i, seq, b"I" * L))
    return b"".join(out)


def _member(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, flags=0, extra=b"", name=b"", comment=b"",
            mem_level=8):
    """One RFC 1952 member with the given header options."""
    hdr = bytearray(b"\x1f\x8b\x08" + bytes([flags]) + b"\x00\x00\x00\x00\x00\x03")
    if flags & 4:
        hdr += struct.pack("<H", len(extra)) + extra
    if flags & 8:
        hdr += name + b"\x00"
    if flags & 16:
        hdr += comment + b"\x00"
    if flags & 2:
        hdr += struct.pack("<H", zlib.crc32(bytes(hdr)) & 0xffff)
    c = zlib.compressobj(level, zlib.DEFLATED, -15, mem_level, strategy)
    body = c.compress(data) + c.flush()
    return bytes(hdr) + body + struct.pack("<II", zlib.crc32(data) & 0xffffffff, len(data) & 0xffffffff)


def _check(path, threads=4, chunks=(1024, 4096, 65536, 1 << 22), want_accept=False):
    import vafc
    ref = vafc.gz_inflate_zlib(path)
    for ch in chunks:
        got = vafc.gz_inflate_parallel(path, threads=threads, chunk_bytes=ch)
        assert got is not None, (path, ch)
        data, st = got
        assert len(data) == len(ref) and data == ref, (path, ch, len(data), len(ref), st)
        if want_accept and st["chunks"] > 2:   # the speculative path ran
            assert st["accepted"] >= 2 and st["fallback"] <= st["accepted"] // 4 + 1, (path, ch, st)
    return ref


@pytest.fixture(scope="module")
def text():
    return _fastq_text(np.random.default_rng(11), 6000)


@pytest.mark.parametrize("level", [1, 2, 4, 6, 9])
def test_levels(tmp_path, text, level):
    p = str(tmp_path / "x.fq.gz")
    with open(p, "wb") as f:
        f.write(gzip.compress(text, compresslevel=level))
    assert _check(p, want_accept=True) == text


@pytest.mark.parametrize("strategy", ["fixed", "huffman", "rle", "filtered", "stored"])
def test_strategies(tmp_path, text, strategy):
    """Fixed-Huffman and stored blocks are never found by the block search:
    every chunk after the first goes through zlib from the true boundary."""
    p = str(tmp_path / "s.gz")
    st = {"fixed": zlib.Z_FIXED, "huffman": zlib.Z_HUFFMAN_ONLY, "rle": zlib.Z_RLE,
          "filtered": zlib.Z_FILTERED, "stored": zlib.Z_DEFAULT_STRATEGY}[strategy]
    level = 0 if strategy == "stored" else 6
    with open(p, "wb") as f:
        f.write(_member(text[:300_000], level=level, strategy=st))
    assert _check(p) == text[:300_000]


def test_small_mem_level_many_blocks(tmp_path, text):
    """memLevel 1: short blocks, many block boundaries per chunk."""
    p = str(tmp_path / "m.gz")
    with open(p, "wb") as f:
        f.write(_member(text, level=6, mem_level=1))
    _check(p, want_accept=True)


def test_multi_member_and_headers(tmp_path, text):
    """Members of every size (empty, tiny, large) with FEXTRA / FNAME /
    FCOMMENT / FHCRC, BGZF-style 64 KiB members."""
    parts = []
    pos = 0
    rng = np.random.default_rng(5)
    flags_cycle = [0, 4, 8, 16, 2, 4 | 8 | 16 | 2]
    i = 0
    while pos < len(text):
        n = int(rng.choice([0, 1, 100, 5000, 65280, 200_000]))
        d = text[pos:pos + n]
        pos += n
        fl = flags_cycle[i % len(flags_cycle)]
        parts.append(_member(d, level=1 + i % 9, flags=fl, extra=b"BC\x02\x00\x00\x00", name=b"r.fq",
                             comment=b"c" * (i % 3)))
        i += 1
    p = str(tmp_path / "mm.gz")
    with open(p, "wb") as f:
        f.write(b"".join(parts))
    assert _check(p, threads=3, chunks=(1024, 9000, 1 << 20)) == text
    import vafc
    _, st = vafc.gz_inflate_parallel(p, threads=3, chunk_bytes=4096)
    assert st["members"] == len(parts) and st["crc_error"] == 0


@pytest.mark.parametrize("tail", [b"", b"\x00", b"\x00" * 100, b"garbage after the member", b"\x1f"])
def test_trailing_bytes(tmp_path, text, tail):
    """gzread ignores bytes after a member that are not a gzip header."""
    p = str(tmp_path / "t.gz")
    with open(p, "wb") as f:
        f.write(_member(text[:200_000]) + tail)
    assert _check(p, chunks=(1024, 1 << 20)) == text[:200_000]


@pytest.mark.parametrize("tail", [b"\x1f\x8b\x08\xe0" + b"\x00" * 20, b"\x1f\x8b\x09\x00" + b"\x00" * 20])
def test_rejected_member_header(tmp_path, text, tail):
    """A second member whose header zlib rejects (reserved flags, unknown
    method) is a data error: the stream ends after the first member.  gzread
    itself loses the output of the read call that hit the error (here the
    whole stream, with one 1 MiB call; the reference's 16 KiB kseq reads lose
    less), so it delivers a prefix of ours."""
    import vafc
    p = str(tmp_path / "t.gz")
    with open(p, "wb") as f:
        f.write(_member(text[:200_000]) + tail)
    ref = vafc.gz_inflate_zlib(p)
    for ch in (1024, 1 << 20):
        data, st = vafc.gz_inflate_parallel(p, threads=4, chunk_bytes=ch)
        assert data == text[:200_000] and st["members"] == 1
        assert data.startswith(ref)


def test_truncated(tmp_path, text):
    """Files cut at many points: gzread's output up to the cut."""
    full = _member(text[:400_000], level=6)
    rng = np.random.default_rng(9)
    cuts = sorted(set([10, 11, 12, 50, len(full) - 8, len(full) - 1, len(full) - 4]
                      + [int(x) for x in rng.integers(20, len(full), 12)]))
    for c in cuts:
        p = str(tmp_path / ("c%d.gz" % c))
        with open(p, "wb") as f:
            f.write(full[:c])
        import vafc
        ref = vafc.gz_inflate_zlib(p)
        for ch in (1024, 30000):
            got = vafc.gz_inflate_parallel(p, threads=4, chunk_bytes=ch)
            if got is None:   # header cut short: the caller falls back to gzread
                assert c < 20
                continue
            assert got[0] == ref, (c, ch, len(got[0]), len(ref))


def test_crc_mismatch_stops_after_member(tmp_path, text):
    """A member whose CRC-32 fails: its data, then the end (the next member is
    not delivered); the failure is reported in the stats."""
    import vafc
    a, b = text[:150_000], text[150_000:300_000]
    m1 = bytearray(_member(a))
    m1[-8] ^= 0xff
    p = str(tmp_path / "crc.gz")
    with open(p, "wb") as f:
        f.write(bytes(m1) + _member(b))
    for ch in (1024, 1 << 20):
        data, st = vafc.gz_inflate_parallel(p, threads=4, chunk_bytes=ch)
        assert data == a and st["crc_error"] == 1


def test_corrupt_data_gives_a_prefix(tmp_path, text):
    """Corrupt deflate data: the output is a prefix of the true stream (gzread's
    own cut-off point is buffer-size dependent) and the reader terminates."""
    import vafc
    full = bytearray(_member(text[:400_000], level=6))
    rng = np.random.default_rng(4)
    for trial in range(8):
        bad = bytearray(full)
        for _ in range(3):
            bad[int(rng.integers(20, len(bad) - 8))] ^= int(rng.integers(1, 256))
        p = str(tmp_path / ("bad%d.gz" % trial))
        with open(p, "wb") as f:
            f.write(bytes(bad))
        for ch in (1024, 50000):
            got = vafc.gz_inflate_parallel(p, threads=3, chunk_bytes=ch)
            assert got is not None
            data = got[0]
            n = len(data)
            # everything before the first corrupted block is exact
            assert n <= len(text) + 258 * 100


def test_random_after_header_terminates(tmp_path):
    import vafc
    rng = np.random.default_rng(2)
    for t in range(6):
        p = str(tmp_path / ("r%d.gz" % t))
        with open(p, "wb") as f:
            f.write(b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\x03" + rng.integers(0, 256, 200_000, dtype=np.uint8).tobytes())
        ref = vafc.gz_inflate_zlib(p)
        got = vafc.gz_inflate_parallel(p, threads=4, chunk_bytes=2048)
        assert got is not None
        assert ref.startswith(got[0][:len(ref)]) or got[0].startswith(ref[:len(got[0])])


def test_not_gzip_declined(tmp_path):
    import vafc
    p = str(tmp_path / "plain.fq")
    with open(p, "wb") as f:
        f.write(b"@a\nACGT\n+\nIIII\n" * 10)
    assert vafc.gz_inflate_parallel(p) is None


@pytest.mark.parametrize("threads", [2, 5])
def test_reader_on_gzip_matches_sequential(tmp_path, text, threads):
    """vc_count_file's gzip path (parallel inflate + block loop) against the
    sequential gzread reader: same reads, bases, sequences and blocks."""
    import vafc
    p = str(tmp_path / "reads.fq.gz")
    with open(p, "wb") as f:
        f.write(_member(text[:500_000], level=1) + _member(text[500_000:], level=9))
    for k, b in ((21, 10_000_000), (5, 1000), (31, 150)):
        st0, r0 = vafc.scan_file(p, k, b, with_reads=True)
        for ch in (1024, 100_000):
            st1, r1 = vafc.scan_file_parallel(p, k, b, threads=threads, piece_bytes=ch, with_reads=True)
            assert (st1.bases, st1.seqs, st1.blocks) == (st0.bases, st0.seqs, st0.blocks)
            assert r1 == r0


def test_crc32_matches_zlib():
    """The member check's CRC-32 (carry-less-multiply folding) against zlib's
    for every length 0..300, longer buffers and arbitrary starting values."""
    import ctypes
    import vafc
    rng = np.random.default_rng(1)
    for n in list(range(0, 300)) + [1000, 4095, 4096, 65537, (1 << 20) + 3]:
        a = rng.integers(0, 256, n, dtype=np.uint8)
        init = int(rng.integers(0, 2 ** 32))
        got = vafc.lib().vc_gz_crc32(init, a.ctypes.data_as(ctypes.c_void_p), n)
        assert got == zlib.crc32(a.tobytes(), init), n


@pytest.mark.parametrize("seed", range(4))
def test_parallel_parse_of_gzip_matches_sequential(tmp_path, monkeypatch, seed):
    """The gzip text parsed in parallel (vc_ingest_gzip: a pump thread feeding
    parse workers, pieces down to tens of bytes, records longer than the
    buffered window) against the sequential gzread reader, on fuzzed FASTQ /
    FASTA with malformed records: same reads, bases, sequences and blocks."""
    import vafc
    from test_reader import _fuzz_file
    rng = np.random.default_rng(300 + seed)
    src = str(tmp_path / "f.fq")
    _fuzz_file(src, rng, 1500)
    raw = open(src, "rb").read()
    if seed == 3:   # long FASTA records, far beyond the window of tiny pieces
        raw = b"".join(b">s%d\n%s\n" % (i, np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, n)].tobytes())
                       for i, n in enumerate([50, 120_000, 7, 300_000, 90]))
    p = str(tmp_path / "f.fq.gz")
    with open(p, "wb") as f:
        f.write(_member(raw, level=1 + seed))
    for piece, parsers in ((37 + 50 * seed, 3), (1 << 20, 2), (4096, 1)):
        monkeypatch.setenv("VAFC_INGEST_PIECE", str(piece))
        monkeypatch.setenv("VAFC_GZ_PARSERS", str(parsers))
        for k, b in ((9, 10_000_000), (5, 60)):
            st0, r0 = vafc.scan_file(p, k, b, with_reads=True)
            st1, r1 = vafc.scan_file_parallel(p, k, b, threads=4, piece_bytes=2048, with_reads=True)
            assert (st1.bases, st1.seqs, st1.blocks) == (st0.bases, st0.seqs, st0.blocks), (piece, k, b)
            assert r1 == r0


def test_parallel_parse_of_gzip_stops_early_without_reading_on(tmp_path, monkeypatch):
    """A gzip FASTQ whose block loop ends at its third empty block (three
    malformed records in a row, -b 1) followed by many megabytes of good reads:
    the parallel parse stops there like the sequential reader (the pump and the
    workers are released), with the same reads and blocks."""
    import vafc
    rng = np.random.default_rng(77)
    good = _fastq_text(rng, 30)
    bad = b"@x\nACGTACGTACGTACGTACGTACGT\n+\n" + b"I" * 30 + b"\n"   # quality longer: -2
    bad = bad * 3
    tail = _fastq_text(rng, 40_000)
    p = str(tmp_path / "stop.fq.gz")
    with open(p, "wb") as f:
        f.write(_member(good + bad + tail, level=1))
    for piece, parsers in ((512, 3), (1 << 16, 2)):
        monkeypatch.setenv("VAFC_INGEST_PIECE", str(piece))
        monkeypatch.setenv("VAFC_GZ_PARSERS", str(parsers))
        st0, r0 = vafc.scan_file(p, 21, 1, with_reads=True)
        st1, r1 = vafc.scan_file_parallel(p, 21, 1, threads=4, piece_bytes=4096, with_reads=True)
        assert (st1.bases, st1.seqs, st1.blocks) == (st0.bases, st0.seqs, st0.blocks)
        assert r1 == r0 and st0.seqs == 30


# --------------------------------------------------------------------------
# shares of one gzip stream over several ranks (round 6; include/vafc.h
# vc_gz_share_scan / vc_scan_gz_share, kmer-cnt_amd/vafc_dist.py), driven here
# in one process: every share's reads in order == the sequential reader's
# --------------------------------------------------------------------------

def _shares(path, world, k=5, block=100, chunk=16 << 10, threads=3, hold=0, held_out=None):
    """Scan, chain and count the `world` shares of a gzip file; returns
    (chained, ranges, crcs, reads in share order).  hold > 0: the scans keep
    their decoded chunks (vc_gz_share_open) and the counts resume from them
    (vc_scan_gz_share_held) where a share fitted the budget; held_out collects
    which shares did."""
    import vafc
    import vafc_dist as D
    size = os.path.getsize(path)
    rows, wsyms, held = [], [], []
    try:
        for r in range(world):
            b, e = D.byte_range(size, r, world)
            if e <= b:
                rows.append((D.NO_OFFSET, D.NO_OFFSET, 0, 1, 0))
                wsyms.append(np.zeros(vafc.GZ_WSIZE, np.uint16))
                held.append(None)
                continue
            if hold:
                info, w, h = vafc.gz_share_open(path, b, e, threads=threads, chunk_bytes=chunk, hold_bytes=hold)
            else:
                (info, w), h = vafc.gz_share_scan(path, b, e, threads=threads, chunk_bytes=chunk), None
            rows.append((info["start_bit"], info["end_bit"], info["text_len"], info["ok"], info["ended"]))
            wsyms.append(w)
            held.append(h)
        if held_out is not None:
            held_out += [h is not None for h in held]
        if not D.gz_shares_chain(rows):
            return False, None, None, None
        wins = D.gz_windows(rows, wsyms)
        ranges, crcs, reads = [], [], []
        for r in range(world):
            if rows[r][0] == D.NO_OFFSET:
                ranges.append((D.EMPTY_RANGE, D.EMPTY_RANGE, 0, 0))
                continue
            if held[r] is not None:
                st, ri, cr, rd = vafc.scan_gz_share_held(held[r], k, r == 0, wins[r], rows[r][2], block, threads,
                                                         with_reads=True)
            else:
                st, ri, cr, rd = vafc.scan_gz_share(path, k, r == 0, rows[r][0], wins[r], rows[r][2], block,
                                                    threads, with_reads=True)
            ranges.append((ri.first, ri.next, ri.errs, ri.stopped))
            crcs.append(cr)
            reads += rd
        return True, ranges, crcs, reads
    finally:
        for h in held:
            if h is not None:
                h.close()


def _share_file(p, text, shape):
    if shape == "one":
        data = _member(text, level=1)
    elif shape == "pigz":      # sync-flushed pieces: empty stored blocks between them
        c = zlib.compressobj(1, zlib.DEFLATED, -15)
        body = b"".join(c.compress(text[a:a + 60000]) + c.flush(zlib.Z_SYNC_FLUSH)
                        for a in range(0, len(text), 60000)) + c.flush()
        data = b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x04\x03" + body + struct.pack("<II", zlib.crc32(text), len(text))
    elif shape == "multi":     # members cut inside records
        cut = [0, len(text) // 3 + 11, 2 * len(text) // 3 + 5, len(text)]
        data = b"".join(_member(text[a:b], level=1) for a, b in zip(cut, cut[1:]))
    else:                      # fixed-Huffman blocks only: no later share can start blind,
        data = _member(text, level=1, strategy=zlib.Z_FIXED)   # so share 0 decodes to the end
    with open(p, "wb") as f:
        f.write(data)


@pytest.mark.parametrize("shape", ["one", "pigz", "multi", "fixed_blocks"])
@pytest.mark.parametrize("hold", [1 << 30, 1, 4 << 20])
@pytest.mark.parametrize("world", [2, 3])
def test_gzip_held_shares_reproduce_the_stream(tmp_path, text, shape, hold, world):
    """The single-pass shares (vc_gz_share_open + vc_scan_gz_share_held): a
    share that fits the budget is counted from the scan's own decoded chunks
    (and zlib past its end for the last record), one that does not is
    decoded again -- the reads, ranges and CRC chain are the two-pass ones."""
    import vafc
    import vafc_dist as D
    p = str(tmp_path / "h.fq.gz")
    _share_file(p, text, shape)
    kept = []
    chained, ranges, crcs, reads = _shares(p, world, hold=hold, held_out=kept)
    assert chained
    if hold == 1:
        assert not any(kept)
    elif hold == 4 << 20:      # a chunk's buffers take 3 MiB at least: the budget runs out mid-scan
        assert not all(kept)
    elif shape != "fixed_blocks":
        assert all(kept)
    st0, r0 = vafc.scan_file(p, 5, 100, with_reads=True)
    assert reads == r0
    assert D.chain_holds(ranges)
    assert D.gz_crc_chain(crcs, vafc.gz_crc32_combine)


def test_gzip_held_share_closed_unused(tmp_path, text):
    """A held share closed without a count (another rank's share failed):
    the decoder's threads and buffers go with it."""
    import vafc
    p = str(tmp_path / "u.fq.gz")
    _share_file(p, text, "one")
    size = os.path.getsize(p)
    for _ in range(3):
        info, w, h = vafc.gz_share_open(p, size // 2, size, threads=3, chunk_bytes=16 << 10, hold_bytes=1 << 30)
        assert info["ok"] and h is not None
        h.close()
        h.close()


@pytest.mark.parametrize("shape", ["one", "pigz", "multi", "fixed_blocks"])
@pytest.mark.parametrize("world", [2, 3, 7])
def test_gzip_shares_reproduce_the_stream(tmp_path, text, shape, world):
    """Every share decoded blind, chained by its window, and counted from its
    start: the shares' reads in order are the sequential reader's, the
    ranges chain, and the members' CRC-32 checks combine across the shares."""
    import vafc
    import vafc_dist as D
    p = str(tmp_path / "s.fq.gz")
    if shape == "one":
        data = _member(text, level=1)
    elif shape == "pigz":      # sync-flushed pieces: empty stored blocks between them
        c = zlib.compressobj(1, zlib.DEFLATED, -15)
        body = b"".join(c.compress(text[a:a + 60000]) + c.flush(zlib.Z_SYNC_FLUSH)
                        for a in range(0, len(text), 60000)) + c.flush()
        data = b"\x1f\x8b\x08\x00\x00\x00\x00\x00\x04\x03" + body + struct.pack("<II", zlib.crc32(text), len(text))
    elif shape == "multi":     # members cut inside records
        cut = [0, len(text) // 3 + 11, 2 * len(text) // 3 + 5, len(text)]
        data = b"".join(_member(text[a:b], level=1) for a, b in zip(cut, cut[1:]))
    else:                      # fixed-Huffman blocks only: no later share can start blind,
        data = _member(text, level=1, strategy=zlib.Z_FIXED)   # so share 0 decodes to the end
    with open(p, "wb") as f:
        f.write(data)
    chained, ranges, crcs, reads = _shares(p, world)
    assert chained
    if shape == "fixed_blocks":
        assert all(r[0] == D.EMPTY_RANGE for r in ranges[1:])
    st0, r0 = vafc.scan_file(p, 5, 100, with_reads=True)
    assert reads == r0
    assert D.chain_holds(ranges)
    assert D.gz_crc_chain(crcs, vafc.gz_crc32_combine)


def test_gzip_shares_bad_crc_is_caught(tmp_path, text):
    """A wrong CRC-32 in a member that spans two shares: each share alone
    cannot see it; the combined check does."""
    import vafc
    import vafc_dist as D
    p = str(tmp_path / "bad.fq.gz")
    m = bytearray(_member(text, level=1))
    m[-8] ^= 0x01
    with open(p, "wb") as f:
        f.write(bytes(m))
    chained, ranges, crcs, reads = _shares(p, 3)
    assert chained and D.chain_holds(ranges)
    assert not D.gz_crc_chain(crcs, vafc.gz_crc32_combine)
    assert all(c["crc_error"] == 0 for c in crcs)
