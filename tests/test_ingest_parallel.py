"""The parallel plain-file reader of vc_count_file (vafc_ingest.cpp) against the
sequential one (vafc_fastq.cpp, pinned to the reference by test_reader.py):
same accepted reads in the same order, same bases / sequences / blocks, for
every piece size down to a few bytes (every record boundary is then a piece
boundary, and most guesses land inside records)."""
import os

import numpy as np
import pytest

from conftest import CASES

from test_reader import READER_FILES, _fuzz_file

PLAIN = [f for f in READER_FILES if not f.endswith(".gz")]


def _same(path, k, b, threads, piece):
    import vafc
    st0, r0 = vafc.scan_file(path, k, b, with_reads=True)
    st1, r1 = vafc.scan_file_parallel(path, k, b, threads=threads, piece_bytes=piece, with_reads=True)
    assert (st1.bases, st1.seqs, st1.blocks) == (st0.bases, st0.seqs, st0.blocks), (path, k, b, threads, piece)
    assert r1 == r0, (path, k, b, threads, piece)


@pytest.mark.parametrize("fn", PLAIN)
@pytest.mark.parametrize("piece", [2, 7, 64, 1000, 1 << 20])
def test_golden_reader_files(fn, piece):
    path = os.path.join(CASES, fn)
    for k, b in ((1, 10_000_000), (5, 1), (21, 100)):
        _same(path, k, b, threads=3, piece=piece)


@pytest.mark.parametrize("seed", range(16))
def test_fuzzed_inputs(seed, tmp_path):
    """Noise lines, wrapped FASTA, bad quality lengths, CR, '@'/'+' inside
    records: -2 events end blocks, empty blocks can end a file early."""
    rng = np.random.default_rng(500 + seed)
    p = str(tmp_path / "fuzz.fq")
    _fuzz_file(p, rng, 400)
    for piece in (3, 17, 111, 4096):
        for k, b in ((5, 10_000_000), (5, 1), (12, 50), (1, 7)):
            _same(p, k, b, threads=1 + seed % 5, piece=piece)


@pytest.mark.parametrize("mmap", ["0", "1"])
@pytest.mark.parametrize("seed", range(4))
def test_fuzzed_inputs_pread_and_mapped(seed, mmap, tmp_path, monkeypatch):
    """Both plain-file sources of the parallel reader: pread into each
    worker's window (the default) and the mapped file parsed in place
    (VAFC_MMAP=1); one-line sequences are handed out as pointers into the
    window either way, copied out only when the window is refilled."""
    monkeypatch.setenv("VAFC_MMAP", mmap)
    rng = np.random.default_rng(900 + seed)
    p = str(tmp_path / "fuzz.fq")
    _fuzz_file(p, rng, 300)
    for piece in (5, 97, 4096):
        for k, b in ((5, 10_000_000), (3, 1), (12, 50)):
            _same(p, k, b, threads=2 + seed % 3, piece=piece)


@pytest.mark.parametrize("window", [1, 5, 64, 333])
def test_tiny_reader_windows(window, tmp_path, monkeypatch):
    """Workers' windows far smaller than a record: every one-line sequence
    handed out in place is copied out when its window is refilled mid-record
    (VAFC_READER_WINDOW, a test knob)."""
    monkeypatch.setenv("VAFC_READER_WINDOW", str(window))
    rng = np.random.default_rng(77 + window)
    p = str(tmp_path / "fuzz.fq")
    _fuzz_file(p, rng, 200)
    for piece in (13, 4096):
        for k, b in ((5, 10_000_000), (3, 1)):
            _same(p, k, b, threads=3, piece=piece)


def _fastq(path, rng, n, L=150, crlf=False):
    nl = b"\r\n" if crlf else b"\n"
    with open(path, "wb") as f:
        for i in range(n):
            seq = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, L)].tobytes()
            f.write(b"@r%d extra" % i + nl + seq + nl + b"+" + nl + b"I" * L + nl)


@pytest.mark.parametrize("crlf", [False, True])
def test_clean_fastq_many_pieces(tmp_path, crlf):
    """Well-formed FASTQ: every guess is right, pieces of every size."""
    rng = np.random.default_rng(7)
    p = str(tmp_path / "clean.fq")
    _fastq(p, rng, 5000, crlf=crlf)
    for piece in (100, 311, 4099, 65536):
        for threads in (1, 2, 8):
            _same(p, 21, 10_000, threads, piece)


def test_quality_lines_that_look_like_headers(tmp_path):
    """Quality strings starting with '@' followed by a '+' line: the four-line
    guess is fooled, the boundary check catches it."""
    with open(tmp_path / "q.fq", "wb") as f:
        for i in range(400):
            s = b"ACGT" * (3 + i % 5)
            q = b"@" * len(s) if i % 2 else b"+" * len(s)
            f.write(b"@h%d\n" % i + s + b"\n+\n" + q + b"\n")
    for piece in (5, 13, 50, 333):
        _same(str(tmp_path / "q.fq"), 7, 40, 4, piece)


def test_fasta_and_long_records(tmp_path):
    """FASTA (pieces guessed at '>' lines) and records longer than many pieces."""
    rng = np.random.default_rng(3)
    with open(tmp_path / "a.fa", "wb") as f:
        for i in range(60):
            L = int(rng.integers(1, 5000))
            s = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, L)].tobytes()
            f.write(b">c%d\n" % i + b"\n".join(s[j:j + 61] for j in range(0, L, 61)) + b"\n")
    for piece in (7, 100, 2000, 1 << 20):
        _same(str(tmp_path / "a.fa"), 15, 3000, 3, piece)


def test_gzip_goes_to_the_inflater(tmp_path):
    """gzip input takes the parallel inflater + the sequential block loop
    (tests/test_gzip.py checks it in depth)."""
    import gzip
    import vafc
    p = str(tmp_path / "x.fq.gz")
    with gzip.open(p, "wb") as f:
        f.write(b"@a\nACGT\n+\nIIII\n")
    st, reads = vafc.scan_file_parallel(p, 3, with_reads=True)
    assert reads == [b"ACGT"] and st.bases == 4


# --------------------------------------------------------------------------
# byte ranges (vc_scan_file_range, the reader of vc_count_file_range): one
# rank's share of a file in the torchrun driver (kmer-cnt_amd/vafc_dist.py)
# --------------------------------------------------------------------------

def _ranges(path, k, b, cuts, threads=2, piece=4096):
    """Scan [0, c1), [c1, c2), ..., [cn, end) and apply vafc_dist's chain rule."""
    import vafc
    import vafc_dist as D
    bounds = [0] + sorted(cuts) + [D.NO_OFFSET]
    infos, reads, bases, seqs = [], [], 0, 0
    for a, e in zip(bounds, bounds[1:]):
        if e <= a:
            infos.append((D.EMPTY_RANGE, D.EMPTY_RANGE, 0, 0))
            continue
        st, ri, r = vafc.scan_file_range(path, k, a, e, b, threads, piece, with_reads=True)
        assert ri.whole == 0
        infos.append((ri.first, ri.next, ri.errs, ri.stopped))
        reads += r
        bases += st.bases
        seqs += st.seqs
    return D.chain_holds(infos), infos, reads, bases, seqs


@pytest.mark.parametrize("crlf", [False, True])
@pytest.mark.parametrize("n_cuts", [1, 2, 7])
def test_ranges_of_clean_fastq_chain_and_equal_the_whole_file(tmp_path, crlf, n_cuts):
    """Well-formed FASTQ cut at arbitrary bytes (inside headers, sequences,
    '+' lines and qualities): every range finds the record where the previous
    one stopped, and the ranges' reads are the whole file's, in order."""
    import vafc
    rng = np.random.default_rng(11 + n_cuts)
    p = str(tmp_path / "clean.fq")
    _fastq(p, rng, 3000, crlf=crlf)
    st0, r0 = vafc.scan_file(p, 21, 10_000, with_reads=True)
    size = os.path.getsize(p)
    for trial in range(6):
        cuts = rng.integers(1, size, n_cuts).tolist()
        ok, infos, reads, bases, seqs = _ranges(p, 21, 10_000, cuts, piece=int(rng.integers(50, 5000)))
        assert ok, infos
        assert reads == r0 and (bases, seqs) == (st0.bases, st0.seqs)


def test_range_edges(tmp_path):
    """A range that starts past the end or inside the last record counts
    nothing (first = next = the end); an empty file; a range at offset 0 is
    the whole-file reader's prefix."""
    import vafc
    import vafc_dist as D
    rng = np.random.default_rng(5)
    p = str(tmp_path / "c.fq")
    _fastq(p, rng, 50)
    size = os.path.getsize(p)
    st, ri, reads = vafc.scan_file_range(p, 21, size + 10, D.NO_OFFSET, with_reads=True)
    assert (ri.first, ri.next, st.seqs) == (D.NO_OFFSET, D.NO_OFFSET, 0)
    st, ri, reads = vafc.scan_file_range(p, 21, size - 20, D.NO_OFFSET, with_reads=True)
    assert ri.first == D.NO_OFFSET and st.seqs == 0
    st, ri, reads = vafc.scan_file_range(p, 21, 0, 1, with_reads=True)
    assert ri.first == 0 and st.seqs == 1 and ri.next > 0 and ri.next < size
    st2, ri2, _ = vafc.scan_file_range(p, 21, 1, D.NO_OFFSET, with_reads=True)
    assert ri2.first == ri.next and st.seqs + st2.seqs == 50 and ri2.next == D.NO_OFFSET and ri2.stopped
    e = str(tmp_path / "empty.fq")
    open(e, "wb").close()
    st, ri, _ = vafc.scan_file_range(e, 21, 0, D.NO_OFFSET, with_reads=True)
    assert st.seqs == 0 and ri.first == D.NO_OFFSET


@pytest.mark.parametrize("seed", range(8))
def test_ranges_of_fuzzed_inputs_are_exact_or_refused(seed, tmp_path):
    """Malformed and odd inputs: whenever vafc_dist's chain rule accepts a
    split, its reads and tallies equal the whole file's; a split it refuses
    falls back to one whole-file range (which is vc_count_file)."""
    import vafc
    rng = np.random.default_rng(1300 + seed)
    p = str(tmp_path / "fuzz.fq")
    _fuzz_file(p, rng, 300)
    size = os.path.getsize(p)
    for k, b in ((5, 10_000_000), (5, 1), (12, 50)):
        st0, r0 = vafc.scan_file(p, k, b, with_reads=True)
        for trial in range(4):
            cuts = rng.integers(1, size, 1 + trial).tolist()
            ok, infos, reads, bases, seqs = _ranges(p, k, b, cuts, threads=1 + seed % 3,
                                                    piece=int(rng.integers(7, 700)))
            if ok:
                assert reads == r0 and (bases, seqs) == (st0.bases, st0.seqs), (k, b, cuts, infos)


def test_ranges_of_gzip_are_whole(tmp_path):
    """gzip is not split: begin 0 reads the whole file, later ranges nothing."""
    import gzip
    import vafc
    import vafc_dist as D
    p = str(tmp_path / "x.fq.gz")
    with gzip.open(p, "wb") as f:
        f.write(b"@a\nACGTACGT\n+\nIIIIIIII\n" * 10)
    st, ri, reads = vafc.scan_file_range(p, 3, 0, 5, with_reads=True)
    assert ri.whole == 1 and st.seqs == 10 and ri.next == D.NO_OFFSET
    st, ri, reads = vafc.scan_file_range(p, 3, 5, D.NO_OFFSET, with_reads=True)
    assert ri.whole == 1 and st.seqs == 0 and ri.first == D.NO_OFFSET
    assert not D.splittable(p)


def _feed_fifo(fifo, data, result):
    """Writer side of a named pipe: the whole text, then close; records an
    EPIPE (the reader went away early) instead of raising."""
    try:
        with open(fifo, "wb") as w:
            w.write(data)
        result["ok"] = True
    except BrokenPipeError:
        result["ok"] = False


@pytest.mark.parametrize("how", ["range", "parallel"])
def test_fifo_is_opened_once(tmp_path, how):
    """A named pipe is read by one open, as the reference's gzopen reads it
    (vc_count_file_range opened the path, looked at it, closed it
    and reopened it, so the writer could see its reader go away): the range
    reader and the parallel reader take it whole through the sequential
    reader, with the same reads as the regular file."""
    import threading
    import vafc
    src = os.path.join(CASES, PLAIN[0])
    data = open(src, "rb").read()
    fifo = str(tmp_path / "in.fifo")
    os.mkfifo(fifo)
    res = {}
    t = threading.Thread(target=_feed_fifo, args=(fifo, data, res))
    t.start()
    if how == "range":
        st, ri, _ = vafc.scan_file_range(fifo, 5, 0, 1 << 40, 100, threads=3, piece_bytes=64)
        assert ri.whole == 1
    else:
        st, _ = vafc.scan_file_parallel(fifo, 5, 100, threads=3, piece_bytes=64)
    t.join(timeout=60)
    assert res.get("ok") is True
    st0, _ = vafc.scan_file(src, 5, 100)
    assert (st.bases, st.seqs, st.blocks) == (st0.bases, st0.seqs, st0.blocks) and st0.seqs > 0
