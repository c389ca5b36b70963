"""HIP path parity (needs an MI355X): every test calls libvafc.so through its C
ABI and compares with the reference's goldens or the oracle, bit-exactly."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PRODUCT_CLI, run_cli

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "manifest.json")) as _f:
    CASE_NAMES = [c["name"] for c in json.load(_f)["cases"]]

ALPHABET = np.frombuffer(b"ACGTACGTACGTACGTACGTacgtNnUuSWDQE\x00\x01\x02\x03\x80\xc1\xd4\xff -", np.uint8)


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda", 0)


def random_reads(rng, lens):
    out = []
    for L in lens:
        if rng.integers(0, 3) == 0:
            out.append(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        else:
            out.append(ALPHABET[rng.integers(0, ALPHABET.size, L)].tobytes())
    return out


def table_from_reads(k, reads, rng, n_pat=500):
    """Keys drawn from k-mers that really occur (so there are hits), plus misses."""
    import oracle as O
    pool = np.unique(np.concatenate([O.read_kmers(k, r) for r in reads] + [np.zeros(0, np.uint64)]))
    sel = pool[rng.permutation(pool.size)[: min(pool.size, n_pat)]] if pool.size else pool
    mask = np.uint64((1 << (2 * k)) - 1)
    extra = rng.integers(0, 1 << 62, 200, dtype=np.uint64) & mask
    keys = np.concatenate([sel, extra]).astype(np.uint64)
    vals = (np.arange(keys.size, dtype=np.uint32) % (2 * n_pat)).astype(np.uint32)
    return keys, vals, n_pat


def gpu_counts(k, keys, vals, n_pat, reads, blocks=1, env=None):
    import vafc
    import vafc_synth as S
    old = {}
    for kk, v in (env or {}).items():
        old[kk] = os.environ.get(kk)
        os.environ[kk] = v
    try:
        m = vafc.KmerMap(k, keys, vals, n_pat, 0)
    finally:
        for kk, v in old.items():
            if v is None:
                os.environ.pop(kk, None)
            else:
                os.environ[kk] = v
    step = max(1, (len(reads) + blocks - 1) // blocks)
    for i in range(0, len(reads), step):
        seq, offs, lens = S.pack_reads(reads[i:i + step])
        if seq.size == 0:
            seq = np.zeros(1, np.uint8)
        m.count_block(seq, offs, lens)
    c, km = m.finish()
    m.close()
    return c, km


def oracle_counts(k, keys, vals, n_pat, reads):
    import oracle as O
    import vafc_synth as S
    orc = O.Oracle(k, keys=keys, vals=vals)
    seq, offs, lens = S.pack_reads(reads)
    if seq.size == 0:
        seq = np.zeros(1, np.uint8)
    return orc.count_reads(seq, offs, lens, n_patterns=n_pat)


# --------------------------------------------------------------------------
# the drop-in CLI on the reference's golden cases
# --------------------------------------------------------------------------

@pytest.mark.parametrize("name", CASE_NAMES)
def test_cli_matches_reference(name, manifest, synth_dir, tmp_path):
    entry = next(c for c in manifest["cases"] if c["name"] == name)
    rc, stats, data, err = run_cli(PRODUCT_CLI, entry, synth_dir, tmp_path)
    assert rc == entry["exit"], err[-2000:]
    if entry["vaf_md5"] is not None:
        assert hashlib.md5(data).hexdigest() == entry["vaf_md5"]
        for key in ("bases", "seqs", "kmers"):
            assert stats.get(key) == entry["stats"].get(key), key
    assert ("collisions detected" in err) == entry["collision_warning"]


@pytest.mark.parametrize("name", ["c1_plumbing_k21", "pe_k31", "edge_k15", "mal_gbbbg_b1"])
def test_python_mirror_matches_reference(name, manifest, synth_dir, tmp_path):
    import vafc
    from conftest import case_dir
    entry = next(c for c in manifest["cases"] if c["name"] == name)
    out = str(tmp_path / "py.vaf")
    cwd = os.getcwd()
    os.chdir(case_dir(entry, synth_dir))
    try:
        rc = vafc.main(entry["argv"] + ["-o", out])
    finally:
        os.chdir(cwd)
    assert rc == 0
    assert hashlib.md5(open(out, "rb").read()).hexdigest() == entry["vaf_md5"]


# --------------------------------------------------------------------------
# kernels vs oracle on random inputs
# --------------------------------------------------------------------------

@pytest.mark.parametrize("k", [1, 5, 15] + list(range(16, 32)))
def test_random_reads_vs_oracle(k):
    """Every k of the packed path (16..31, one kernel instantiation each) and the
    run-time-k kernel (k < 16)."""
    rng = np.random.default_rng(k)
    lens = list(rng.integers(0, 200, 3000)) + [0, 1, k - 1, k, k + 1, 15, 16, 17, 31, 32, 33, 150, 151, 1000, 5000]
    reads = random_reads(rng, lens)
    keys, vals, n_pat = table_from_reads(k, reads, rng)
    got, km = gpu_counts(k, keys, vals, n_pat, reads, blocks=3)
    want, km_want = oracle_counts(k, keys, vals, n_pat, reads)
    assert km == km_want
    assert np.array_equal(got, want)
    assert int(want.sum()) > 0


@pytest.mark.parametrize("filt", ["bloom", "flank"])
@pytest.mark.parametrize("k", [21, 22, 26, 27, 31])
def test_prefilter_modes_vs_oracle(k, filt):
    """Both LDS prefilters (VAFC_FILTER: the Bloom filter, the flank bitmap of
    vafc_common.h) count identically to the oracle, whole and long reads
    (the long-read kernel's segments start mid-read), with keys that occur."""
    rng = np.random.default_rng(500 + k)
    lens = list(rng.integers(0, 400, 2500)) + [k - 1, k, k + 1, 30, 31, 32, 33, 47, 48, 49, 150, 16384, 16400, 40000]
    reads = random_reads(rng, lens)
    keys, vals, n_pat = table_from_reads(k, reads, rng, n_pat=3000)
    got, km = gpu_counts(k, keys, vals, n_pat, reads, blocks=2, env={"VAFC_FILTER": filt})
    want, km_want = oracle_counts(k, keys, vals, n_pat, reads)
    assert km == km_want
    assert np.array_equal(got, want)
    assert int(want.sum()) > 200


@pytest.mark.parametrize("filt", ["bloom", "flank"])
@pytest.mark.parametrize("k", [16, 21, 31])
def test_tail_bytes_vs_oracle(k, filt):
    """Reads of ACGT whose last bytes (the tail chunk: len & 15 of them, every
    value 1..15, which the kernels decode with seq_nt4_table) come from the
    odd alphabet: lower case, U, N, other letters, bytes 0..3 (which map to
    themselves) and bytes >= 0x80; whole waves of tails at once."""
    rng = np.random.default_rng(900 + k)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    reads = []
    for i in range(6000):
        L = int(16 * rng.integers(1, 12) + 1 + i % 15) if i % 7 else int(rng.integers(1, 200))
        r = acgt[rng.integers(0, 4, L)]
        t = L & 15
        odd = ALPHABET[rng.integers(0, ALPHABET.size, t)]
        keep = rng.random(t) < 0.7
        r[L - t:] = np.where(keep, r[L - t:], odd)
        reads.append(r.tobytes())
    keys, vals, n_pat = table_from_reads(k, reads, rng, n_pat=3000)
    got, km = gpu_counts(k, keys, vals, n_pat, reads, blocks=2, env={"VAFC_FILTER": filt})
    want, km_want = oracle_counts(k, keys, vals, n_pat, reads)
    assert km == km_want
    assert np.array_equal(got, want)
    assert int(want.sum()) > 1000


@pytest.mark.parametrize("k", [21, 31])
def test_every_kmer_of_golden_reads_flank(k):
    """The flank bitmap forced on with a dense key set (every k-mer of the golden
    reads): a necessary-condition filter may pass more, never fewer."""
    import oracle as O
    z = np.load(os.path.join(GOLDEN, "kmers_k%d.npz" % k))
    seq, lens = z["seq"], z["lens"]
    reads, pos = [], 0
    for L in lens:
        reads.append(seq[pos:pos + int(L)].tobytes())
        pos += int(L)
    allk = np.concatenate([O.read_kmers(k, r) for r in reads])
    uniq, mult = np.unique(allk, return_counts=True)
    vals = np.arange(uniq.size, dtype=np.uint32)
    got, km = gpu_counts(k, uniq, vals, (uniq.size + 1) // 2, reads, env={"VAFC_FILTER": "flank"})
    assert km == allk.size
    assert np.array_equal(got[: uniq.size], mult.astype(np.uint32))


@pytest.mark.parametrize("k", [21, 31, 9, 16, 26])
def test_long_reads_segmented_kernel(k):
    """Reads > VC_LONG_READ (16384) take the segmented long-read kernel."""
    rng = np.random.default_rng(77 + k)
    lens = [16384, 16385, 20000, 65536 + 7, 300_000] + list(rng.integers(100, 300, 500))
    reads = random_reads(rng, lens)
    keys, vals, n_pat = table_from_reads(k, reads, rng, n_pat=2000)
    got, km = gpu_counts(k, keys, vals, n_pat, reads)
    want, km_want = oracle_counts(k, keys, vals, n_pat, reads)
    assert km == km_want
    assert np.array_equal(got, want)


@pytest.mark.parametrize("filt", [None, "bloom128"])
@pytest.mark.parametrize("k", [21, 31])
def test_long_reads_large_panel(k, filt):
    """Large tables (> 65,536 keys: second-level filter, and for k >= 21 the
    144 KiB LDS filter with 128-entry queues, VC_KV_BIG) in the segmented
    long-read kernel, whose segments start mid-read (HAS_LO); VAFC_FILTER=
    bloom128 keeps the 128 KiB filter."""
    rng = np.random.default_rng(3100 + k)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    lens = [16385, 65543, 300_000] + list(rng.integers(100, 300, 1200))
    reads = [acgt[rng.integers(0, 4, int(L))].tobytes() for L in lens]
    keys, vals, n_pat = table_from_reads(k, reads, rng, n_pat=70_000)
    assert keys.size > 65_536
    env = {"VAFC_FILTER": filt} if filt else None
    got, km = gpu_counts(k, keys, vals, n_pat, reads, blocks=2, env=env)
    want, km_want = oracle_counts(k, keys, vals, n_pat, reads)
    assert km == km_want
    assert np.array_equal(got, want)
    assert int(want.sum()) > 40_000


@pytest.mark.parametrize("k,n_sel", [(16, 65336), (16, 65337), (27, 65337), (31, 90000)])
def test_second_level_filter_threshold(k, n_sel):
    """Tables of > 65536 keys (VC_L2F_MIN_KEYS) also build the second-level filter;
    either side of the threshold must count identically to the oracle."""
    rng = np.random.default_rng(1000 + k + n_sel)
    reads = [np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(L))].tobytes()
             for L in rng.integers(100, 300, 1500)]
    keys, vals, n_pat = table_from_reads(k, reads, rng, n_pat=n_sel)
    assert keys.size == n_sel + 200
    got, km = gpu_counts(k, keys, vals, n_pat, reads, blocks=2)
    want, km_want = oracle_counts(k, keys, vals, n_pat, reads)
    assert km == km_want
    assert np.array_equal(got, want)
    assert int(want.sum()) > 50_000


@pytest.mark.parametrize("k", list(range(21, 32)))
def test_large_panel_kernels_every_k(k):
    """The large-panel kernels (144 KiB LDS filter, strand-keyed second-level
    filter, pipelined near-full drains) for every k they are built for, on a
    read set dense in keys (about a quarter of the windows are keys): the
    drains' survivors often overflow the room kept for them, so the
    probe-at-once paths run too.  Counts equal the oracle's."""
    rng = np.random.default_rng(3000 + k)
    reads = [np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(L))].tobytes()
             for L in rng.integers(100, 300, 1500)]
    reads += random_reads(rng, list(rng.integers(0, 400, 300)))   # odd bytes, short and long reads
    keys, vals, n_pat = table_from_reads(k, reads, rng, n_pat=70_000)
    got, km = gpu_counts(k, keys, vals, n_pat, reads, blocks=2)
    want, km_want = oracle_counts(k, keys, vals, n_pat, reads)
    assert km == km_want
    assert np.array_equal(got, want)
    assert int(want.sum()) > 50_000


@pytest.mark.parametrize("k", [1, 5, 15, 16, 17, 21, 31])
def test_every_kmer_of_golden_reads(k):
    """Table = every distinct k-mer of the golden reads (whose k-mer lists are pinned
    to the reference's extract_kmers_to_buf); GPU multiplicities must match."""
    import oracle as O
    z = np.load(os.path.join(GOLDEN, "kmers_k%d.npz" % k))
    seq, lens = z["seq"], z["lens"]
    reads, pos = [], 0
    for L in lens:
        reads.append(seq[pos:pos + int(L)].tobytes())
        pos += int(L)
    allk = np.concatenate([O.read_kmers(k, r) for r in reads])
    uniq, mult = np.unique(allk, return_counts=True)
    vals = np.arange(uniq.size, dtype=np.uint32)
    n_pat = (uniq.size + 1) // 2
    got, km = gpu_counts(k, uniq, vals, n_pat, reads)
    assert km == allk.size == int(z["counts"].sum())
    assert np.array_equal(got[: uniq.size], mult.astype(np.uint32))


def test_device_decode_matches_oracle(torch_dev):
    import torch
    import vafc
    import oracle as O
    rng = np.random.default_rng(3)
    reads = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for L in list(range(0, 80)) * 4 + [150, 1000]]
    import vafc_synth as S
    seq, offs, lens = S.pack_reads(reads)
    d_seq = torch.from_numpy(seq).to(torch_dev)
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(torch_dev)
    d_lens = torch.from_numpy(lens.astype(np.int32)).to(torch_dev)
    d_codes = torch.full((seq.size,), 9, dtype=torch.uint8, device=torch_dev)
    torch.cuda.synchronize()
    vafc.debug_decode(d_seq.data_ptr(), seq.size, d_offs.data_ptr(), d_lens.data_ptr(), len(reads),
                      d_codes.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = d_codes.cpu().numpy()
    want = np.concatenate([O.decode(r) for r in reads])
    assert np.array_equal(got, want)


def test_device_generator_matches_numpy(torch_dev):
    import torch
    import vafc
    import vafc_synth as S
    panel = S.make_panel(S.synthetic_bed(500))
    win = torch.from_numpy(panel.windows().reshape(-1)).to(torch_dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(torch_dev)
    for first, n, L, f in ((0, 4000, 150, 0.3), (12_345_678, 3000, 150, 1.0), (5, 1000, 100, 0.0)):
        d_seq = torch.empty(n * L, dtype=torch.uint8, device=torch_dev)
        d_offs = torch.empty(n, dtype=torch.int64, device=torch_dev)
        d_lens = torch.empty(n, dtype=torch.int32, device=torch_dev)
        torch.cuda.synchronize()
        vafc.synth_reads(d_seq.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), first, n, L, 42, f,
                         win.data_ptr(), dos.data_ptr(), panel.n, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        want = S.gen_reads(panel, n, first=first, seed=42, f_snp=f, read_len=L)
        assert np.array_equal(d_seq.cpu().numpy().reshape(n, L), want)
        assert np.array_equal(d_offs.cpu().numpy(), np.arange(n) * L)
        assert np.all(d_lens.cpu().numpy() == L)


@pytest.mark.parametrize("k", [21, 31, 25, 13])
def test_device_resident_unaligned(torch_dev, k):
    """count_device on HBM reads at every byte misalignment; compile-time k (21, 31:
    packed streams) and run-time k (25, 13: rolling scan)."""
    import torch
    import vafc
    import vafc_synth as S
    import oracle as O
    import tempfile
    panel = S.make_panel(S.synthetic_bed(3000))
    with tempfile.TemporaryDirectory() as d:
        pat = os.path.join(d, "p.txt")
        panel.write_patterns(pat, k)
        db = vafc.load_patterns(pat)
        keys, vals, _ = db.keys(k)
        reads = S.gen_reads(panel, 20000, f_snp=0.5)
        seq, offs, lens = S.pack_reads(reads)
        want, km_want = O.Oracle(k, pattern_fn=pat).count_reads(seq, offs, lens)
    m = vafc.KmerMap(k, keys, vals, db.n, 0)
    res = []
    for mis in range(4):
        buf = torch.zeros(seq.size + 8, dtype=torch.uint8, device=torch_dev)
        buf[mis:mis + seq.size] = torch.from_numpy(seq).to(torch_dev)
        d_offs = torch.from_numpy(offs.astype(np.int64)).to(torch_dev)
        d_lens = torch.from_numpy(lens.astype(np.int32)).to(torch_dev)
        torch.cuda.synchronize()
        m.reset()
        m.count_device(buf.data_ptr() + mis, seq.size, d_offs.data_ptr(), d_lens.data_ptr(), lens.size)
        got, km = m.finish()
        assert km == km_want, mis
        assert np.array_equal(got, want), mis
        res.append(int(got.sum()))
    m.close()
    assert min(res) > 0


def test_count_file_equals_oracle_file_pass(tmp_path):
    """The product's streaming file path (pinned batches, -b blocks) on a 300k-read FASTQ."""
    import vafc
    import vafc_synth as S
    import oracle as O
    panel = S.grch38_panel()
    pat = str(tmp_path / "p.txt")
    panel.write_patterns(pat, 21)
    fq = str(tmp_path / "r.fq")
    S.write_fastq(fq, panel, 300_000, seed=7, f_snp=0.2)
    db = vafc.load_patterns(pat)
    m = vafc.create_combined_kmer_map(db, 21)
    st = m.count_file(fq, 10_000_000, 4)
    got, km = m.finish()
    orc = O.Oracle(21, pattern_fn=pat)
    want = np.zeros(2 * orc.n_patterns + 2, np.uint32)
    rc, bases, seqs, km_want = orc.count_file(fq, 10_000_000, want)
    assert (st.bases, st.seqs) == (bases, seqs)
    assert km == km_want
    assert np.array_equal(got, want[: 2 * orc.n_patterns])


@pytest.mark.parametrize("world,piece", [(3, 1 << 20), (5, 4_000_037), (2, 0)])
def test_count_file_ranges_chain_to_whole_file(world, piece, tmp_path, monkeypatch):
    """vc_count_file_range over a 120k-read FASTQ (~45 MB) cut into `world`
    byte ranges the way vafc_dist.byte_range cuts it (cuts fall inside
    records), every range counted into ONE map on the device, many reader
    pieces per range (piece 0: the default size): the ranges chain (each
    begins where the previous one ended, no truncated record), their bases and
    reads add up to the oracle's whole-file pass, and the counts and k-mer
    tally equal it bit for bit."""
    import vafc
    import vafc_dist as D
    import vafc_synth as S
    import oracle as O
    panel = S.grch38_panel()
    pat = str(tmp_path / "p.txt")
    panel.write_patterns(pat, 21)
    fq = str(tmp_path / "r.fq")
    S.write_fastq(fq, panel, 120_000, seed=11 + world, f_snp=0.2)
    size = os.path.getsize(fq)
    monkeypatch.setenv("VAFC_INGEST_MIN", "0")
    if piece:
        monkeypatch.setenv("VAFC_INGEST_PIECE", str(piece))
    db = vafc.load_patterns(pat)
    m = vafc.create_combined_kmer_map(db, 21)
    infos, bases, seqs = [], 0, 0
    for r in range(world):
        b, e = D.byte_range(size, r, world)
        st, ri = m.count_file_range(fq, b, e, 10_000_000, 4)
        assert ri.whole == 0 and ri.errs == 0 and ri.stopped == (r == world - 1)
        infos.append((ri.first, ri.next, ri.errs, ri.stopped))
        bases += st.bases
        seqs += st.seqs
    assert D.chain_holds(infos), infos
    assert infos[-1][1] == D.NO_OFFSET
    got, km = m.finish()
    m.close()
    orc = O.Oracle(21, pattern_fn=pat)
    want = np.zeros(2 * orc.n_patterns + 2, np.uint32)
    rc, wb, ws, km_want = orc.count_file(fq, 10_000_000, want)
    assert rc == 0 and (bases, seqs) == (wb, ws) == (bases, 120_000)
    assert km == km_want
    assert np.array_equal(got, want[: 2 * orc.n_patterns])
    assert int(got.sum()) > 0


@pytest.mark.parametrize("seed", range(4))
def test_count_file_parallel_reader_on_fuzzed_input(seed, tmp_path, monkeypatch):
    """vc_count_file's parallel reader (forced onto a small file with tiny
    pieces) on malformed FASTQ/FASTA: counts, bases and k-mers equal the
    oracle's whole-file pass.  Odd seeds reserve the reader's buffers up
    front (vc_reserve_file_ingest), even seeds let the workers allocate each
    slot on first use; seed 3 also runs with four slots for three workers,
    seed 2 reads the file through a read-only mapping (VAFC_MMAP=1)."""
    import re
    import vafc
    import oracle as O
    from test_reader import _fuzz_file
    rng = np.random.default_rng(900 + seed)
    fq = str(tmp_path / "fuzz.fq")
    _fuzz_file(fq, rng, 3000)
    text = open(fq, "rb").read()
    runs = [m.group(0).decode() for m in re.finditer(rb"[ACGT]{9,}", text)][:60]
    pat = str(tmp_path / "p.txt")
    with open(pat, "w") as f:
        for i, r in enumerate(runs):
            f.write("chr1\t%d\t%d\trs%d\tA\tC\t%s\t%s\n" % (i, i + 1, i, r[:9], r[1:10]))
    monkeypatch.setenv("VAFC_INGEST_MIN", "0")
    monkeypatch.setenv("VAFC_INGEST_PIECE", str(37 + 101 * seed))
    if seed == 3:
        monkeypatch.setenv("VAFC_INGEST_SLOTS", "4")
    if seed == 2:
        monkeypatch.setenv("VAFC_MMAP", "1")   # the mapped-file source, parsed in place
    for b in (10_000_000, 50):
        db = vafc.load_patterns(pat)
        m = vafc.create_combined_kmer_map(db, 9)
        if seed % 2:
            m.reserve_file_ingest(3)
        st = m.count_file(fq, b, 3)
        got, km = m.finish()
        orc = O.Oracle(9, pattern_fn=pat)
        want = np.zeros(2 * orc.n_patterns + 2, np.uint32)
        rc, bases, seqs, km_want = orc.count_file(fq, b, want)
        assert (st.bases, st.seqs) == (bases, seqs)
        assert km == km_want
        assert np.array_equal(got, want[: 2 * orc.n_patterns])
        assert int(want.sum()) > 0
        m.close()


def test_large_panel_c5_shape():
    """C5 shape: a 200k-SNP panel (~400k keys, saturated LDS prefilter)."""
    import vafc
    import vafc_synth as S
    import oracle as O
    import tempfile
    panel = S.make_panel(S.synthetic_bed(200_000))
    with tempfile.TemporaryDirectory() as d:
        pat = os.path.join(d, "p.txt")
        panel.write_patterns(pat, 21)
        db = vafc.load_patterns(pat)
        keys, vals, coll = db.keys(21)
        reads = S.gen_reads(panel, 60_000, f_snp=0.5)
        seq, offs, lens = S.pack_reads(reads)
        want, km_want = O.Oracle(21, pattern_fn=pat).count_reads(seq, offs, lens)
    m = vafc.KmerMap(21, keys, vals, db.n, 0)
    m.count_block(seq, offs, lens)
    got, km = m.finish()
    assert km == km_want and np.array_equal(got, want)
    assert int(got.sum()) > 20_000


def _oracle_windows(m, orc, d_seq, d_offs, d_lens, R, L, n=1_000_000):
    """Full-size parity past the prefix (the per-read loop being replaced is
    vaf-counter.c:349-427): windows of n reads counted in place -- the whole
    HBM buffer as the read bytes, the offsets and lengths from read j on, so
    the kernel addresses the reads by their absolute byte offsets -- against
    the oracle on the same reads copied out.  The windows: the one straddling
    byte offset 2^32, one in the middle (not aligned to anything), the last n
    reads (offsets near the end, above 4 GiB for every full-size config).
    Returns the windows checked."""
    js = sorted({max(0, min(R - n, (1 << 32) // L - n // 2)), max(0, min(R - n, R // 2 + 12_345)), R - n})
    for j in js:
        m.reset()
        m.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr() + 8 * j, d_lens.data_ptr() + 4 * j, n)
        c, km = m.finish()
        seq = d_seq[j * L:(j + n) * L].cpu().numpy()
        want, km_want = orc.count_reads(seq, np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint32))
        assert km == km_want, (j, km, km_want)
        assert np.array_equal(c, want), (j, int((c != want).sum()))
    assert (R - n) * L > (1 << 32) or R * L <= (1 << 32)
    return js


FULL_SIZE = {   # BASELINE.json configs at their full size on one GPU
    "c2": (21, "grch38", 100_000_000),    # 100M reads, ~20k SNPs
    "c3": (31, "grch38", 200_000_000),    # 100M pairs = 200M reads, k = 31
    "c5": (21, "syn200k", 100_000_000),   # 200k-SNP panel, 100M reads
}


@pytest.mark.parametrize("config", sorted(FULL_SIZE))
def test_full_size_linearity_and_prefix_parity(torch_dev, config):
    """At BASELINE size (HBM-resident): count(all) == count(first half) +
    count(second half) (mod 2^32), k-mer tallies add up, and exact 1M-read
    windows -- the prefix, across byte offset 2^32, the middle, the last reads --
    match the oracle."""
    import torch
    import vafc
    import vafc_synth as S
    import oracle as O
    import tempfile
    k, panel_name, R = FULL_SIZE[config]
    panel = S.grch38_panel() if panel_name == "grch38" else S.make_panel(S.synthetic_bed(200_000))
    L = 150
    d_seq = torch.empty(R * L, dtype=torch.uint8, device=torch_dev)
    d_offs = torch.empty(R, dtype=torch.int64, device=torch_dev)
    d_lens = torch.empty(R, dtype=torch.int32, device=torch_dev)
    win = torch.from_numpy(panel.windows().reshape(-1)).to(torch_dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(torch_dev)
    torch.cuda.synchronize()
    vafc.synth_reads(d_seq.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), 0, R, L, 42, 0.01,
                     win.data_ptr(), dos.data_ptr(), panel.n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    with tempfile.TemporaryDirectory() as d:
        pat = os.path.join(d, "p.txt")
        panel.write_patterns(pat, k)
        db = vafc.load_patterns(pat)
        keys, vals, _ = db.keys(k)
        orc = O.Oracle(k, pattern_fn=pat)
    m = vafc.KmerMap(k, keys, vals, db.n, 0)

    def run(first, n):
        m.reset()
        m.count_device(d_seq.data_ptr() + first * L, n * L, d_offs.data_ptr(), d_lens.data_ptr(), n)
        return m.finish()

    all_c, all_k = run(0, R)
    h = R // 2
    a_c, a_k = run(0, h)
    # second half: offsets are absolute, so pass the offsets tail with the full base
    m.reset()
    m.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr() + h * 8, d_lens.data_ptr() + h * 4, R - h)
    b_c, b_k = m.finish()
    assert all_k == a_k + b_k
    assert np.array_equal(all_c, (a_c.astype(np.uint64) + b_c).astype(np.uint32))
    assert all_k > R * (150 - k - 10)
    assert int(all_c.astype(np.uint64).sum()) > R // 200
    n = 1_000_000
    p_c, p_k = run(0, n)
    seq = d_seq[: n * L].cpu().numpy()
    want, km_want = orc.count_reads(seq, np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint32))
    assert p_k == km_want and np.array_equal(p_c, want)
    _oracle_windows(m, orc, d_seq, d_offs, d_lens, R, L)
    m.close()


@pytest.mark.parametrize("shards", [1, 2])
def test_count_device_default_stream_order(torch_dev, shards):
    """stream = 0 is HIP's null stream, i.e. torch's default stream (the seam
    of count_fastq_kmers, vaf-counter.c:550, fed from device memory): the
    counter's outputs are zeroed and the reads generated on torch's default
    stream behind a long queue of unrelated work, then counted with stream 0
    and no host synchronisation; vc_finish (which waits on the counter's own
    stream only) must see exactly the oracle's counts.  Repeated after a
    vc_reset issued while the next reads are still being written."""
    import torch
    import vafc
    import vafc_synth as S
    import oracle as O
    import tempfile
    assert torch.cuda.current_stream().cuda_stream == 0
    panel = S.grch38_panel()
    R, L, k = 1_000_000, 150, 21
    with tempfile.TemporaryDirectory() as d:
        pat = os.path.join(d, "p.txt")
        panel.write_patterns(pat, k)
        db = vafc.load_patterns(pat)
        keys, vals, _ = db.keys(k)
        orc = O.Oracle(k, pattern_fn=pat)
    m = vafc.KmerMap(k, keys, vals, db.n, 0) if shards == 1 else vafc.KmerMap(k, keys, vals, db.n, devices=[0] * shards)
    win = torch.from_numpy(panel.windows().reshape(-1)).to(torch_dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(torch_dev)
    busy = torch.empty(1 << 30, dtype=torch.uint8, device=torch_dev)
    torch.cuda.synchronize()
    for rnd, seed in enumerate((42, 43)):
        d_seq = torch.empty(R * L, dtype=torch.uint8, device=torch_dev)
        d_offs = torch.empty(R, dtype=torch.int64, device=torch_dev)
        d_lens = torch.empty(R, dtype=torch.int32, device=torch_dev)
        for i in range(40):   # ~40 GB of unrelated writes queued ahead of the reads
            busy.fill_(i)
        vafc.synth_reads(d_seq.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), 0, R, L, seed, 0.01,
                         win.data_ptr(), dos.data_ptr(), panel.n, 0)
        if rnd:
            m.reset()
        for a in range(0, R, R // 4):   # four batches (dealt over the shards)
            m.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr() + 8 * a, d_lens.data_ptr() + 4 * a, R // 4)
        got, km = m.finish()
        seq = d_seq.cpu().numpy()
        want, km_want = orc.count_reads(seq, np.arange(R, dtype=np.uint64) * L, np.full(R, L, np.uint32))
        assert km == km_want and np.array_equal(got, want)
        assert int(want.astype(np.uint64).sum()) > 1000
    m.close()


def test_c4_full_size_sharded(torch_dev):
    """C4 at its full size on one GPU: 1B x 150 bp reads HBM-resident (162 GB of
    288).  Counted once by a single-shard counter and once through
    vc_create_multi(devices=[0, 0]) -- the two halves dealt to the two shards by
    vc_count_device, summed on the device by vc_finish -- the totals are equal
    (linearity: all = first half + second half, mod 2^32), the k-mer tallies add
    up, and exact 1M-read windows (the prefix, across 2^32, the middle, the
    last reads at 148 GB) match the oracle.  The reference counts
    every block of every file into one set of u32 counters
    (vaf-counter.c:473-477,647-650); sharding must not change them."""
    import torch
    import vafc
    import vafc_synth as S
    import oracle as O
    import tempfile
    torch.cuda.empty_cache()
    R, L, k = 1_000_000_000, 150, 21
    panel = S.grch38_panel()
    d_seq = torch.empty(R * L, dtype=torch.uint8, device=torch_dev)
    d_offs = torch.empty(R, dtype=torch.int64, device=torch_dev)
    d_lens = torch.empty(R, dtype=torch.int32, device=torch_dev)
    win = torch.from_numpy(panel.windows().reshape(-1)).to(torch_dev)
    dos = torch.from_numpy(panel.dosage.astype(np.uint8)).to(torch_dev)
    torch.cuda.synchronize()
    vafc.synth_reads(d_seq.data_ptr(), d_offs.data_ptr(), d_lens.data_ptr(), 0, R, L, 42, 0.01,
                     win.data_ptr(), dos.data_ptr(), panel.n, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    with tempfile.TemporaryDirectory() as d:
        pat = os.path.join(d, "p.txt")
        panel.write_patterns(pat, k)
        db = vafc.load_patterns(pat)
        keys, vals, _ = db.keys(k)
        orc = O.Oracle(k, pattern_fn=pat)
    one = vafc.KmerMap(k, keys, vals, db.n, 0)
    one.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr(), d_lens.data_ptr(), R)
    all_c, all_k = one.finish()
    two = vafc.KmerMap(k, keys, vals, db.n, devices=[0, 0])
    h = R // 2
    two.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr(), d_lens.data_ptr(), h)
    two.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr() + 8 * h, d_lens.data_ptr() + 4 * h, R - h)
    assert [b for _, b in two.shards()] == [1, 1]
    sh_c, sh_k = two.finish()
    assert sh_k == all_k and np.array_equal(sh_c, all_c)
    # the halves on their own add up to the whole
    one.reset()
    one.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr(), d_lens.data_ptr(), h)
    a_c, a_k = one.finish()
    one.reset()
    one.count_device(d_seq.data_ptr(), R * L, d_offs.data_ptr() + 8 * h, d_lens.data_ptr() + 4 * h, R - h)
    b_c, b_k = one.finish()
    assert all_k == a_k + b_k
    assert np.array_equal(all_c, (a_c.astype(np.uint64) + b_c).astype(np.uint32))
    assert all_k > R * (L - k - 10)
    assert int(all_c.astype(np.uint64).sum()) > R // 200
    n = 1_000_000
    one.reset()
    one.count_device(d_seq.data_ptr(), n * L, d_offs.data_ptr(), d_lens.data_ptr(), n)
    p_c, p_k = one.finish()
    seq = d_seq[: n * L].cpu().numpy()
    want, km_want = orc.count_reads(seq, np.arange(n, dtype=np.uint64) * L, np.full(n, L, np.uint32))
    assert p_k == km_want and np.array_equal(p_c, want)
    _oracle_windows(one, orc, d_seq, d_offs, d_lens, R, L)
    one.close()
    two.close()
    del d_seq, d_offs, d_lens
    torch.cuda.empty_cache()


def test_short_reads_whole_wave(torch_dev):
    """Waves whose reads all fit in one 16-base chunk (lengths 0..16, below k):
    the quad scan's peeled chunk 0 is the whole span; nothing is counted
    twice, and mixed waves with longer reads still match the oracle."""
    rng = np.random.default_rng(44)
    for k in (21, 31):
        short = random_reads(rng, list(rng.integers(0, 17, 4096)))
        mixed = random_reads(rng, list(rng.integers(0, 17, 2000)) + [150] * 64 + list(rng.integers(0, 40, 2000)))
        for reads in (short, mixed):
            keys, vals, n_pat = table_from_reads(k, reads + random_reads(rng, [200] * 20), rng, n_pat=300)
            want, km_want = oracle_counts(k, keys, vals, n_pat, reads)
            got, km = gpu_counts(k, keys, vals, n_pat, reads)
            assert km == km_want and np.array_equal(got, want)


def test_bound_outputs_accumulate_and_wrap(torch_dev):
    """Counts bound to a caller buffer accumulate modulo 2^32 (uint32 semantics)."""
    import torch
    import vafc
    import vafc_synth as S
    rng = np.random.default_rng(5)
    reads = random_reads(rng, [150] * 2000)
    keys, vals, n_pat = table_from_reads(21, reads, rng, n_pat=100)
    want, km_want = oracle_counts(21, keys, vals, n_pat, reads)
    m = vafc.KmerMap(21, keys, vals, n_pat, 0)
    start = np.full(2 * n_pat, 0xFFFFFFF0, np.uint32)
    t = torch.from_numpy(start.view(np.int32).copy()).to(torch_dev)
    tally = torch.zeros(1, dtype=torch.int64, device=torch_dev)
    m.bind_outputs(t.data_ptr(), tally.data_ptr())
    seq, offs, lens = S.pack_reads(reads)
    m.count_block(seq, offs, lens)
    m.finish()
    got = t.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, ((start.astype(np.uint64) + want) & 0xFFFFFFFF).astype(np.uint32))
    assert int(tally.item()) == km_want
    m.close()


def test_empty_inputs():
    import vafc
    m = vafc.KmerMap(21, np.zeros(0, np.uint64), np.zeros(0, np.uint32), 3, 0)
    m.count_block(np.zeros(1, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32))
    m.count_block(np.frombuffer(b"ACGTN" * 10, np.uint8), np.array([0, 10], np.uint64), np.array([5, 20], np.uint32))
    c, km = m.finish()
    assert int(c.sum()) == 0 and km == 0
    m.close()


def test_long_read_list_overflow_is_reported(torch_dev):
    """Device reads may overlap: more reads longer than 16,384 bases than the
    long-read list holds (sized from seq_bytes) must fail loudly in finish(),
    never under-count silently; reset() clears the error."""
    import torch
    import vafc
    rng = np.random.default_rng(8)
    L = 20_000
    seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, L)]
    keys, vals, n_pat = table_from_reads(21, [seq.tobytes()], rng, n_pat=50)
    m = vafc.KmerMap(21, keys, vals, n_pat, 0)
    d_seq = torch.from_numpy(seq.copy()).to(torch_dev)
    n = 70_000   # reads on the same bytes; the list holds max(2^30 // 16385 + 1, seq_bytes // 16385 + 1) = 65,537
    d_offs = torch.zeros(n, dtype=torch.int64, device=torch_dev)
    d_lens = torch.full((n,), L, dtype=torch.int32, device=torch_dev)
    torch.cuda.synchronize()
    m.count_device(d_seq.data_ptr(), L, d_offs.data_ptr(), d_lens.data_ptr(), n)
    with pytest.raises(vafc.VafcError):
        m.finish()
    m.reset()
    m.count_device(d_seq.data_ptr(), L, d_offs.data_ptr(), d_lens.data_ptr(), 1)
    c, km = m.finish()
    want, km_want = oracle_counts(21, keys, vals, n_pat, [seq.tobytes()])
    assert km == km_want and np.array_equal(c, want)
    m.close()


# --------------------------------------------------------------------------
# the reference's own main() bound to libvafc.so
# --------------------------------------------------------------------------

BIND_CLI = os.path.join(os.path.dirname(PRODUCT_CLI), "..", "..", "oracle", "_ref", "vaf-counter-vafc")


@pytest.mark.parametrize("name", CASE_NAMES)
def test_reference_main_bound_to_libvafc(name, manifest, synth_dir, tmp_path):
    """oracle/_ref/vaf-counter-vafc is /root/reference/vaf-counter.c patched
    exactly as INTEGRATION.md §2 shows (oracle/bind_reference.py): its loader,
    map and writer, with count_fastq_kmers replaced by vc_count_file.  Every
    golden case gives the reference's .vaf, -v tallies and exit code."""
    assert os.path.exists(BIND_CLI), "oracle/_ref/vaf-counter-vafc not built (make -C oracle)"
    entry = next(c for c in manifest["cases"] if c["name"] == name)
    rc, stats, data, err = run_cli(BIND_CLI, entry, synth_dir, tmp_path)
    assert rc == entry["exit"], err[-2000:]
    if entry["vaf_md5"] is not None:
        assert hashlib.md5(data).hexdigest() == entry["vaf_md5"]
        for key in ("bases", "seqs", "kmers"):
            assert stats.get(key) == entry["stats"].get(key), key


def test_build_id_of_the_loaded_library(torch_dev):
    """On the GPU box: the libvafc.so this process has loaded (the one every GPU
    test here runs) carries the hash of this tree's sources, and so does every
    CLI the tests run (tests/conftest.py refuses the session otherwise)."""
    import vafc
    want = vafc.tree_build_id()
    assert vafc.lib().vc_build_id().decode() == want
    vafc.check_build()
