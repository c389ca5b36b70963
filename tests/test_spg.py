"""snp-pattern-gen on the GPU: the product's genome
loader against the oracle's kseq restatement (CPU), the drop-in CLI against
the reference's golden outputs, and vc_count_candidates against the oracle's
count_candidate_kmers restatement on random genomes (GPU)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, PKG
from test_spg_oracle import SPG, SPG_CASES, run_spg

SPG_CLI = os.path.join(PKG, "lib", "snp-pattern-gen")
GENOMES = ["g1.fa", "g1.fa.gz", "g2_crlf.fa", "g3_oneline.fa"]


@pytest.mark.parametrize("fn", GENOMES)
def test_fasta_loader_matches_oracle(fn):
    import vafc
    import oracle as O
    path = os.path.join(SPG, fn)
    assert vafc.load_fasta(path) == O.fasta_records(path)


def test_fasta_loader_on_fuzzed_records(tmp_path):
    """Names, comments, FASTQ records and noise mixed in: same records."""
    import vafc
    import oracle as O
    from test_reader import _fuzz_file
    for seed in range(8):
        p = str(tmp_path / ("f%d.fa" % seed))
        _fuzz_file(p, np.random.default_rng(700 + seed), 200)
        assert vafc.load_fasta(p) == O.fasta_records(p), seed


def _plain_fasta(rng, n_rec):
    """FASTA the mapped loader takes (first byte '>', no CR, no line starting
    with '+'/'@'): ragged and empty lines, empty records, '>' inside lines,
    tabs/spaces/\\v/\\f in headers, NUL and high bytes, no final newline."""
    alpha = np.frombuffer(b"ACGTNacgtn>\x00\xc1RYSW", np.uint8)
    out = []
    for r in range(n_rec):
        head = b">" + rng.choice([b"chr%d" % r, b"c%d\tdesc x" % r, b"s%d d\x0bv" % r, b"", b"r%d\x0cff" % r])
        out.append(head + b"\n")
        for _ in range(int(rng.integers(0, 6))):
            line = alpha[rng.integers(0, len(alpha), int(rng.integers(0, 90)))].tobytes()
            if line[:1] in (b">",):
                line = b"A" + line
            out.append(line + b"\n")
    data = b"".join(out)
    return data[:-1] if rng.random() < 0.5 and data.endswith(b"\n") else data


@pytest.mark.parametrize("threads", ["1", "3", "16"])
def test_fasta_mapped_loader_matches_oracle(tmp_path, threads, monkeypatch):
    """The parallel mapped loader (plain FASTA) against the oracle's kseq
    restatement, and against the sequential reader, for thread counts that
    cut records and lines at every kind of place."""
    import vafc
    import oracle as O
    monkeypatch.setenv("VAFC_THREADS", threads)
    for seed in range(12):
        rng = np.random.default_rng(900 + seed)
        p = str(tmp_path / ("m%d.fa" % seed))
        with open(p, "wb") as f:
            f.write(_plain_fasta(rng, int(rng.integers(1, 40))))
        got = vafc.load_fasta(p)
        assert got == O.fasta_records(p), seed
        monkeypatch.setenv("VAFC_FASTA_SEQUENTIAL", "1")
        assert vafc.load_fasta(p) == got, seed
        monkeypatch.delenv("VAFC_FASTA_SEQUENTIAL")
        # the same genome gzipped (two members for odd seeds): inflated in
        # memory, then the same parallel parse
        import gzip
        with open(p, "rb") as f:
            raw = f.read()
        pz = p + ".gz"
        with open(pz, "wb") as f:
            if seed % 2:
                f.write(gzip.compress(raw[: len(raw) // 2]) + gzip.compress(raw[len(raw) // 2:]))
            else:
                f.write(gzip.compress(raw, 6))
        assert vafc.load_fasta(pz) == got, seed
    # tiny files (fewer bytes than threads) and the fallback triggers
    for i, data in enumerate([b">a\nAC", b">\n", b">x\nAC\r\nGT\n", b">x\nAC\n+\nII\n", b"AC\n>x\nGG\n",
                              b">x\nAC\n@y\nGG\n", b">a\n>b\nA\n>c"]):
        p = str(tmp_path / ("t%d.fa" % i))
        with open(p, "wb") as f:
            f.write(data)
        assert vafc.load_fasta(p) == O.fasta_records(p), data


ERROR_CASES = [c for c in SPG_CASES if c["exit"] != 0]
RUN_CASES = [c for c in SPG_CASES if c["exit"] == 0]


@pytest.mark.parametrize("case", ERROR_CASES, ids=[c["name"] for c in ERROR_CASES])
def test_cli_error_paths(case, tmp_path):
    """Usage, even k, unopenable inputs: exit code and messages (no device use)."""
    rc, err, md5 = run_spg(SPG_CLI, case, tmp_path)
    assert (rc, err, md5) == (case["exit"], case["stderr"], case["out_md5"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", RUN_CASES, ids=[c["name"] for c in RUN_CASES])
def test_cli_matches_reference(case, tmp_path):
    rc, err, md5 = run_spg(SPG_CLI, case, tmp_path)
    assert (rc, err, md5) == (case["exit"], case["stderr"], case["out_md5"])


def _oracle_counts(k, seqs, keys):
    nt4 = np.full(256, 4, np.int64)
    for i, ch in enumerate(b"ACGT"):
        nt4[ch] = nt4[ch + 32] = i
        nt4[i] = i
    nt4[ord("U")] = nt4[ord("u")] = 3
    idx = {int(x): i for i, x in enumerate(keys)}
    out = np.zeros(len(keys), np.uint32)
    mask, shift = (1 << (2 * k)) - 1, 2 * (k - 1)
    for s in seqs:
        x0 = x1 = l = 0
        for b in s:
            c = int(nt4[b])
            if c < 4:
                x0 = ((x0 << 2) | c) & mask
                x1 = (x1 >> 2) | ((3 - c) << shift)
                l += 1
                if l >= k:
                    y = min(x0, x1)
                    if y in idx:
                        out[idx[y]] += 1
            else:
                x0 = x1 = l = 0
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("k", [21, 31, 17, 11, 9, 25])
def test_count_candidates_random_genome(k):
    """Long sequences (the segmented long-read kernel), short ones, every byte
    value; keys drawn from occurring k-mers plus absent ones."""
    import vafc
    import oracle as O
    rng = np.random.default_rng(40 + k)
    alpha = np.frombuffer(b"ACGTACGTacgtNnSWDRYMuU\x00\x01\x02\x03\xc1", np.uint8)
    seqs = [np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, L)].tobytes() for L in (70_000, 40_000, 20_001)]
    seqs += [alpha[rng.integers(0, alpha.size, int(L))].tobytes() for L in rng.integers(0, 3000, 40)]
    seqs += [b"", b"A" * k, seqs[0][:16384], seqs[1][:16385]]
    pool = np.unique(np.concatenate([O.read_kmers(k, s) for s in seqs[:3]]))
    keys = np.unique(np.concatenate([pool[rng.permutation(pool.size)[:3000]],
                                     rng.integers(0, 1 << (2 * k), 500, dtype=np.uint64)]))
    canon = np.array([min(int(x), int(_rc(int(x), k))) for x in keys], np.uint64)
    keys = np.unique(canon)
    got = vafc.count_candidate_kmers(k, seqs, keys)
    want = _oracle_counts(k, seqs, keys)
    assert np.array_equal(got, want)
    assert int(want.sum()) > 1000


@pytest.mark.gpu
@pytest.mark.parametrize("k", [21, 31, 17])
def test_count_candidates_long_odd_alphabet(k):
    """Chromosomes over 16,384 bases (the segmented kernel, every lane the same
    length) with len % 16 in {0, 4, 12} and bytes that the reference's PSHUFB
    head decode accepts but seq_nt4_table rejects (S/W/D/E/Q either case,
    bytes 4..7): in seq_nt4 mode all 16 bytes of every chunk take the table
    (snp-pattern-gen.c:39-56,159-190)."""
    import vafc
    import oracle as O
    rng = np.random.default_rng(70 + k)
    odd = np.frombuffer(b"SWDEQswdeq\x04\x05\x06\x07Nn", np.uint8)
    seqs = []
    for L in (16_400, 20_004, 30_012, 65_536 + 12):
        s = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, L)].copy()
        pos = rng.integers(0, L, L // 200)
        s[pos] = odd[rng.integers(0, odd.size, pos.size)]
        seqs.append(s.tobytes())
    assert all(len(s) % 16 in (0, 4, 12) and len(s) > 16384 for s in seqs)
    # keys: canonical k-mers of the table decode, plus k-mers that occur only
    # when the odd bytes take the PSHUFB head decode (vaf-counter's quirk)
    pool = np.unique(np.concatenate([_nt4_kmers(k, s) for s in seqs]))
    head = np.unique(np.concatenate([O.read_kmers(k, s) for s in seqs]))
    fake = np.setdiff1d(head, pool)
    assert fake.size > 500
    keys = np.unique(np.concatenate([pool[rng.permutation(pool.size)[:2000]], fake[rng.permutation(fake.size)[:2000]]]))
    got = vafc.count_candidate_kmers(k, seqs, keys)
    want = _oracle_counts(k, seqs, keys)
    assert np.array_equal(got, want)
    assert int(want.sum()) > 1000


def _nt4_kmers(k, s):
    """Canonical k-mers of s under seq_nt4_table (snp-pattern-gen.c:159-190)."""
    nt4 = np.full(256, 4, np.int64)
    for i, ch in enumerate(b"ACGT"):
        nt4[ch] = nt4[ch + 32] = i
        nt4[i] = i
    nt4[ord("U")] = nt4[ord("u")] = 3
    mask, shift = (1 << (2 * k)) - 1, 2 * (k - 1)
    out, x0, x1, l = [], 0, 0, 0
    for b in s:
        c = int(nt4[b])
        if c < 4:
            x0 = ((x0 << 2) | c) & mask
            x1 = (x1 >> 2) | ((3 - c) << shift)
            l += 1
            if l >= k:
                out.append(min(x0, x1))
        else:
            x0 = x1 = l = 0
    return np.array(out, np.uint64)


def _rc(x, k):
    r = 0
    for _ in range(k):
        r = (r << 2) | (3 - (x & 3))
        x >>= 2
    return r
