"""The product's FASTA/FASTQ reader + block loop (host side of vc_count_file)
against the oracle's literal kseq restatement, the golden stats, and -- on
fuzzed inputs -- the real reference binary."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import CASES, REF_CLI, ORACLE_CLI, case_dir

READER_FILES = ["edge.fq", "edge_crlf.fq", "edge.fq.gz", "multiline.fq", "truncated.fq", "empty.fq",
                "mal_gbbg.fq", "mal_gbbbg.fq", "mal_bbg.fq", "mal_bbbg.fq", "mal_gbbbgbbbg.fq", "mal_bg.fq",
                "mal_g.fq"]


@pytest.mark.parametrize("fn", READER_FILES)
def test_record_codes_match_oracle(fn):
    import vafc
    import oracle as O
    path = os.path.join(CASES, fn)
    assert np.array_equal(vafc.scan_records(path), O.scan_records(path))


def test_block_loop_stats_match_golden(manifest, synth_dir):
    """bases / sequences of every single-file CLI case, via the host-only scan."""
    import vafc
    n = 0
    for e in manifest["cases"]:
        if e["exit"] != 0 or not e["stats"]:
            continue
        argv = e["argv"]
        k = int(argv[argv.index("-k") + 1]) if "-k" in argv else 21
        b = int(argv[argv.index("-b") + 1]) if "-b" in argv else 10_000_000
        files = [a for a in argv if a.endswith((".fq", ".gz")) and not a.startswith("-")]
        bases = seqs = 0
        for f in files:
            p = os.path.join(case_dir(e, synth_dir), f)
            if not os.path.exists(p):
                continue
            st, _ = vafc.scan_file(p, k, b)
            bases += st.bases
            seqs += st.seqs
        assert (bases, seqs) == (e["stats"]["bases"], e["stats"]["seqs"]), e["name"]
        n += 1
    assert n >= 30


def _fuzz_file(path, rng, n_records):
    """FASTQ/FASTA-ish text with every parser corner mixed in."""
    out = bytearray()
    alphabet = b"ACGTACGTACGTNacgtuU@>+\r\n \t"
    for _ in range(n_records):
        kind = rng.integers(0, 10)
        L = int(rng.integers(0, 60))
        seq = bytes(alphabet[i] for i in rng.integers(0, 13, L))
        if kind < 5:      # FASTQ, maybe bad quality length
            q = L + (int(rng.integers(-2, 3)) if kind == 0 else 0)
            out += b"@r x\n" + seq + b"\n+\n" + b"I" * max(q, 0) + b"\n"
        elif kind < 7:    # FASTA, wrapped
            out += b">f\n" + seq[: L // 2] + b"\n" + seq[L // 2:] + b"\n"
        else:             # noise line
            out += bytes(alphabet[i] for i in rng.integers(0, len(alphabet), int(rng.integers(0, 20))))
            if rng.integers(0, 2):
                out += b"\n"
    with open(path, "wb") as f:
        f.write(bytes(out))


@pytest.mark.parametrize("seed", range(12))
def test_fuzzed_inputs_match_oracle_reader(seed, tmp_path):
    import vafc
    import oracle as O
    rng = np.random.default_rng(seed)
    p = str(tmp_path / "fuzz.fq")
    _fuzz_file(p, rng, 300)
    assert np.array_equal(vafc.scan_records(p), O.scan_records(p))
    for k, b in ((5, 10_000_000), (5, 1), (12, 50)):
        st, reads = vafc.scan_file(p, k, b, with_reads=True)
        orc = O.Oracle(k, keys=np.zeros(0, np.uint64), vals=np.zeros(0, np.uint32))
        counts = np.zeros(2, np.uint32)
        rc, bases, seqs, km = orc.count_file(p, b, counts)
        assert (st.bases, st.seqs) == (bases, seqs), (seed, k, b)


@pytest.mark.skipif(not os.path.exists(REF_CLI), reason="reference binary not built")
@pytest.mark.parametrize("seed", range(6))
def test_fuzzed_inputs_oracle_cli_matches_reference(seed, tmp_path):
    """Fuzzed FASTQ through the real reference and the oracle CLI: same .vaf, same stats."""
    rng = np.random.default_rng(100 + seed)
    fq = str(tmp_path / "fuzz.fq")
    _fuzz_file(fq, rng, 400)
    # a pattern file whose k-mers occur in the fuzz text
    text = open(fq, "rb").read()
    import re
    runs = [m.group(0).decode() for m in re.finditer(rb"[ACGT]{9,}", text)][:30]
    pat = str(tmp_path / "p.txt")
    with open(pat, "w") as f:
        for i, r in enumerate(runs):
            f.write("chr1\t%d\t%d\trs%d\tA\tC\t%s\t%s\n" % (i, i + 1, i, r[:9], r[-9:]))
    res = []
    for binary in (REF_CLI, ORACLE_CLI):
        out = str(tmp_path / ("o_%s.vaf" % os.path.basename(binary)))
        p = subprocess.run([binary, "-v", "-k", "9", "-b", "37", "-p", pat, "-o", out, fq],
                           capture_output=True, text=True, timeout=120)
        stats = [l for l in p.stderr.splitlines() if "processed" in l or "extracted" in l]
        res.append((p.returncode, hashlib.md5(open(out, "rb").read()).hexdigest(), stats))
    assert res[0] == res[1]
