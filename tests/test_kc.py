"""kc-c4 k-mer histogram.

CPU: the restatement (oracle/kc_oracle.c) against the real reference's outputs
recorded in tests/golden/kc/manifest.json (stdout md5, non-zero histogram rows,
stderr, exit code).  GPU: the drop-in CLI kmer-cnt_amd/lib/kc-c4 and the
KmerHistogram mirror (vc_kc_* in libvafc.so) against the same fixtures, and
against the oracle on larger seeded inputs (ragged lengths, long records,
partitions, a table too small)."""
import ctypes as C
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG, ROOT

KC = os.path.join(GOLDEN, "kc")
with open(os.path.join(KC, "manifest.json")) as _f:
    KC_CASES = json.load(_f)
KC_ORACLE = os.path.join(ROOT, "oracle", "build", "kc-c4-oracle")
KC_CLI = os.path.join(PKG, "lib", "kc-c4")


def run_kc(binary, case, env=None):
    p = subprocess.run([binary] + case["argv"], cwd=KC, capture_output=True, timeout=300, env=env)
    return p.returncode, p.stdout, p.stderr.decode()


def hist_rows(stdout: bytes):
    out = {}
    for line in stdout.decode().splitlines():
        i, c = line.split("\t")
        if int(c):
            out[i] = int(c)
    return out


def oracle_lib():
    L = C.CDLL(os.path.join(ROOT, "oracle", "build", "libkcoracle.so"))
    P = C.c_void_p
    L.kco_hist_file.argtypes = [C.c_char_p, C.c_int, C.c_int, P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.kco_hist_reads.argtypes = [C.c_int, P, P, P, C.c_uint64, P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    return L


def oracle_reads(k, seq, offs, lens):
    L = oracle_lib()
    hist = np.zeros(256, np.uint64)
    d, km = C.c_uint64(), C.c_uint64()
    seq = np.ascontiguousarray(seq, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    L.kco_hist_reads(k, seq.ctypes.data, offs.ctypes.data, lens.ctypes.data, lens.size, hist.ctypes.data,
                     C.byref(d), C.byref(km))
    return hist, d.value, km.value


# ---------------------------------------------------------------- CPU: oracle

@pytest.mark.parametrize("case", KC_CASES, ids=[c["name"] for c in KC_CASES])
def test_oracle_cli_matches_reference(case):
    rc, out, err = run_kc(KC_ORACLE, case)
    assert rc == case["rc"]
    assert hashlib.md5(out).hexdigest() == case["stdout_md5"]
    if case["rc"]:
        assert err == case["stderr"]


@pytest.mark.parametrize("case", [c for c in KC_CASES if c["rc"] == 0 and "-p" not in c["argv"]],
                         ids=lambda c: c["name"])
def test_oracle_lib_matches_reference(case):
    argv = case["argv"]
    k = int(argv[argv.index("-k") + 1]) if "-k" in argv else 31
    b = int(argv[argv.index("-b") + 1]) if "-b" in argv else 10_000_000
    hist = np.zeros(256, np.uint64)
    d, km = C.c_uint64(), C.c_uint64()
    assert oracle_lib().kco_hist_file(os.path.join(KC, argv[-1]).encode(), k, b, hist.ctypes.data,
                                      C.byref(d), C.byref(km)) == 0
    assert {str(i): int(hist[i]) for i in range(1, 256) if hist[i]} == case["hist"]
    assert d.value == int(hist[1:].sum())


def test_fixture_exercises_saturation_and_blocks():
    by = {c["name"]: c for c in KC_CASES}
    assert "255" in by["weird_k21"]["hist"]                 # poly-A beyond 255 (and 1023)
    assert len(by["cov_k21"]["hist"]) > 100                 # counts spread over 1..255
    assert by["badqual_k21"]["hist"] != by["badqual_b1_k21"]["hist"]   # -2 ends blocks early
    assert by["empty_k21"]["hist"] == {} and by["empty_k21"]["stdout_lines"] == 255


def test_cli_usage_without_gpu():
    rc, out, err = run_kc(KC_CLI, {"argv": []})
    assert rc == 1 and out == b"" and err.startswith("Usage: kc-c4")
    rc, out, err = run_kc(KC_CLI, {"argv": ["-p", "8", "cov.fq"]})
    assert rc == 1 and err == "ERROR: -p should be at least 10\n"


# ---------------------------------------------------------------- GPU: product

@pytest.mark.gpu
@pytest.mark.parametrize("case", KC_CASES, ids=[c["name"] for c in KC_CASES])
def test_cli_matches_reference(case):
    rc, out, err = run_kc(KC_CLI, case)
    assert rc == case["rc"], err
    assert hashlib.md5(out).hexdigest() == case["stdout_md5"]
    if case["rc"]:
        assert err == case["stderr"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cov_k21", "long_k21", "weird_k5"])
def test_cli_small_table_partitions(name):
    """A table far smaller than the distinct k-mers: counted in hash slices."""
    case = next(c for c in KC_CASES if c["name"] == name)
    env = dict(os.environ, VAFC_KC_SLOTS="1024")
    rc, out, err = run_kc(KC_CLI, case, env=env)
    assert rc == 0, err
    assert hashlib.md5(out).hexdigest() == case["stdout_md5"]


def _random_reads(seed, n, genome_len=40_000, long_every=0):
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    g = acgt[rng.integers(0, 4, genome_len)]
    lens = rng.integers(1, 301, n).astype(np.uint32)
    if long_every:
        lens[::long_every] = rng.integers(4000, 20000, lens[::long_every].size)
    parts = []
    for L in lens:
        s = int(rng.integers(0, genome_len - min(int(L), genome_len) + 1))
        r = g[s:s + int(L)].copy()
        if r.size < L:
            r = np.concatenate([r, acgt[rng.integers(0, 4, int(L) - r.size)]])
        m = rng.random(r.size)
        r[m < 0.005] = ord("N")
        r[(m >= 0.005) & (m < 0.01)] = ord("a")
        parts.append(r)
    seq = np.concatenate(parts)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64)
    return seq, offs, lens


@pytest.mark.gpu
@pytest.mark.parametrize("k,long_every", [(21, 0), (31, 0), (13, 0), (17, 97), (1, 0), (32 - 1, 53)])
def test_device_histogram_matches_oracle(k, long_every):
    import vafc
    seq, offs, lens = _random_reads(100 + k, 60_000, long_every=long_every)
    want, wd, wk = oracle_reads(k, seq, offs, lens)
    h = vafc.KmerHistogram(k, 1 << 22)
    try:
        h.count_block(seq, offs, lens)
        h.finish()
        got, gd, gk = h.histogram()
    finally:
        h.close()
    assert gk == wk and gd == wd
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_partitions_add_up_and_full_is_reported():
    import vafc
    seq, offs, lens = _random_reads(7, 20_000)
    want, wd, wk = oracle_reads(21, seq, offs, lens)
    h = vafc.KmerHistogram(21, 1 << 21)
    try:
        total, dsum = np.zeros(256, np.uint64), 0
        for part in range(3):
            h.set_partition(3, part)
            h.count_block(seq, offs, lens)
            h.finish()
            hist, d, km = h.histogram()
            assert km == wk
            total += hist
            dsum += d
        assert np.array_equal(total, want) and dsum == wd
    finally:
        h.close()
    small = vafc.KmerHistogram(21, 1024)
    try:
        small.count_block(seq, offs, lens)
        small.finish()
        with pytest.raises(vafc.VafcError) as e:
            small.histogram()
        assert e.value.code == vafc.VC_EFULL
        small.reset()   # usable again after a reset
        n3 = int(offs[3])
        w3 = oracle_reads(21, seq[:n3], offs[:3], lens[:3])
        small.count_block(seq[:n3], offs[:3], lens[:3])
        small.finish()
        g3 = small.histogram()
        assert np.array_equal(g3[0], w3[0]) and g3[1:] == w3[1:]
    finally:
        small.close()


@pytest.mark.gpu
def test_python_mirror_matches_cli(capsys):
    import vafc
    case = next(c for c in KC_CASES if c["name"] == "cov_gz_k21")
    assert vafc.kc_main(["-k", "21", os.path.join(KC, "cov.fq.gz")]) == 0
    out = capsys.readouterr().out.encode()
    assert hashlib.md5(out).hexdigest() == case["stdout_md5"]
