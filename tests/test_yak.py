"""yak-count k-mer histogram (second program).

CPU: the restatement (oracle/yak_oracle.c) against the real reference's
outputs recorded in tests/golden/yak/manifest.json (stdout md5, last stderr
line, non-zero histogram rows, exit code).  GPU: the drop-in CLI
kmer-cnt_amd/lib/yak-count and the Python mirror against the same fixtures,
with a table small enough to force partitions, and against the oracle on
larger seeded two-file inputs whose Bloom filters produce many false
positives (the replay of yak's filters must pick exactly the same keys)."""
import ctypes as C
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG, ROOT

YAK = os.path.join(GOLDEN, "yak")
with open(os.path.join(YAK, "manifest.json")) as _f:
    YAK_CASES = json.load(_f)
YAK_ORACLE = os.path.join(ROOT, "oracle", "build", "yak-count-oracle")
YAK_CLI = os.path.join(PKG, "lib", "yak-count")


def run_yak(binary, argv, cwd=YAK, env=None):
    p = subprocess.run([binary] + argv, cwd=cwd, capture_output=True, timeout=600, env=env)
    err = p.stderr.decode()
    return p.returncode, p.stdout, err, (err.splitlines()[-1] if err else "")


def check(case, rc, out, last, err):
    assert rc == case["rc"], err
    assert hashlib.md5(out).hexdigest() == case["stdout_md5"]
    assert last == case["stderr_last"]
    if case["rc"]:
        assert err == case["stderr"]


# ---------------------------------------------------------------- CPU: oracle

@pytest.mark.parametrize("case", YAK_CASES, ids=[c["name"] for c in YAK_CASES])
def test_oracle_cli_matches_reference(case):
    rc, out, err, last = run_yak(YAK_ORACLE, case["argv"])
    check(case, rc, out, last, err)


def _opts(argv):
    o = {"-k": 31, "-p": 10, "-b": 0, "-H": 4, "-K": 10_000_000}
    files = []
    i = 0
    while i < len(argv):
        if argv[i] in o:
            o[argv[i]] = int(argv[i + 1])
            i += 2
        else:
            files.append(os.path.join(YAK, argv[i]))
            i += 1
    return o, files


@pytest.mark.parametrize("case", [c for c in YAK_CASES if c["rc"] == 0], ids=lambda c: c["name"])
def test_oracle_lib_matches_reference(case):
    L = C.CDLL(os.path.join(ROOT, "oracle", "build", "libyakoracle.so"))
    L.yko_hist.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int64, C.c_void_p,
                           C.POINTER(C.c_uint64)]
    o, files = _opts(case["argv"])
    hist = np.zeros(1024, np.uint64)
    tot = C.c_uint64()
    fn2 = files[1] if len(files) > 1 else files[0]
    assert L.yko_hist(files[0].encode(), fn2.encode(), o["-k"], o["-p"], o["-b"], o["-H"], o["-K"],
                      hist.ctypes.data, C.byref(tot)) == 0
    assert {str(i): int(hist[i]) for i in range(1, 1024) if hist[i]} == case["hist"]
    assert "%d distinct" % tot.value in case["stderr_last"]


def test_fixture_exercises_the_filter():
    by = {c["name"]: c for c in YAK_CASES}
    nf = by["bf14_too_small"]["stderr_last"]
    # false positives of small filters keep singletons of file 1 that file 2 sees twice
    assert by["bf19_two_fp"]["stderr_last"] != nf and by["bf19_two_fp_H32"]["stderr_last"] != nf
    assert by["bf20_two_fp_H1"]["stderr_last"] != by["bf19_two_fp"]["stderr_last"]
    assert "1" not in by["bf24_one"]["hist"] and "1" in by["nobf_k21"]["hist"]


def test_cli_usage_without_gpu():
    rc, out, err, last = run_yak(YAK_CLI, [])
    assert rc == 1 and out == b"" and err.startswith("Usage: yak-count")
    rc, out, err, last = run_yak(YAK_CLI, ["-p", "9", "r1.fq"])
    assert rc == 1 and err == "ERROR: -p should be at least 10\n"


# ---------------------------------------------------------------- GPU: product

@pytest.mark.gpu
@pytest.mark.parametrize("case", YAK_CASES, ids=[c["name"] for c in YAK_CASES])
def test_cli_matches_reference(case):
    rc, out, err, last = run_yak(YAK_CLI, case["argv"])
    check(case, rc, out, last, err)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["nobf_k21", "bf19_two_fp", "bf24_one", "bf19_two_fp_H32"])
def test_cli_small_table_partitions(name):
    case = next(c for c in YAK_CASES if c["name"] == name)
    rc, out, err, last = run_yak(YAK_CLI, case["argv"], env=dict(os.environ, VAFC_KC_SLOTS="4096"))
    check(case, rc, out, last, err)


def _write_reads(path, seed, n, genome, L=150):
    rng = np.random.default_rng(seed)
    comp = np.zeros(256, np.uint8)
    for a, b in zip(b"ACGTN", b"TGCAN"):
        comp[a] = b
    st = rng.integers(0, genome.size - L + 1, n)
    r = genome[st[:, None] + np.arange(L)[None, :]]
    rev = rng.random(n) < 0.5
    r[rev] = comp[r[rev][:, ::-1]]
    u = rng.random(r.shape)
    sub = u < 0.01
    r[sub] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(sub.sum()))]
    r[(u >= 0.01) & (u < 0.011)] = ord("N")
    with open(path, "wb") as f:
        for i in range(n):
            f.write(b"@r%d\n%s\n+\n%s\n" % (i, r[i].tobytes(), b"I" * L))


@pytest.mark.gpu
@pytest.mark.parametrize("opts", [["-k", "21", "-b", "20"], ["-k", "31", "-b", "22", "-H", "2"],
                                  ["-k", "25", "-b", "21", "-p", "11", "-K", "100000"], ["-k", "17"],
                                  ["-k", "21", "-b", "23"]])
def test_cli_matches_oracle_large(opts, tmp_path):
    rng = np.random.default_rng(5)
    genome = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 300_000)]
    _write_reads(tmp_path / "a.fq", 1, 40_000, genome)
    _write_reads(tmp_path / "b.fq", 2, 40_000, genome)
    argv = opts + ["a.fq", "b.fq"]
    want = run_yak(YAK_ORACLE, argv, cwd=tmp_path)
    got = run_yak(YAK_CLI, argv, cwd=tmp_path)
    assert want[0] == 0 and got[0] == 0, got[2]
    assert got[1] == want[1]
    assert got[3] == want[3]


@pytest.mark.gpu
def test_python_mirror_matches_cli(capsys):
    import vafc
    case = next(c for c in YAK_CASES if c["name"] == "bf19_two_fp")
    assert vafc.yak_main(["-k", "21", "-b", "19", os.path.join(YAK, "r1.fq"), os.path.join(YAK, "r2.fq")]) == 0
    cap = capsys.readouterr()
    assert hashlib.md5(cap.out.encode()).hexdigest() == case["stdout_md5"]
    assert cap.err.splitlines()[-1] == case["stderr_last"]
