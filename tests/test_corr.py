"""correlation-matrix: depth-aware Pearson between .vaf samples + UPGMA tree
(SURVEY.md §8(f) rank 4).

CPU: the restatement (oracle/corr_oracle.c) against the real reference's
outputs recorded in tests/golden/corr/manifest.json (.corr/.tree content,
stderr, exit code); the product's host side (vc_vafset loader, .corr writer,
tree) on the same cases, fed with correlations from a sequential Python
statement of the reference's pair formula.  GPU: the drop-in CLI
kmer-cnt_amd/lib/correlation-matrix and the VafSamples mirror against the same
fixtures, and against the oracle on larger random sample sets (ragged row
counts, depth-0 rows, tile edges, many samples)."""
import math
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, PKG, ROOT

sys.path.insert(0, GOLDEN)
import make_golden_corr as MG  # noqa: E402

CORR = os.path.join(GOLDEN, "corr")
with open(os.path.join(CORR, "manifest.json")) as _f:
    import json
    CASES = json.load(_f)
ORACLE = os.path.join(ROOT, "oracle", "build", "correlation-matrix-oracle")
CLI = os.path.join(PKG, "lib", "correlation-matrix")


@pytest.fixture(scope="module")
def work(tmp_path_factory):
    """A private copy of the fixture inputs (+ the generated 100,001-row file)."""
    d = str(tmp_path_factory.mktemp("corr"))
    for sub in ("s", "e", "t", "m"):
        shutil.copytree(os.path.join(CORR, sub), os.path.join(d, sub))
    os.makedirs(os.path.join(d, "_big"))
    with open(os.path.join(d, "_big", "big.vaf"), "w") as f:
        f.write(MG.big_vaf())
    return d


def run(binary, case, cwd):
    return MG.run_case(binary, case["argv"], cwd)


def check(case, got):
    rc, err, files = got
    assert rc == case["rc"]
    assert err == case["stderr"]
    assert files == case["files"]


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_reference(name, work):
    check(CASES[name], run(ORACLE, CASES[name], work))


# --- host side of the product, no GPU ----------------------------------------

def py_pair(a, b, n, min_snps, min_depth):
    """correlation-matrix.c:94-143 in Python floats (IEEE doubles, same order)."""
    ok = [a[1][i] >= min_depth and b[1][i] >= min_depth for i in range(n)]
    cnt = sum(ok)
    if cnt < min_snps:
        return 0.0
    sx = sy = 0.0
    for i in range(n):
        if ok[i]:
            sx += a[0][i]
            sy += b[0][i]
    mx, my = (sx / cnt, sy / cnt) if cnt else (0.0, 0.0)   # unused when no row is valid
    sxy = sxx = syy = 0.0
    for i in range(n):
        if ok[i]:
            dx, dy = a[0][i] - mx, b[0][i] - my
            sxy += dx * dy
            sxx += dx * dx
            syy += dy * dy
    da, db = math.sqrt(sxx), math.sqrt(syy)
    if da < 1e-10 or db < 1e-10:
        return sxy / (math.sqrt(sxx * syy) + 0.00001)
    return sxy / (da * db)


def case_options(argv):
    opts = {"m": 20, "d": 1}
    presets = {"matched": (5, 10), "unmatched": (1, 20), "default": (1, 20), "strict": (10, 30)}
    it, own, mode = iter(argv), set(), None
    files, out, tree = [], None, False
    for a in it:
        if a == "-o":
            out = next(it)
        elif a == "-t":
            tree = True
        elif a in ("-m", "-d"):
            opts[a[1]] = int(next(it))
            own.add(a[1])
        elif a == "-M":
            mode = next(it)
        else:
            files.append(a)
    if mode in presets:
        if "d" not in own:
            opts["d"] = presets[mode][0]
        if "m" not in own:
            opts["m"] = presets[mode][1]
    return files, out, tree, opts["m"], opts["d"]


HOST_CASES = sorted(n for n, c in CASES.items() if c["rc"] == 0 and not n.startswith(("nan", "inf", "truncate", "messy")))


@pytest.mark.parametrize("name", HOST_CASES)
def test_host_loader_writer_tree(name, work, tmp_path):
    """vc_vafset_add + vc_corr_write + vc_corr_tree reproduce the reference files
    when given the reference's doubles (computed here in Python, same order)."""
    import vafc
    case = CASES[name]
    files, out, tree, min_snps, min_depth = case_options(case["argv"])
    S = vafc.VafSamples()
    for fn in files:
        S.load_vaf_file(os.path.join(work, fn))
    n = len(S)
    data = []
    for i in range(n):
        # re-read what the loader kept, through the oracle-independent path:
        # parse the rows as the reference's sscanf does for these well-formed files
        rows = []
        with open(os.path.join(work, files[i])) as f:
            for line in f:
                if line.startswith("#") or line.startswith("CHR"):
                    continue
                p = line.split()
                if len(p) != 9:
                    continue
                try:
                    int(p[1])
                except ValueError:
                    continue
                rows.append((float(p[8]), int(p[7])))
        rows = rows[:100000]
        assert S.n_snps(i) == len(rows)
        data.append(rows)
    width = max([len(r) for r in data] + [1])
    pad = [([r[0] for r in rows] + [0.0] * (width - len(rows)), [r[1] for r in rows] + [0] * (width - len(rows)))
           for rows in data]
    corr = np.eye(n)
    for i in range(n):
        for j in range(i + 1, n):
            corr[i, j] = corr[j, i] = py_pair(pad[i], pad[j], S.n_snps(i), min_snps, min_depth)
    os.makedirs(os.path.join(tmp_path, "o"))
    S.write_corr(corr, os.path.join(tmp_path, out))
    if tree:
        cut = out.find(".corr")
        S.build_tree(corr, os.path.join(tmp_path, out[:cut] + ".tree" if cut >= 0 else out + ".tree"))
    got = {}
    for fn in sorted(os.listdir(os.path.join(tmp_path, "o"))):
        with open(os.path.join(tmp_path, "o", fn)) as f:
            got["o/" + fn] = f.read()
    assert got == case["files"]
    S.close()


def test_loader_missing_file():
    import vafc
    S = vafc.VafSamples()
    with pytest.raises(vafc.VafcError) as e:
        S.load_vaf_file("/nonexistent/x.vaf")
    assert e.value.code == vafc.VC_EIO


def test_loader_names_and_truncation(work):
    import vafc
    S = vafc.VafSamples()
    for fn in ("t/other.vaf.vaf", "t/noext", "_big/big.vaf", "e/messy.vaf", "e/empty.vaf"):
        S.load_vaf_file(os.path.join(work, fn))
    assert [S.name(i) for i in range(len(S))] == ["other", "noext", "big", "messy", "empty"]
    assert S.n_snps(2) == 100000 and S.n_snps(4) == 0
    # malformed / split / CRLF rows: the reference's own row count
    assert "[M::main] Loaded messy: %d SNPs\n" % S.n_snps(3) in CASES["messy"]["stderr"]


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_loader_parallel_matches_sequential(work, threads):
    """vc_vafset_add_many: same samples, in file order, as one vc_vafset_add
    per file; truncation flags per file; stops at the first unopenable file
    with the ones before it added."""
    import vafc
    fns = [os.path.join(work, f) for f in ("t/other.vaf.vaf", "_big/big.vaf", "e/messy.vaf", "t/noext",
                                           "e/empty.vaf", "_big/big.vaf", "e/messy.vaf")]
    A, B = vafc.VafSamples(), vafc.VafSamples()
    for fn in fns:
        A.load_vaf_file(fn)
    assert B.load_vaf_files(fns, threads) == [False, True, False, False, False, True, False]
    assert [(A.name(i), A.n_snps(i)) for i in range(len(A))] == [(B.name(i), B.n_snps(i)) for i in range(len(B))]
    C_ = vafc.VafSamples()
    with pytest.raises(vafc.VafcError) as e:
        C_.load_vaf_files(fns[:3] + ["/nonexistent/x.vaf"] + fns[3:], threads)
    assert e.value.code == vafc.VC_EIO and len(C_) == 3
    assert [C_.name(i) for i in range(3)] == ["other", "big", "messy"]
    # nothing after the first unopenable file is opened: a FIFO there (no
    # writer) would block the call forever if it were
    fifo = os.path.join(work, "after_missing_%d.fifo" % threads)
    if not os.path.exists(fifo):
        os.mkfifo(fifo)
    D = vafc.VafSamples()
    with pytest.raises(vafc.VafcError):
        D.load_vaf_files(fns[:2] + ["/nonexistent/x.vaf", fifo] + fns[2:], threads)
    assert len(D) == 2
    # n_added may be NULL
    arr = (vafc.C.c_char_p * 1)(fns[0].encode())
    assert vafc.lib().vc_vafset_add_many(D._h, vafc.C.cast(arr, vafc.P), 1, threads, None,
                                         np.zeros(1, np.uint8).ctypes.data_as(vafc.P)) == 0
    for S in (A, B, C_, D):
        S.close()


_MANY_FILES = r"""
import os, resource, sys
sys.path.insert(0, sys.argv[1])
import vafc
vafc.lib()
resource.setrlimit(resource.RLIMIT_NOFILE, (128, resource.getrlimit(resource.RLIMIT_NOFILE)[1]))
d = sys.argv[2]
fns = [os.path.join(d, "s%04d.vaf" % i) for i in range(int(sys.argv[3]))]
S = vafc.VafSamples()
assert S.load_vaf_files(fns, int(sys.argv[4])) == [False] * len(fns)
assert [S.name(i) for i in range(len(S))] == ["s%04d" % i for i in range(len(fns))]
assert all(S.n_snps(i) == 3 for i in range(len(S)))
print("ok", len(S))
"""


@pytest.mark.parametrize("threads", [1, 8, 64])
def test_loader_more_files_than_descriptors(tmp_path, threads):
    """vc_vafset_add_many keeps a bounded window of open files: 600 inputs load
    under a 128-descriptor limit (at most 64 open at once) (the reference opens and closes one file at a
    time, correlation-matrix.c:304,329-335, so it has no such limit)."""
    row = "chr1\t%d\trs%d\tA\tC\t5\t5\t10\t0.500000\n"
    for i in range(600):
        with open(os.path.join(tmp_path, "s%04d.vaf" % i), "w") as f:
            f.write("#header\n" + "".join(row % (j, j) for j in range(3)))
    p = subprocess.run([sys.executable, "-c", _MANY_FILES, PKG, str(tmp_path), "600", str(threads)],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "ok 600" in p.stdout, p.stderr[-2000:]


# --- GPU ---------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_cli_matches_reference(name, work):
    check(CASES[name], run(CLI, CASES[name], work))


def random_set(rng, n_samples, n_rows, ragged=True):
    g = [rng.integers(0, 3, n_rows) for _ in range(4)]
    vaf = np.zeros((n_samples, n_rows))
    dep = np.zeros((n_samples, n_rows), np.int32)
    ns = np.full(n_samples, n_rows, np.int32)
    for s in range(n_samples):
        d = rng.poisson(rng.integers(1, 40), n_rows)
        d[rng.random(n_rows) < rng.random() * 0.3] = 0
        alt = rng.binomial(d, np.clip(g[s % 4] / 2.0, 0.01, 0.99))
        vaf[s] = np.where(d > 0, np.round(alt / np.maximum(d, 1), 4), 0.0)
        dep[s] = d
        if ragged and rng.random() < 0.3:
            ns[s] = int(rng.integers(0, n_rows + 1))
    return vaf, dep, ns


def write_set(d, vaf, dep, ns):
    paths = []
    for s in range(vaf.shape[0]):
        p = os.path.join(d, "r%03d.vaf" % s)
        lines = ["# Average depth: 1.00\n", "CHR\tPOS\tRSID\tREF\tALT\tREF_COUNT\tALT_COUNT\tTOTAL_COUNT\tVAF\n"]
        for i in range(ns[s]):
            lines.append("chr1\t%d\trs%d\tA\tC\t0\t0\t%d\t%.4f\n" % (i, i, dep[s, i], vaf[s, i]))
        with open(p, "w") as f:
            f.write("".join(lines))
        paths.append(p)
    return paths


@pytest.mark.gpu
@pytest.mark.parametrize("n_samples,n_rows,opts", [(70, 700, []), (130, 257, ["-M", "strict"]),
                                                   (17, 2000, ["-d", "0", "-m", "0"]), (65, 64, ["-m", "3"])])
def test_cli_matches_oracle_random(n_samples, n_rows, opts, tmp_path):
    rng = np.random.default_rng(n_samples * 1000 + n_rows)
    paths = write_set(str(tmp_path), *random_set(rng, n_samples, n_rows))
    outs = {}
    for tag, binary in (("gpu", CLI), ("orc", ORACLE)):
        o = str(tmp_path / ("%s.corr" % tag))
        p = subprocess.run([binary, "-t", "-o", o] + opts + paths, capture_output=True, timeout=600)
        assert p.returncode == 0, p.stderr
        with open(o) as f, open(str(tmp_path / ("%s.tree" % tag))) as g:
            outs[tag] = (f.read(), g.read(), p.stderr.decode().replace(tag + ".", "X."))
    assert outs["gpu"] == outs["orc"]


@pytest.mark.gpu
def test_mirror_matrix_matches_python_statement():
    import vafc
    rng = np.random.default_rng(7)
    vaf, dep, ns = random_set(rng, 23, 300)
    corr, ms = vafc.correlation_matrix_raw(vaf, dep, ns, min_snps=5, min_depth=2)
    assert ms > 0
    for i in range(23):
        assert corr[i, i] == 1.0
        for j in range(i + 1, 23):
            inj = np.arange(300) < ns[j]
            want = py_pair((list(vaf[i]), list(dep[i])), (list(vaf[j] * inj), list(dep[j] * inj)),
                           int(ns[i]), 5, 2)
            got = corr[i, j]
            assert got == want or (math.isnan(got) and math.isnan(want)), (i, j, got, want)
            assert corr[j, i] == got or math.isnan(got)


@pytest.mark.gpu
def test_mirror_edges():
    import vafc
    c, _ = vafc.correlation_matrix_raw(np.zeros((1, 5)), np.ones((1, 5), np.int32))
    assert c.shape == (1, 1) and c[0, 0] == 1.0
    c, _ = vafc.correlation_matrix_raw(np.zeros((3, 0)).reshape(3, 0), np.zeros((3, 0), np.int32))
    assert np.array_equal(c, np.eye(3))
