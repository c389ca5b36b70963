"""libvafc.so: loads, exports every symbol include/vafc.h declares, and its
host-side logic (pattern loader, key table content, .vaf writer) agrees with
the oracle -- no GPU needed."""
import hashlib
import os
import re

import numpy as np
import pytest

from conftest import CASES, ROOT


def header_functions():
    with open(os.path.join(ROOT, "include", "vafc.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vc_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import vafc
    L = vafc.lib()
    declared = header_functions()
    assert len(declared) >= 25
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert set(declared) == set(vafc.EXPORTS)
    assert L.vc_version() == 1


def test_strerror_and_nodev():
    import ctypes as C
    import vafc
    L = vafc.lib()
    assert L.vc_strerror(vafc.VC_EHIP) == b"HIP runtime error"
    h = C.c_void_p()
    keys = np.zeros(1, np.uint64)
    vals = np.zeros(1, np.uint32)
    rc = L.vc_create(C.byref(h), 40, keys.ctypes.data_as(C.c_void_p), vals.ctypes.data_as(C.c_void_p), 1, 1, 0)
    assert rc == vafc.VC_EINVAL or rc == vafc.VC_ENODEV       # k=40 rejected (or no device)
    import torch
    if not torch.cuda.is_available():
        rc = L.vc_create(C.byref(h), 21, keys.ctypes.data_as(C.c_void_p), vals.ctypes.data_as(C.c_void_p), 1, 1, 0)
        assert rc == vafc.VC_ENODEV


def test_missing_pattern_file():
    import vafc
    with pytest.raises(vafc.VafcError) as e:
        vafc.load_patterns("/nonexistent/patterns.txt")
    assert e.value.code == vafc.VC_EIO


@pytest.mark.parametrize("fn,k", [("pat_k21.txt", 21), ("pat_edge_k21.txt", 21), ("pat_edge_k31.txt", 31),
                                  ("pat_edge_k15.txt", 15), ("empty_patterns.txt", 21)])
def test_pattern_keys_match_oracle(fn, k):
    """create_combined_kmer_map content: same (key -> value) mapping, same collisions."""
    import vafc
    import oracle as O
    db = vafc.load_patterns(os.path.join(CASES, fn))
    keys, vals, coll = db.keys(k)
    orc = O.Oracle(k, pattern_fn=os.path.join(CASES, fn))
    ok, ov = orc.keys()
    assert db.n == orc.n_patterns
    assert coll == orc.n_collisions
    assert dict(zip(keys.tolist(), vals.tolist())) == dict(zip(ok.tolist(), ov.tolist()))


def test_vaf_writer_matches_reference_output(manifest, tmp_path):
    """Host .vaf writer fed the oracle's counts reproduces the reference's file."""
    import vafc
    import oracle as O
    entry = next(c for c in manifest["cases"] if c["name"] == "edge_k21")
    orc = O.Oracle(21, pattern_fn=os.path.join(CASES, "pat_k21.txt"))
    counts = np.zeros(2 * orc.n_patterns + 2, np.uint32)
    rc, b, s, km = orc.count_file(os.path.join(CASES, "edge.fq"), 10_000_000, counts)
    db = vafc.load_patterns(os.path.join(CASES, "pat_k21.txt"))
    out = str(tmp_path / "w.vaf")
    db.write_vaf(counts, out)
    assert hashlib.md5(open(out, "rb").read()).hexdigest() == entry["vaf_md5"]


def test_vaf_writer_u32_wraparound(tmp_path):
    """TOTAL_COUNT is a uint32 sum that wraps (vaf-counter.c:673); the average is not."""
    import vafc
    db = vafc.load_patterns(os.path.join(CASES, "pat_k21.txt"))
    counts = np.zeros(2 * db.n, np.uint32)
    counts[0], counts[1] = 0xFFFFFFF0, 0x20
    out = str(tmp_path / "wrap.vaf")
    db.write_vaf(counts, out)
    lines = open(out).read().splitlines()
    f = lines[2].split("\t")
    assert f[5:8] == [str(0xFFFFFFF0), str(0x20), str((0xFFFFFFF0 + 0x20) & 0xFFFFFFFF)]
    assert float(f[8]) == pytest.approx(0x20 / 0x10, abs=1e-4)
    assert lines[0] == "# Average depth: %.2f" % ((0xFFFFFFF0 + 0x20) / db.n)


def test_reference_binding_patch_applies():
    """oracle/bind_reference.py finds each of its anchors exactly once in the
    reference's vaf-counter.c (skipped where the reference is absent)."""
    import importlib.util
    src = "/root/reference/vaf-counter.c"
    if not os.path.exists(src):
        pytest.skip("reference sources not present")
    spec = importlib.util.spec_from_file_location("bind_reference", os.path.join(ROOT, "oracle", "bind_reference.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    out = m.patch(open(src).read())
    assert out.count("vc_count_file(") == 1 and out.count("vc_create(") == 1 and "count_fastq_kmers(argv[i]" not in out


def test_build_id_matches_tree():
    """Every product binary carries the hash of the sources it was built from
    ("VAFC_BUILD_ID=<hex>", vc_build_id); it equals the hash of this tree's
    kmer-cnt_amd/csrc/* + include/vafc.h, so a stale binary cannot pass."""
    import vafc
    want = vafc.tree_build_id()
    assert re.fullmatch(r"[0-9a-f]{16}", want)
    vafc.check_build()
    assert vafc.lib().vc_build_id().decode() == want


def _lib_dir():
    lib = os.environ.get("VAFC_LIB")
    return os.path.dirname(lib) if lib else os.path.join(ROOT, "kmer-cnt_amd", "lib")


def test_rccl_missing_fails_loudly(tmp_path):
    """More than one distinct device and no loadable RCCL: vc_create_multi
    returns VC_EHIP before any device is touched, and the CLI with
    VAFC_DEVICES=0,1 exits 1 with the error (no GPU needed: RCCL is loaded
    first).  Under tools/asan_tests.sh the CLI is the sanitizer build and runs
    with leak detection on, so a leak on this path fails the test."""
    import subprocess
    import sys
    import vafc
    env = dict(os.environ, VAFC_RCCL_LIB="/nonexistent/librccl.so.1")
    code = ("import sys, ctypes as C, numpy as np; sys.path.insert(0, %r); import vafc; L = vafc.lib(); "
            "h = C.c_void_p(); k = np.zeros(1, np.uint64); v = np.zeros(1, np.uint32); "
            "d = np.array([0, 1], np.int32); "
            "print(L.vc_create_multi(C.byref(h), 21, k.ctypes.data_as(C.c_void_p), v.ctypes.data_as(C.c_void_p), "
            "1, 1, d.ctypes.data_as(C.c_void_p), 2), h.value)" % os.path.join(ROOT, "kmer-cnt_amd"))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert p.stdout.split() == [str(vafc.VC_EHIP), "None"], p.stdout
    assert "cannot load RCCL" in p.stderr
    pat = tmp_path / "p.txt"
    pat.write_text("chr1\t1\t2\trs1\tA\tC\tACGTACGTACGTACGTACGTA\tACGTACGTACGAACGTACGTA\n")
    fq = tmp_path / "r.fq"
    fq.write_text("@r\nACGTACGTACGTACGTACGTACGT\n+\nIIIIIIIIIIIIIIIIIIIIIIII\n")
    cli = os.path.join(_lib_dir(), "vaf-counter")
    env2 = dict(env, VAFC_DEVICES="0,1")
    if "asan" in env.get("LD_PRELOAD", ""):
        env2["ASAN_OPTIONS"] = env.get("ASAN_OPTIONS", "").replace("detect_leaks=0", "detect_leaks=1")
    p = subprocess.run([cli, "-p", str(pat), "-o", str(tmp_path / "o.vaf"), str(fq)], env=env2,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 1, p.stderr[-3000:]
    assert "cannot load RCCL" in p.stderr and "failed to create k-mer map" in p.stderr
    assert not (tmp_path / "o.vaf").exists()
