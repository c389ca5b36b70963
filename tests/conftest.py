import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
CASES = os.path.join(GOLDEN, "cases")
PKG = os.path.join(ROOT, "kmer-cnt_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

PRODUCT_CLI = os.path.join(PKG, "lib", "vaf-counter")
ORACLE_CLI = os.path.join(ROOT, "oracle", "build", "vaf-counter-oracle")
REF_CLI = os.path.join(ROOT, "oracle", "_ref", "vaf-counter")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def built():
    """Build the oracle and the product once per session (no-op when up to date)."""
    if os.environ.get("VAFC_SKIP_BUILD") == "1":   # sanitizer runs (tools/asan_tests.sh) bring their own build
        return
    jobs = str(min(8, os.cpu_count() or 2))
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "oracle")], check=True)
    # The product is prebuilt in-tree (its objects do not travel to the GPU
    # box, so make would rebuild it there from scratch).  Every binary carries
    # the hash of the sources it was built from (vc_build_id, the Makefile's
    # BUILD_ID); it must equal the hash of this tree's sources.  Where the
    # build host's reference tree is present, a mismatch rebuilds; elsewhere
    # (the GPU box) it stops the session instead of testing a stale library.
    import vafc
    try:
        vafc.check_build()
        return
    except vafc.VafcError as e:
        if not os.path.isdir("/root/reference") and os.environ.get("VAFC_AUTO_BUILD") != "1":
            pytest.exit(str(e), returncode=3)
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(PKG, "csrc")], check=True)
    vafc.check_build()


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def synth_dir(tmp_path_factory, manifest):
    """Regenerate the synthetic golden inputs and check their md5 first."""
    import hashlib
    import gzip
    import vafc_synth as S
    d = str(tmp_path_factory.mktemp("synth"))
    full = S.grch38_panel()
    full.write_patterns(os.path.join(d, "grch38_k21.txt"), 21)
    full.write_patterns(os.path.join(d, "grch38_k31.txt"), 31)
    S.write_fastq(os.path.join(d, "c1_10k.fq"), full, 10_000, seed=S.READ_SEED_R1, f_snp=1.0)
    S.write_fastq(os.path.join(d, "pe_R1.fq"), full, 2_000, seed=S.READ_SEED_R1, f_snp=0.5)
    S.write_fastq(os.path.join(d, "pe_R2.fq"), full, 2_000, seed=S.READ_SEED_R2, f_snp=0.5)
    with open(os.path.join(d, "c1_10k.fq"), "rb") as f, \
            gzip.open(os.path.join(d, "c1_10k.fq.gz"), "wb", compresslevel=1) as g:
        g.write(f.read())
    import gz_variants
    gz_variants.make(d)
    for fn, want in manifest["synth"].items():
        with open(os.path.join(d, fn), "rb") as f:
            assert hashlib.md5(f.read()).hexdigest() == want, "synthetic generator drifted: " + fn
    return d


def case_dir(entry, synth_dir):
    return synth_dir if entry["inputs"] and entry["inputs"][0].startswith("synth:") else CASES


def run_cli(binary, entry, synth_dir, tmp_path, env=None):
    """Run a vaf-counter CLI on a manifest case; returns (rc, stats, vaf bytes or None)."""
    out = os.path.join(str(tmp_path), "out_%s.vaf" % entry["name"])
    p = subprocess.run([binary] + entry["argv"] + ["-o", out], cwd=case_dir(entry, synth_dir),
                       capture_output=True, text=True, timeout=600, env=env)
    stats = {}
    for key, pat in (("bases", "Bases processed:"), ("seqs", "Sequences processed:"),
                     ("kmers", "K-mers extracted:")):
        for line in p.stderr.splitlines():
            if pat in line:
                stats[key] = int(line.split(":")[1].split()[0])
    data = None
    if os.path.exists(out):
        with open(out, "rb") as f:
            data = f.read()
    return p.returncode, stats, data, p.stderr
