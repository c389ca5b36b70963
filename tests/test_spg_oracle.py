"""snp-pattern-gen: the CPU restatement
(oracle/spg_oracle.c) against the real reference's outputs recorded in
tests/golden/spg/manifest.json -- output file md5, stderr text, exit code."""
import hashlib
import json
import os
import shutil
import subprocess

import pytest

from conftest import GOLDEN, ROOT

SPG = os.path.join(GOLDEN, "spg")
with open(os.path.join(SPG, "manifest.json")) as _f:
    SPG_CASES = json.load(_f)["cases"]
SPG_ORACLE = os.path.join(ROOT, "oracle", "build", "snp-pattern-gen-oracle")


def run_spg(binary, case, tmp_path, env=None):
    for fn in os.listdir(SPG):
        if not fn.endswith(".json"):
            shutil.copy(os.path.join(SPG, fn), tmp_path)
    p = subprocess.run([binary] + case["argv"], cwd=tmp_path, capture_output=True, text=True, timeout=300,
                       env=env)
    out = os.path.join(tmp_path, "out.txt")
    md5 = hashlib.md5(open(out, "rb").read()).hexdigest() if os.path.exists(out) else None
    return p.returncode, p.stderr, md5


@pytest.mark.parametrize("case", SPG_CASES, ids=[c["name"] for c in SPG_CASES])
def test_oracle_matches_reference(case, tmp_path):
    rc, err, md5 = run_spg(SPG_ORACLE, case, tmp_path)
    assert rc == case["exit"]
    assert err == case["stderr"]
    assert md5 == case["out_md5"]


def test_fixture_has_both_outcomes():
    lines = {c["name"]: c["out_lines"] for c in SPG_CASES}
    assert lines["g1_k21"] > 300 and lines["g1_k3"] == 0 and 0 < lines["g1_k9"] < lines["g1_k21"]
