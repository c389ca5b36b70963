#!/usr/bin/env python3
"""Golden cases of the split-gzip driver (round 6), from the REAL reference:
the gzip shapes of tests/gz_variants.py built from the synthetic c1_10k.fq,
the reference run on them, and the cases appended to manifest.json (any
earlier gz_* cases replaced).  Needs `make -C oracle` (oracle/_ref/vaf-counter).

    python tests/golden/make_golden_gz.py
"""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import gz_variants  # noqa: E402
import make_golden as G  # noqa: E402
import vafc_synth as S  # noqa: E402


def main():
    if not os.path.exists(G.REF):
        sys.exit("build the reference first: make -C oracle")
    mpath = os.path.join(HERE, "manifest.json")
    with open(mpath) as f:
        manifest = json.load(f)
    d = tempfile.mkdtemp(prefix="vafc_gz_golden_")
    full = S.grch38_panel()
    full.write_patterns(os.path.join(d, "grch38_k21.txt"), 21)
    S.write_fastq(os.path.join(d, "c1_10k.fq"), full, 10_000, seed=S.READ_SEED_R1, f_snp=1.0)
    assert G.md5(os.path.join(d, "c1_10k.fq")) == manifest["synth"]["c1_10k.fq"]
    gz_variants.make(d)
    for fn in gz_variants.VARIANTS:
        manifest["synth"][fn] = G.md5(os.path.join(d, fn))
        manifest["synth_spec"][fn] = "tests/gz_variants.py make()"
    manifest["cases"] = [c for c in manifest["cases"] if not c["name"].startswith("gz_")]
    for name, files in (("gz_multi_k21", ["c1_10k_multi.fq.gz"]),
                        ("gz_trailing_k21", ["c1_10k_trailing.fq.gz"]),
                        ("gz_mixed_k21", ["c1_10k_multi.fq.gz", "c1_10k.fq", "c1_10k_trailing.fq.gz"]),
                        # consecutive gzip files: one wave of rank groups in vafc_dist (round 6)
                        ("gz_pair_k21", ["c1_10k_multi.fq.gz", "c1_10k_trailing.fq.gz"]),
                        ("gz_trio_k21", ["c1_10k_trailing.fq.gz", "c1_10k_multi.fq.gz", "c1_10k_trailing.fq.gz"])):
        argv = ["-v", "-k", "21", "-t", "2", "-p", "grch38_k21.txt"] + files
        rc, stats, err = G.run_ref(argv + ["-o", "out.vaf"], d)
        out = os.path.join(d, "out.vaf")
        entry = {"name": name, "argv": argv, "inputs": ["synth:grch38_k21.txt"] + ["synth:" + f for f in files],
                 "exit": rc, "stats": stats, "vaf_md5": G.md5(out) if os.path.exists(out) else None,
                 "collision_warning": "collisions detected" in err}
        if os.path.exists(out):
            os.remove(out)
        manifest["cases"].append(entry)
        print("%-28s rc=%d %s %s" % (name, rc, entry["vaf_md5"], stats))
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
