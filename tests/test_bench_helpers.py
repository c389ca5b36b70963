"""bench.py's host helpers (CPU): the pigz-style gzip writer used for the
end-to-end leg produces one valid gzip member whose text is the input, the
CPU-share rule, and the reference CLI's -v parsing."""
import gzip
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_gzip_level1_is_one_member_with_the_input_text(tmp_path):
    import bench
    import vafc
    rng = np.random.default_rng(0)
    for size in (0, 1, 40_000, 3 * (1 << 20) + 17):
        src = tmp_path / ("t%d.fq" % size)
        data = np.frombuffer(b"ACGT\n@+I", np.uint8)[rng.integers(0, 8, size)].tobytes()
        src.write_bytes(data)
        dst = str(src) + ".gz"
        bench.gzip_level1(str(src), dst, 3, chunk=1 << 20)
        raw = open(dst, "rb").read()
        assert raw[:4] == b"\x1f\x8b\x08\x00"
        assert gzip.decompress(raw) == data
        assert vafc.gz_inflate_zlib(dst) == data
        if size:   # the product's parallel inflater reads it as gzread does, one member
            got = vafc.gz_inflate_parallel(dst, threads=3, chunk_bytes=4096)
            assert got is not None and got[0] == data and got[1]["members"] == 1


def test_cpu_share_bounds():
    import bench
    n = len(os.sched_getaffinity(0))
    assert bench.cpu_share() == max(1, min(16, n))
    assert bench.cpu_share(8) == max(1, min(128, n))


def test_cli_run_parses_reference_speed_line(tmp_path):
    """cli_run on the reference binary (when built here): Speed, k-mer rate and
    bases come from the -v report."""
    import bench
    import vafc_synth as S
    if not os.path.exists(bench.REF_CLI):
        import pytest
        pytest.skip("reference binary not built")
    panel = S.make_panel(S.synthetic_bed(200))
    pat = str(tmp_path / "p.txt")
    panel.write_patterns(pat, 21)
    fq = str(tmp_path / "r.fq")
    S.write_fastq(fq, panel, 2000, f_snp=0.5)
    r = bench.cli_run(bench.REF_CLI, pat, fq, 1, str(tmp_path / "o.vaf"), 21)
    assert r["bases"] == 2000 * 150 and r["mbases"] > 0 and r["mkmers"] > 0


def test_fastq_bytes_np_equals_fastq_bytes():
    """The array-built FASTQ records of the end-to-end file are the bytes of the
    per-record writer the goldens use, across read-number digit boundaries."""
    import vafc_synth as S
    rng = np.random.default_rng(3)
    reads = np.frombuffer(b"ACGTN", np.uint8)[rng.integers(0, 5, (3000, 150))]
    for first in (0, 7, 98, 997, 9_999_000, 99_999_999 - 1500):
        assert S.fastq_bytes_np(reads, first) == S.fastq_bytes(reads, first), first


def test_vaf_counts_reads_the_writer_output(tmp_path):
    """bench.vaf_counts parses the .vaf writer's counts back (the N > 1 parity
    compares all-reduced counts with N x the reference's)."""
    import bench
    import vafc
    import vafc_synth as S
    panel = S.make_panel(S.synthetic_bed(50))
    pat = str(tmp_path / "p.txt")
    panel.write_patterns(pat, 21)
    db = vafc.load_patterns(pat)
    counts = np.random.default_rng(1).integers(0, 2 ** 32, 2 * db.n, dtype=np.uint64).astype(np.uint32)
    db.write_vaf(counts, str(tmp_path / "o.vaf"))
    assert np.array_equal(bench.vaf_counts(str(tmp_path / "o.vaf")), counts)


def test_bench_spawns_one_rank_per_gpu(tmp_path):
    """`bench.py --gpus N` outside torchrun starts N rank processes with the
    torchrun environment (rank 0's stdout is the bench's), and returns the
    first failing rank's status after stopping the others."""
    import subprocess
    import sys
    import bench
    child = tmp_path / "child.py"
    child.write_text("import os, sys, time\n"
                     "r = int(os.environ['RANK'])\n"
                     "print('rank', r, os.environ['LOCAL_RANK'], os.environ['WORLD_SIZE'], os.environ['MASTER_ADDR'],"
                     " flush=True)\n"
                     "if 'fail' in sys.argv and r == 1: sys.exit(3)\n"
                     "if 'fail' in sys.argv: time.sleep(30)\n")
    out = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); import bench; "
                          "sys.exit(bench.spawn_ranks(['x'], 3, %r))" % (os.path.dirname(bench.__file__), str(child))],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0
    assert out.stdout.split() == ["rank", "0", "0", "3", "127.0.0.1"]          # only rank 0 prints
    import time
    t0 = time.time()
    assert bench.spawn_ranks(["fail"], 2, str(child)) == 3
    assert time.time() - t0 < 20                                                # rank 0 was stopped


def test_bench_refuses_world_size_other_than_gpus():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 2 and "WORLD_SIZE" in p.stderr and p.stdout == ""


def test_rank_threads_split_the_share():
    import bench
    assert 1 <= bench.rank_threads(1) <= 16
    assert bench.rank_threads(8) <= max(1, bench.rank_threads(1))
