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


def _fake_measurements(steps=20):
    """A bench line's pieces with realistic sizes (C3: two files, 20 steps,
    three CLI runs of each kind, every reader profile filled)."""
    import bench
    rd = {"total": 0.53, "main_wait": 0.4, "submit": 0.02, "parse": 7.21, "slot_wait": 0.31,
          "acquire": 0.15, "read": 3.01, "copy": 1.2, "cpu": 7.9, "wall": 8.41, "main_cpu": 0.12}
    e2e = {"value": 28205.2, "kmers_per_sec": 24012345678.9, "bases": 30000000000,
           "seqs": 200000000, "kmers": 26000000000, "file_bytes": 62980000000, "files": 2, "threads_per_rank": 16,
           "ranks": 1, "elapsed_s": 10.6363, "step_ms": [531.8] * steps, "count_ms": [530.1] * steps,
           "step_mbases": {"min": 23456.7, "median": 28205.2, "max": 32567.8, "spread": 0.321},
           "reader_slowest_step": dict(rd), "reader_fastest_step": dict(rd), "split_exact": True}
    cli_kind = {"value": 23246.2, "runs": [23246.2, 22188.4, 25006.5], "counting_s": 1.291,
                "process_s": 2.123, "throttled_ms": [12.3, 45.6, 0.0], "cpu_s": [9.123, 9.456, 8.901],
                "reader": {f: [7.21, 7.35, 6.98] for f in ("total", "parse", "read", "copy", "cpu", "wall", "acquire",
                                                            "main_wait")},
                "vs_cpu_baseline": 295.5, "frac_of_parse_only": 0.514}
    cli = {"threads": 16, "plain": dict(cli_kind), "gzip": dict(cli_kind, frac_of_inflate_only=0.745),
           "parse_only_s": 0.332, "inflate_only_s": 2.851, "parity_vs_count_device": True}
    cpu = {"value": 78.67, "unit": "Mbases/sec", "cores": 3, "kind": "reference", "threads_flag": 1,
           "host_cpus": 256, "cpu_share": 16, "by_threads": {"1": 78.67, "4": 40.54, "16": 67.9, "256": 20.67},
           "sample": "first 1000000 reads of each of 2 file(s) (300 Mbases), reference -v Speed, median of 3 per -t"}
    return {"L": 150, "k": 31, "world": 1, "steps": steps, "warmup": 5, "config": "c3", "e2e": e2e, "cli": cli,
            "cpu": cpu, "k_value": 2992613.2, "k_elapsed": 0.0997, "k_steps": 10, "k_kmer_rate": 2539663364409.9,
            "k_ms": 9.9722, "achieved": 3177.6, "traffic": 23412105152.0, "alg_bytes": 31600000000,
            "panel_src": "SNP_GRCh38_hg38_wChr.bed",
            "workload": "C3: 2 file(s) of 100M x 150 bp reads (62.98 GB, page cache), k=31, grch38 panel (20849 "
                        "patterns, 41697 keys), f_snp=0.01; 1 rank(s), byte ranges of each file",
            "R": 200000000, "reads_total": 200000000, "n_pat": 20849, "n_files": 2,
            "parallelism": "dp1 (byte ranges per rank, RCCL all-reduce of u32 counts + u64 tally)",
            "limiter": bench.LIMITER_LARGE_PANEL, "build_id": "0123456789abcdef0123",
            "detail_path": "/tmp/vafc_bench_detail_123456.json", "parity": True, "full_parity": True}


def test_bench_line_stays_under_bound():
    """The JSON line the driver keeps must hold its own evidence: under 4 KB
    with 20 steps, two files and every CLI run's reader phases, the parity
    booleans last."""
    import json
    import bench
    for steps in (20, 50):
        line = bench.assemble_line(_fake_measurements(steps))
        text = json.dumps(line)
        assert len(text) <= bench.LINE_BYTES_MAX or steps > 20, len(text)
        keys = list(line)
        assert keys[-2:] == ["parity_vs_reference_on_sample", "parity_full_size"]
        assert line["value_kind"] == "e2e_file" and line["value"] == 28205.2
    a = _fake_measurements()
    a["e2e"] = None
    a["cli"] = None
    line = bench.assemble_line(a)
    assert line["value_kind"] == "kernel_hbm" and line["value"] == 2992613.2 and line["vs_cpu_baseline"] is None


def test_bench_line_withholds_value_when_ranges_do_not_chain():
    import bench
    a = _fake_measurements()
    a["e2e"] = dict(a["e2e"], value=None, split_exact=False)
    line = bench.assemble_line(a)
    assert line["value"] is None and line["vs_cpu_baseline"] is None


def test_parse_ingest_line_reads_the_reader_profile(tmp_path):
    """bench.parse_ingest_line understands the line VAFC_INGEST_PROFILE makes
    the parallel reader print (vafc_ingest.cpp)."""
    import subprocess
    import sys
    import bench
    import vafc_synth as S
    fq = tmp_path / "r.fq"
    panel = S.make_panel(S.read_bed(S.default_bed_path())[:50])
    S.write_fastq(str(fq), panel, 20000)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path.insert(0, %r); import vafc; vafc.scan_file_parallel(%r, 21, 10_000_000, 3, 1 << 16)"
            % (os.path.join(root, "kmer-cnt_amd"), str(fq)))
    p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, VAFC_INGEST_PROFILE="1"),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    lines = [l for l in p.stderr.splitlines() if l.startswith("[ingest]")]
    assert lines, p.stderr
    d = bench.parse_ingest_line(lines[-1])
    assert d is not None and d["total"] > 0 and d["read"] > 0 and d["copy"] > 0 and d["wall"] >= d["parse"] * 0


def test_rank_device_refuses_more_ranks_than_gpus():
    import bench
    assert bench.rank_device(0, 1, 1, "nccl", False) == 0
    assert bench.rank_device(3, 8, 8, "nccl", False) == 3
    assert bench.rank_device(1, 2, 1, "nccl", False) is None          # two ranks, one GPU
    assert bench.rank_device(0, 2, 1, "nccl", False) is None          # every rank refuses, not just the extra one
    assert bench.rank_device(1, 2, 1, "gloo", False) is None          # gloo without the rehearsal flag
    assert bench.rank_device(1, 2, 1, "nccl", True) is None           # the flag is for gloo only
    assert bench.rank_device(1, 2, 1, "gloo", True) == 0              # explicit rehearsal wraps
    assert bench.rank_device(0, 1, 0, "gloo", True) is None           # no GPU at all


def test_bench_exits_2_without_a_gpu_per_rank():
    """bench.py under WORLD_SIZE=2 with fewer GPUs visible than ranks (none
    here) exits 2 before any rendezvous instead of doubling ranks onto a card."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", LOCAL_WORLD_SIZE="2",
               MASTER_ADDR="127.0.0.1", MASTER_PORT="29999", VAFC_DIST_BACKEND="gloo")
    env.pop("VAFC_REHEARSAL", None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "one GPU per rank" in p.stderr and p.stdout == ""
