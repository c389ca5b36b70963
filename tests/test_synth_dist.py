"""Synthetic workload generator, rank sharding and the count all-reduce (gloo,
world_size 2, CPU), and the Python CLI mirror's option parsing."""
import os

import numpy as np
import pytest


def test_generator_is_counter_based():
    import vafc_synth as S
    p = S.make_panel(S.synthetic_bed(50))
    a = S.gen_reads(p, 100, first=0, f_snp=0.3)
    b = S.gen_reads(p, 60, first=40, f_snp=0.3)
    assert np.array_equal(a[40:], b)                     # any slice regenerates alone
    assert set(np.unique(a).tolist()) <= set(b"ACGTN")
    rc = (S.h64(S.READ_SEED_R1, np.arange(100, dtype=np.uint64), 3) & np.uint64(1)) == 1
    assert 20 < int(rc.sum()) < 80


def test_panel_kmers_place_snp_like_snp_pattern_gen():
    import vafc_synth as S
    p = S.make_panel(S.synthetic_bed(10))
    for k in (21, 31, 20):
        ref, alt = p.kmers(k)
        assert ref.shape == (10, k)
        assert np.array_equal(ref[:, k // 2], p.ref) and np.array_equal(alt[:, k // 2], p.alt)
        diff = (ref != alt).sum(axis=1)
        assert np.all(diff == 1)


def test_snp_reads_hit_patterns():
    """Reads cut from SNP windows contain their pattern k-mer (counts are non-trivial)."""
    import vafc_synth as S
    import oracle as O
    import tempfile
    p = S.make_panel(S.synthetic_bed(200))
    with tempfile.TemporaryDirectory() as d:
        pat = os.path.join(d, "p.txt")
        p.write_patterns(pat, 21)
        orc = O.Oracle(21, pattern_fn=pat)
        seq, offs, lens = S.pack_reads(S.gen_reads(p, 2000, f_snp=1.0))
        counts, km = orc.count_reads(seq, offs, lens)
    assert km > 2000 * 120
    assert 1200 < int(counts.sum()) < 2000


@pytest.mark.parametrize("n,world", [(10, 3), (100, 8), (7, 8), (0, 2)])
def test_shard_partition(n, world):
    from vafc_dist import shard
    parts = [shard(n, r, world) for r in range(world)]
    assert sum(c for _, c in parts) == n
    pos = 0
    for first, c in parts:
        assert first == pos
        pos += c
    assert max(c for _, c in parts) - min(c for _, c in parts) <= 1


def _rank_main(rank, world, port, pat, reads_path, out_path, counter="oracle"):
    import torch.distributed as dist
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "kmer-cnt_amd"))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    import oracle as O
    import vafc_dist as D
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    z = np.load(reads_path)
    seq, offs, lens = z["seq"], z["offs"], z["lens"]
    first, cnt = D.shard(lens.size, rank, world)
    if counter == "hip":                     # the product's counter (GPU tests)
        import vafc
        db = vafc.load_patterns(pat)
        m = vafc.create_combined_kmer_map(db, 21, device=0)
        m.count_block(seq, offs[first:first + cnt], lens[first:first + cnt])
        counts, km = m.finish()
        counts = counts.copy()
        m.close()
    else:                                    # CPU stand-in for the per-GPU counter
        orc = O.Oracle(21, pattern_fn=pat)
        counts, km = orc.count_reads(seq, offs[first:first + cnt], lens[first:first + cnt])
    if rank == 0:
        counts[0] = np.uint32((int(counts[0]) + 0xFFFFFFFF) & 0xFFFFFFFF)   # force a wrap
    t = D.counts_to_tensor(counts)
    D.allreduce_counts(t)
    total_km = D.allreduce_u64(int(km))
    if rank == 0:
        np.savez(out_path, counts=D.tensor_to_counts(t), kmers=np.array([total_km], np.uint64))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("counter", ["oracle", pytest.param("hip", marks=pytest.mark.gpu)])
def test_gloo_allreduce_of_sharded_counts_is_bit_exact(tmp_path, counter):
    """Two ranks count their shards (the oracle on CPU; the HIP counter, both
    ranks on device 0, in the GPU suite) and all-reduce over gloo."""
    import socket
    import torch.multiprocessing as mp
    import vafc_synth as S
    import oracle as O
    p = S.make_panel(S.synthetic_bed(300))
    pat = str(tmp_path / "p.txt")
    p.write_patterns(pat, 21)
    seq, offs, lens = S.pack_reads(S.gen_reads(p, 3001, f_snp=0.7))
    rp = str(tmp_path / "reads.npz")
    np.savez(rp, seq=seq, offs=offs, lens=lens)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "out.npz")
    mp.start_processes(_rank_main, args=(2, port, pat, rp, out, counter), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    orc = O.Oracle(21, pattern_fn=pat)
    want, km = orc.count_reads(seq, offs, lens)
    want = want.copy()
    want[0] = np.uint32((int(want[0]) + 0xFFFFFFFF) & 0xFFFFFFFF)   # same forced wrap
    assert np.array_equal(got["counts"], want)
    assert int(got["kmers"][0]) == km


def test_cli_option_parsing_mirror():
    import vafc
    o, files = vafc.parse_args(["a.fq", "-k", "31", "-p", "pat.txt", "b.fq", "-vt8", "-o", "x.vaf", "-b1"])
    assert files == ["a.fq", "b.fq"]
    assert (o["k"], o["p"], o["o"], o["t"], o["b"], o["v"]) == (31, "pat.txt", "x.vaf", 8, 1, True)
    o, files = vafc.parse_args(["-p", "p", "-o", "o", "--", "-weird.fq"])
    assert files == ["-weird.fq"]
    assert vafc.main(["-p", "p.txt"]) == 1                      # usage -> exit 1


# --------------------------------------------------------------------------
# the torchrun driver (kmer-cnt_amd/vafc_dist.py): files dealt over the ranks,
# one all-reduce, rank 0 writes the .vaf -- against the reference's goldens
# --------------------------------------------------------------------------

DIST_CASES = ["pe_k31", "c1_plumbing_k21", "c1_plumbing_k21_gz", "c1_k21_b1", "missing_file", "multiline_k21",
              "edge_crlf_k21", "pat_edge_k31", "truncated", "empty_reads", "mal_gbbbgbbbg_b1", "mal_bg", "pal_k16",
              "edge_gz", "gz_multi_k21", "gz_trailing_k21", "gz_mixed_k21"]
# cases whose every file is well formed and plain: the byte ranges must chain
# (no fallback to a whole-file recount)
DIST_CLEAN = {"pe_k31", "c1_plumbing_k21", "c1_k21_b1", "pal_k16"}
# well-formed gzip (and plain) files: shares of the stream, no whole-file count
DIST_GZ_CLEAN = {"c1_plumbing_k21_gz", "edge_gz", "gz_multi_k21", "gz_trailing_k21", "gz_mixed_k21"}
# consecutive gzip files: counted a wave at a time, each file by its own group of ranks
DIST_GZ_WAVES = {"gz_pair_k21", "gz_trio_k21"}


def _driver_rank(rank, world, port, argv, cwd, out_json, counter):
    import json
    import sys
    import torch.distributed as dist
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "kmer-cnt_amd"))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "oracle"))
    import vafc_dist as D
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank, world_size=world)
    os.chdir(cwd)
    lines = []
    calls = {"ranges": 0, "whole": 0, "restores": 0, "gz_shares": 0, "gz_held": 0}

    class OracleRankCounter(D.RankCounter):     # CPU stand-in for the per-GPU counter (test infrastructure)
        """The oracle counts what the product's host-only range reader
        (vc_scan_file_range) hands it; whole files through the oracle's own
        reader and block loop."""

        def __init__(self, db, k):
            import oracle as O
            self.k = k
            self.n = db.n
            self.orc = O.Oracle(k, pattern_fn=argv[argv.index("-p") + 1])
            self.counts = np.zeros(2 * db.n + 2, np.uint32)
            self.km = 0

        def count_range(self, fn, begin, end, block, threads):
            import vafc
            if begin == 0 and end == D.NO_OFFSET:
                calls["whole"] += 1
                rc, b, s, km = self.orc.count_file(fn, block, self.counts)
                if rc != 0:
                    return False, 0, 0, (D.NO_OFFSET, D.NO_OFFSET, 0, 0)
                self.km += km
                return True, b, s, (0, D.NO_OFFSET, 0, 1)
            calls["ranges"] += 1
            try:
                st, ri, reads = vafc.scan_file_range(fn, self.k, begin, end, block, threads, 64, with_reads=True)
            except FileNotFoundError:
                return False, 0, 0, (D.NO_OFFSET, D.NO_OFFSET, 0, 0)
            if reads:
                lens = np.array([len(r) for r in reads], np.uint32)
                offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
                seq = np.frombuffer(b"".join(reads), np.uint8)
                c, km = self.orc.count_reads(seq, offs, lens, self.n)
                self.counts[:2 * self.n] += c
                self.km += km
            return True, st.bases, st.seqs, (ri.first, ri.next, ri.errs, ri.stopped)

        # the held (single-pass) shares on odd-sized worlds, the two-pass ones on even
        gz_hold_bytes = (1 << 30) if world % 2 else 0

        def count_gz_share(self, fn, first_share, start_bit, window, text_len, block, threads):
            import vafc
            calls["gz_shares"] += 1
            try:
                st, ri, crc, reads = vafc.scan_gz_share(fn, self.k, first_share, start_bit, window, text_len, block,
                                                        threads, with_reads=True)
            except FileNotFoundError:
                return False, 0, 0, (D.NO_OFFSET, D.NO_OFFSET, 0, 0), None
            return self._add(st, ri, crc, reads)

        def count_gz_share_held(self, share, first_share, window, text_len, block, threads):
            import vafc
            calls["gz_shares"] += 1
            calls["gz_held"] += 1
            st, ri, crc, reads = vafc.scan_gz_share_held(share, self.k, first_share, window, text_len, block,
                                                         threads, with_reads=True)
            return self._add(st, ri, crc, reads)

        def _add(self, st, ri, crc, reads):
            if reads:
                lens = np.array([len(r) for r in reads], np.uint32)
                offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
                seq = np.frombuffer(b"".join(reads), np.uint8)
                c, km = self.orc.count_reads(seq, offs, lens, self.n)
                self.counts[:2 * self.n] += c
                self.km += km
            return True, st.bases, st.seqs, (ri.first, ri.next, ri.errs, ri.stopped), crc

        def save(self):
            self._saved = (self.counts.copy(), self.km)

        def restore(self):
            calls["restores"] += 1
            self.counts, self.km = self._saved[0].copy(), self._saved[1]

        def local_counts(self):
            return D.counts_to_tensor(self.counts[:2 * self.n]), self.km

    def make(db, k):
        if counter == "hip":
            return D.HipRankCounter(db, k, 0, "gloo")
        return OracleRankCounter(db, k)

    rc = D.run(argv, make, rank, world, err=lines.append)
    with open(out_json + ".%d" % rank, "w") as f:
        json.dump({"rc": rc, "stderr": "".join(lines), "calls": calls}, f)
    dist.barrier()
    dist.destroy_process_group()


def _run_driver(entry, synth_dir, tmp_path, counter, world=2):
    import json
    import socket
    import torch.multiprocessing as mp
    from conftest import case_dir
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / ("dist_%s.vaf" % entry["name"]))
    res = str(tmp_path / "res.json")
    mp.start_processes(_driver_rank, args=(world, port, entry["argv"] + ["-o", out], case_dir(entry, synth_dir), res,
                                           counter), nprocs=world, join=True, start_method="spawn")
    ranks = [json.load(open(res + ".%d" % r)) for r in range(world)]
    stats = {}
    for key, pat in (("bases", "Bases processed:"), ("seqs", "Sequences processed:"), ("kmers", "K-mers extracted:")):
        for line in ranks[0]["stderr"].splitlines():
            if pat in line:
                stats[key] = int(line.split(":")[1].split()[0])
    data = open(out, "rb").read() if os.path.exists(out) else None
    return [r["rc"] for r in ranks], stats, data, ranks[0]["stderr"], [r.get("calls") for r in ranks]


@pytest.mark.parametrize("counter", ["oracle", pytest.param("hip", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("name,world", [(n, 2) for n in DIST_CASES] + [("c1_plumbing_k21", 3), ("pe_k31", 3),
                                                                       ("mal_bg", 3), ("c1_plumbing_k21_gz", 3),
                                                                       ("gz_multi_k21", 3), ("gz_multi_k21", 5),
                                                                       ("edge_gz", 3), ("gz_mixed_k21", 3),
                                                                       ("gz_pair_k21", 2), ("gz_pair_k21", 3),
                                                                       ("gz_pair_k21", 5), ("gz_trio_k21", 2),
                                                                       ("gz_trio_k21", 4)])
def test_dist_driver_matches_reference(name, world, counter, manifest, synth_dir, tmp_path):
    """vafc_dist.run over gloo ranks (the oracle as the per-rank counter on
    CPU; the HIP counter, every rank on device 0, in the GPU suite): plain
    files split into byte ranges over the ranks, gzip files dealt whole, the
    counts all-reduced; rank 0's .vaf and -v tallies equal the reference's.
    Well-formed plain files must split without a fallback; the malformed ones
    must fall back to a whole-file recount on rank 0."""
    import hashlib
    entry = next(c for c in manifest["cases"] if c["name"] == name)
    rcs, stats, data, err, calls = _run_driver(entry, synth_dir, tmp_path, counter, world)
    assert rcs == [entry["exit"]] * world, err[-2000:]
    assert hashlib.md5(data).hexdigest() == entry["vaf_md5"]
    for key in ("bases", "seqs", "kmers"):
        assert stats.get(key) == entry["stats"].get(key), key
    assert err.count("collisions detected") == (1 if entry["collision_warning"] else 0)
    # the reference's message sequence on rank 0: one Processing line per input, in argv order
    inputs = [a for a in entry["argv"] if a.endswith((".fq", ".gz", ".fa"))]
    assert [ln.split("Processing ")[1][:-3] for ln in err.splitlines() if "Processing " in ln] == inputs
    assert "Ranks:" not in err
    # count_fastq_kmers' -v line (vaf-counter.c:573-578): one per input that
    # opens, in argv order, the files' sequences and bases adding up to the totals
    from conftest import case_dir
    proc = [ln for ln in err.splitlines() if ln.startswith("[V::count_fastq_kmers] Processed ")]
    if "-v" in entry["argv"] and entry["exit"] == 0:
        opened = [i for i in inputs if os.path.exists(os.path.join(case_dir(entry, synth_dir), i))]
        assert [ln.split("Processed ")[1].split(": ")[0] for ln in proc] == opened, proc
        assert sum(int(ln.split(": ")[1].split()[0]) for ln in proc) == stats["seqs"]
        assert sum(int(ln.split(" sequences, ")[1].split()[0]) for ln in proc) == stats["bases"]
    else:
        assert not proc
    if counter == "oracle":
        if name in DIST_CLEAN:
            assert all(c["restores"] == 0 and c["ranges"] >= 1 for c in calls), calls
        if name in DIST_GZ_CLEAN:   # every gzip file split into shares: nothing counted whole, nothing redone
            assert all(c["restores"] == 0 and c["whole"] == 0 for c in calls), calls
            assert sum(c["gz_shares"] for c in calls) >= (world if name != "edge_gz" else 1), calls
            # odd worlds hold their scans' chunks: every share counted in one pass
            assert sum(c["gz_held"] for c in calls) == (sum(c["gz_shares"] for c in calls) if world % 2 else 0)
        if name.startswith("mal_") or name == "truncated":
            assert all(c["restores"] >= 1 for c in calls), calls
        if name in DIST_GZ_WAVES:   # a lone rank counts its file whole, a group splits it into shares
            import vafc_dist as D
            plan = [(2, os.path.getsize(os.path.join(case_dir(entry, synth_dir), f))) for f in inputs]
            whole, split, most = 0, 0, 0
            i = 0
            while i < len(plan):
                wave = D._gz_wave(plan, i, world) or [i]
                groups = D.gz_groups([plan[f][1] for f in wave], world) if len(wave) > 1 else [(0, world)]
                for _, n in groups:
                    whole += n == 1
                    split += n > 1
                    most += n if n > 1 else 0
                i = wave[-1] + 1
            assert all(c["restores"] == 0 for c in calls), calls
            assert sum(c["whole"] for c in calls) == whole, calls
            assert split <= sum(c["gz_shares"] for c in calls) <= most, calls


def test_dist_driver_usage_and_missing_patterns(tmp_path):
    """Usage errors and an unreadable pattern file exit 1 on every rank before
    any collective (single-rank path of the same driver)."""
    import vafc_dist as D
    lines = []
    assert D.run(["-p", "p.txt"], None, err=lines.append) == 1 and "Usage" in "".join(lines)
    lines = []
    assert D.run(["-p", str(tmp_path / "none.txt"), "-o", str(tmp_path / "o.vaf"), "x.fq"], None,
                 err=lines.append) == 1
    assert "failed to load pattern file" in "".join(lines)


@pytest.mark.parametrize("world", [2, 3])
def test_dist_driver_gzip_bad_crc_falls_back(world, manifest, synth_dir, tmp_path):
    """A gzip file whose middle member fails its CRC-32 check: the shares are
    counted, the combined check fails, and the file is counted whole by one
    rank -- the same .vaf as the single-rank driver (gzread's output around a
    failed check is buffer-dependent, so there is no reference golden)."""
    entry = {"name": "gz_badcrc", "argv": ["-v", "-k", "21", "-t", "2", "-p", "grch38_k21.txt", "c1_10k_badcrc.fq.gz"],
             "inputs": ["synth:grch38_k21.txt", "synth:c1_10k_badcrc.fq.gz"]}
    (tmp_path / "w1").mkdir()
    rcs1, stats1, data1, _, _ = _run_driver(entry, synth_dir, tmp_path / "w1", "oracle", 1)
    rcs, stats, data, err, calls = _run_driver(entry, synth_dir, tmp_path, "oracle", world)
    assert rcs == [0] * world and rcs1 == [0], err[-2000:]
    assert data == data1 and stats == stats1
    assert all(c["restores"] >= 1 for c in calls), calls
    assert sum(c["whole"] for c in calls) == 1 and sum(c["gz_shares"] for c in calls) >= 2, calls
    assert sum(c["gz_held"] for c in calls) == (sum(c["gz_shares"] for c in calls) if world % 2 else 0)


def test_gz_hold_budget(monkeypatch):
    """The driver's held-share budget ($VAFC_GZ_HOLD bytes; default a quarter
    of the available memory over the node's ranks, at most 32 GiB; a bad
    value turns holding off rather than failing the run)."""
    import vafc_dist as D
    monkeypatch.setenv("VAFC_GZ_HOLD", "12345")
    assert D.gz_hold_budget() == 12345
    monkeypatch.setenv("VAFC_GZ_HOLD", "-1")
    assert D.gz_hold_budget() == 0
    monkeypatch.setenv("VAFC_GZ_HOLD", "lots")
    assert D.gz_hold_budget() == 0
    monkeypatch.delenv("VAFC_GZ_HOLD")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    one = D.gz_hold_budget()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    eight = D.gz_hold_budget()
    assert 0 < one <= 32 << 30 and eight <= one


def test_dist_driver_gzip_wave_bad_crc_falls_back(manifest, synth_dir, tmp_path):
    """A wave of two gzip files over three ranks, the first with a middle
    member that fails its CRC-32 check: its group of ranks counts shares, the
    combined check fails and its leader counts it whole, while the other
    file's group is not disturbed -- the same .vaf as the single-rank driver."""
    entry = {"name": "gz_wave_badcrc", "argv": ["-v", "-k", "21", "-t", "2", "-p", "grch38_k21.txt",
                                                "c1_10k_badcrc.fq.gz", "c1_10k_multi.fq.gz"],
             "inputs": ["synth:grch38_k21.txt", "synth:c1_10k_badcrc.fq.gz", "synth:c1_10k_multi.fq.gz"]}
    (tmp_path / "w1").mkdir()
    rcs1, stats1, data1, _, _ = _run_driver(entry, synth_dir, tmp_path / "w1", "oracle", 1)
    rcs, stats, data, err, calls = _run_driver(entry, synth_dir, tmp_path, "oracle", 3)
    assert rcs == [0] * 3 and rcs1 == [0], err[-2000:]
    assert data == data1 and stats == stats1
    assert sum(c["restores"] for c in calls) >= 1, calls
    assert sum(c["whole"] for c in calls) == 2, calls   # the bad file's recount, the other file's lone rank


def test_gz_groups_cover_the_ranks():
    """gz_groups: every rank in exactly one group, in file order, each file at
    least one rank, the spare ranks shared by compressed size; _gz_wave: runs
    of consecutive gzip files, at most one per rank, two or more."""
    import vafc_dist as D
    for sizes in ([1, 1], [10, 30], [5, 5, 5], [100, 1], [0, 0, 0], [7, 3, 9, 1]):
        for world in range(len(sizes), 10):
            g = D.gz_groups(sizes, world)
            assert [r0 for r0, _ in g] == [sum(n for _, n in g[:f]) for f in range(len(sizes))]
            assert sum(n for _, n in g) == world and all(n >= 1 for _, n in g)
            big, small = max(range(len(sizes)), key=lambda f: sizes[f]), min(range(len(sizes)), key=lambda f: sizes[f])
            assert g[big][1] >= g[small][1]
    plan = [(2, 5), (2, 5), (1, 9), (2, 5), (2, 5), (2, 5), (0, -1)]
    assert D._gz_wave(plan, 0, 4) == [0, 1]
    assert D._gz_wave(plan, 2, 4) == []
    assert D._gz_wave(plan, 3, 2) == [3, 4] and D._gz_wave(plan, 5, 2) == []
    assert D._gz_wave(plan, 0, 1) == []
