"""Multi-GPU product path (vc_create_multi): several shards --
each a replica of the static table plus its own counts -- take the host batches
round robin, and vc_finish reduces them (same-device shards summed on the
device, then one RCCL reduce over the devices) before the .vaf is written.

On a one-GPU box the shards share device 0, which runs the round-robin dealing
and the on-device shard sum (no RCCL: one distinct device).  Variants over two
distinct devices ([0, 1], [0, 1, 0]: a cross-device ncclReduce, the non-root
zeroing, batches dealt across two hipSetDevice contexts) run where the box has
two GPUs and are skipped otherwise.  The results must be bit-identical to the
reference's goldens and to the oracle."""
import hashlib
import os

import numpy as np
import pytest

from conftest import PRODUCT_CLI, run_cli

pytestmark = pytest.mark.gpu


def _n_devices():
    import torch
    return torch.cuda.device_count()


two_gpus = pytest.mark.skipif("_n_devices() < 2", reason="needs two GPUs")

# golden cases covering plain/gz input, -b 1, two files, the stop rule, empty input
SHARDED_CASES = ["c1_plumbing_k21", "c1_plumbing_k21_gz", "c1_k21_b1", "pe_k31", "missing_file",
                 "mal_gbbbgbbbg", "mal_gbbbgbbbg_b1", "mal_bbbg_b1", "edge_k15", "edge_gz", "truncated",
                 "empty_reads", "empty_patterns", "pal_k21", "pal_k16"]

MODES = {
    # sequential reader, 3 kB batches dealt over two shards
    "batches_2shards": {"VAFC_DEVICES": "0,0", "VAFC_BATCH_BYTES": "3000"},
    # the parallel reader's pieces (4 kB) dealt over three shards
    "pieces_3shards": {"VAFC_DEVICES": "0,0,0", "VAFC_INGEST_MIN": "0", "VAFC_INGEST_PIECE": "4096"},
}


@two_gpus
@pytest.mark.parametrize("devices", ["0,1", "0,1,0"])
@pytest.mark.parametrize("name", ["c1_plumbing_k21", "c1_plumbing_k21_gz", "c1_k21_b1", "pe_k31", "mal_gbbbgbbbg_b1"])
def test_sharded_cli_two_devices(name, devices, manifest, synth_dir, tmp_path):
    """VAFC_DEVICES over two distinct GPUs: batches dealt across devices, one
    cross-device RCCL reduce; the .vaf equals the reference's."""
    entry = next(c for c in manifest["cases"] if c["name"] == name)
    env = dict(os.environ, VAFC_DEVICES=devices, VAFC_BATCH_BYTES="3000")
    rc, stats, data, err = run_cli(PRODUCT_CLI, entry, synth_dir, tmp_path, env=env)
    assert rc == entry["exit"], err[-2000:]
    assert hashlib.md5(data).hexdigest() == entry["vaf_md5"]
    for key in ("bases", "seqs", "kmers"):
        assert stats.get(key) == entry["stats"].get(key), key


@pytest.mark.parametrize("mode", sorted(MODES))
@pytest.mark.parametrize("name", SHARDED_CASES)
def test_sharded_cli_matches_reference(name, mode, manifest, synth_dir, tmp_path):
    entry = next(c for c in manifest["cases"] if c["name"] == name)
    env = dict(os.environ, **MODES[mode])
    rc, stats, data, err = run_cli(PRODUCT_CLI, entry, synth_dir, tmp_path, env=env)
    assert rc == entry["exit"], err[-2000:]
    assert hashlib.md5(data).hexdigest() == entry["vaf_md5"]
    for key in ("bases", "seqs", "kmers"):
        assert stats.get(key) == entry["stats"].get(key), key
    if name == "c1_plumbing_k21":
        assert "Shards:" in err


def _panel_and_reads(tmp_path, n_reads, k=21, f_snp=0.5):
    import vafc
    import vafc_synth as S
    panel = S.make_panel(S.synthetic_bed(3000))
    pat = str(tmp_path / "p.txt")
    panel.write_patterns(pat, k)
    db = vafc.load_patterns(pat)
    reads = S.gen_reads(panel, n_reads, f_snp=f_snp)
    return pat, db, reads


@pytest.mark.parametrize("devices", [[0, 0, 0], pytest.param([0, 1], marks=two_gpus),
                                     pytest.param([0, 1, 0], marks=two_gpus)])
def test_multi_shard_blocks_vs_oracle(tmp_path, devices):
    """count_block batches dealt over the shards; finish() reduces, is
    idempotent (a second finish after the non-root zeroing gives the same
    totals), and reset() clears every shard."""
    import vafc
    import vafc_synth as S
    import oracle as O
    pat, db, reads = _panel_and_reads(tmp_path, 21_000)
    seq, offs, lens = S.pack_reads(reads)
    want, km_want = O.Oracle(21, pattern_fn=pat).count_reads(seq, offs, lens)
    keys, vals, _ = db.keys(21)
    m = vafc.KmerMap(21, keys, vals, db.n, devices=devices)
    assert [d for d, _ in m.shards()] == devices
    for rep in range(2):
        for i in range(0, len(reads), 3000):
            s, o, ln = S.pack_reads(reads[i:i + 3000])
            m.count_block(s, o, ln)
        got, km = m.finish()
        assert km == km_want and np.array_equal(got, want), rep
        again, km2 = m.finish()
        assert km2 == km_want and np.array_equal(again, want)
        m.reset()
    assert all(b >= 4 for _, b in m.shards())
    z, kz = m.finish()
    assert kz == 0 and int(z.sum()) == 0
    m.close()


def test_multi_shard_count_file_vs_oracle(tmp_path):
    """vc_count_file on a 300k-read FASTQ (parallel reader, 16 MB pieces) over two
    shards equals the oracle's whole-file pass; both shards counted pieces."""
    import vafc
    import vafc_synth as S
    import oracle as O
    panel = S.grch38_panel()
    pat = str(tmp_path / "p.txt")
    panel.write_patterns(pat, 21)
    fq = str(tmp_path / "r.fq")
    S.write_fastq(fq, panel, 300_000, seed=9, f_snp=0.2)
    db = vafc.load_patterns(pat)
    m = vafc.create_combined_kmer_map(db, 21, devices=[0, 0])
    st = m.count_file(fq, 10_000_000, 4)
    got, km = m.finish()
    orc = O.Oracle(21, pattern_fn=pat)
    want = np.zeros(2 * orc.n_patterns + 2, np.uint32)
    rc, bases, seqs, km_want = orc.count_file(fq, 10_000_000, want)
    assert (st.bases, st.seqs) == (bases, seqs)
    assert km == km_want
    assert np.array_equal(got, want[: 2 * orc.n_patterns])
    assert all(b >= 2 for _, b in m.shards())
    m.close()


def test_multi_shard_counts_wrap_like_u32(tmp_path):
    """The shard sum and the RCCL reduce add modulo 2^32 (the reference's u32
    counters): counts bound near 2^32 on shard 0 wrap exactly."""
    import torch
    import vafc
    import vafc_synth as S
    import oracle as O
    pat, db, reads = _panel_and_reads(tmp_path, 6000, f_snp=1.0)
    seq, offs, lens = S.pack_reads(reads)
    want, km_want = O.Oracle(21, pattern_fn=pat).count_reads(seq, offs, lens)
    keys, vals, _ = db.keys(21)
    m = vafc.KmerMap(21, keys, vals, db.n, devices=[0, 0])
    start = np.full(2 * db.n, 0xFFFFFFFE, np.uint32)
    t = torch.from_numpy(start.view(np.int32).copy()).to("cuda:0")
    tally = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    m.bind_outputs(t.data_ptr(), tally.data_ptr())
    for i in range(0, len(reads), 1000):
        s, o, ln = S.pack_reads(reads[i:i + 1000])
        m.count_block(s, o, ln)
    got, km = m.finish()
    assert km == km_want
    assert np.array_equal(got, ((start.astype(np.uint64) + want) & 0xFFFFFFFF).astype(np.uint32))
    m.close()


def test_multi_shard_count_device_vs_oracle(tmp_path):
    """vc_count_device on a multi-shard counter deals device batches round robin
    over the shards on the reads' device; the sum equals the oracle."""
    import torch
    import vafc
    import vafc_synth as S
    import oracle as O
    pat, db, reads = _panel_and_reads(tmp_path, 12_000)
    seq, offs, lens = S.pack_reads(reads)
    want, km_want = O.Oracle(21, pattern_fn=pat).count_reads(seq, offs, lens)
    keys, vals, _ = db.keys(21)
    m = vafc.KmerMap(21, keys, vals, db.n, devices=[0, 0, 0])
    d_seq = torch.from_numpy(seq).to("cuda:0")
    d_offs = torch.from_numpy(offs.view(np.int64)).to("cuda:0")
    d_lens = torch.from_numpy(lens.view(np.int32)).to("cuda:0")
    torch.cuda.synchronize()
    for a in range(0, len(reads), 2000):
        b = min(len(reads), a + 2000)
        m.count_device(d_seq.data_ptr(), seq.size, d_offs.data_ptr() + 8 * a, d_lens.data_ptr() + 4 * a, b - a)
    got, km = m.finish()
    assert km == km_want and np.array_equal(got, want)
    assert [b for _, b in m.shards()] == [2, 2, 2]
    m.close()
