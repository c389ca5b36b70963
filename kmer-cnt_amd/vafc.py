"""Python host mirror of the MI355X vaf-counter hot path (ctypes over libvafc.so).

This mirrors the reference's own interface for the path, function by function
(gerbenvoshol/kmer-cnt, vaf-counter.c):

=============================  ==========================================  ===================
reference (vaf-counter.c)       here                                        C ABI (include/vafc.h)
=============================  ==========================================  ===================
load_patterns        :149      ``load_patterns(fn)``                       vc_patterns_load
create_combined_kmer_map :198  ``create_combined_kmer_map(db, k)``         vc_patterns_keys + vc_create
count_fastq_kmers    :550      ``count_fastq_kmers(fn, k, t, b, map, db)`` vc_count_file
worker_pipeline steps 1+2      ``KmerMap.count_block / count_device``      vc_count_block / vc_count_device
main  :584-738                 ``main(argv)``                              (all of the above) + vc_write_vaf
=============================  ==========================================  ===================

Everything that counts goes through the HIP kernels of ``libvafc.so``; if the
library is missing this module raises ``VafcError`` -- there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VAFC_LIB", os.path.join(_HERE, "lib", "libvafc.so"))

# vc_count_device's stream argument for the counter's own stream (VC_STREAM_CTX)
STREAM_CTX = (1 << 64) - 1

VC_OK, VC_EINVAL, VC_ENOMEM, VC_EHIP, VC_ENODEV, VC_EIO, VC_ETOOMANY, VC_EFULL = 0, -1, -2, -3, -4, -5, -6, -7

# every symbol include/vafc.h declares
EXPORTS = (
    "vc_patterns_load", "vc_patterns_free", "vc_patterns_count", "vc_patterns_keys",
    "vc_write_vaf", "vc_pattern_fields", "vc_free", "vc_create", "vc_destroy",
    "vc_count_block", "vc_count_device", "vc_finish", "vc_reset", "vc_device_counts",
    "vc_bind_outputs", "vc_device_tally", "vc_stream", "vc_set_timing", "vc_kernel_ms",
    "vc_table_info", "vc_create_multi", "vc_shard_count", "vc_shard_info", "vc_count_file",
    "vc_count_file_range", "vc_scan_file_range", "vc_ingest_profile", "vc_ingest_profile_ex", "vc_scan_file", "vc_scan_file_parallel",
    "vc_scan_records", "vc_reserve_file_ingest",
    "vc_gz_inflate_parallel", "vc_gz_inflate_zlib", "vc_gz_crc32", "vc_gz_crc32_combine",
    "vc_gz_share_scan", "vc_count_gz_share", "vc_scan_gz_share",
    "vc_gz_share_open", "vc_count_gz_share_held", "vc_scan_gz_share_held", "vc_gz_share_close",
    "vc_fasta_load", "vc_fasta_count", "vc_fasta_name", "vc_fasta_seq", "vc_fasta_data", "vc_fasta_free",
    "vc_count_candidates", "vc_set_nt4_decode",
    "vc_kc_create", "vc_kc_set_partition", "vc_kc_slots", "vc_kc_histogram", "vc_kc_histogram2",
    "vc_kc_track_first", "vc_yak_bloom_select",
    "vc_vafset_create", "vc_vafset_free", "vc_vafset_add", "vc_vafset_add_many", "vc_vafset_add_arrays",
    "vc_vafset_count",
    "vc_vafset_name", "vc_vafset_snps", "vc_corr_matrix", "vc_corr_matrix_raw", "vc_corr_write", "vc_corr_tree",
    "vc_synth_reads",
    "vc_debug_decode", "vc_strerror", "vc_version", "vc_build_id",
)


class VafcError(RuntimeError):
    def __init__(self, what, code=None):
        if code is not None:
            what = "%s: %s (%d)" % (what, lib().vc_strerror(code).decode(), code)
        super().__init__(what)
        self.code = code


class FileStats(C.Structure):
    _fields_ = [("bases", C.c_uint64), ("seqs", C.c_uint64), ("blocks", C.c_uint64),
                ("seconds", C.c_double)]


class RangeInfo(C.Structure):
    """vc_range_info: where one rank's byte range of a file began and ended
    (include/vafc.h, vc_count_file_range)."""
    _fields_ = [("first", C.c_uint64), ("next", C.c_uint64), ("errs", C.c_uint64),
                ("stopped", C.c_uint32), ("whole", C.c_uint32)]


class GzShareInfo(C.Structure):
    """vc_gz_share_info: one rank's share of a gzip stream (vc_gz_share_scan)."""
    _fields_ = [("start_bit", C.c_uint64), ("end_bit", C.c_uint64), ("text_len", C.c_uint64),
                ("ok", C.c_uint32), ("ended", C.c_uint32)]


class GzShareCrc(C.Structure):
    """vc_gz_share_crc: the CRC-32 accounting of one share (vc_count_gz_share)."""
    _fields_ = [("events", C.c_uint32), ("head_crc", C.c_uint32), ("head_len", C.c_uint64),
                ("head_expect_crc", C.c_uint32), ("head_expect_isize", C.c_uint32), ("tail_crc", C.c_uint32),
                ("tail_len", C.c_uint64), ("crc_error", C.c_uint32), ("complete", C.c_uint32)]

    def as_dict(self):
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


NO_OFFSET = (1 << 64) - 1   # vc_range_info's UINT64_MAX
GZ_WSIZE = 32768            # deflate's window; symbols 0x8000 | i name byte i of the window before a share


_lib = None
P = C.c_void_p


def lib():
    """Load libvafc.so (built by ``make -C kmer-cnt_amd/csrc``); raise if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VafcError("libvafc.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
    # torch bundles its own libamdhip64.so.7; loading it first makes libvafc.so
    # bind to that same runtime (one HIP runtime per process).  Loading
    # libvafc.so first would let torch map a second copy later.
    if os.environ.get("VAFC_NO_TORCH", "0") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = C.CDLL(LIB_PATH)
    sig = {
        "vc_patterns_load": (C.c_int, [C.c_char_p, C.POINTER(P)]),
        "vc_patterns_free": (None, [P]),
        "vc_patterns_count": (C.c_int, [P]),
        "vc_patterns_keys": (C.c_int, [P, C.c_int, C.POINTER(P), C.POINTER(P),
                                       C.POINTER(C.c_size_t), C.POINTER(C.c_int)]),
        "vc_write_vaf": (C.c_int, [P, P, C.c_char_p]),
        "vc_pattern_fields": (C.c_int, [P, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_int),
                                        C.POINTER(C.c_char_p), C.POINTER(C.c_char),
                                        C.POINTER(C.c_char), C.POINTER(C.c_char_p),
                                        C.POINTER(C.c_char_p)]),
        "vc_free": (None, [P]),
        "vc_create": (C.c_int, [C.POINTER(P), C.c_int, P, P, C.c_size_t, C.c_uint32, C.c_int]),
        "vc_destroy": (None, [P]),
        "vc_create_multi": (C.c_int, [C.POINTER(P), C.c_int, P, P, C.c_size_t, C.c_uint32, P, C.c_int]),
        "vc_shard_count": (C.c_int, [P]),
        "vc_shard_info": (C.c_int, [P, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_uint64)]),
        "vc_count_block": (C.c_int, [P, P, C.c_size_t, P, P, C.c_uint64]),
        "vc_count_device": (C.c_int, [P, P, C.c_size_t, P, P, C.c_uint64, P]),
        "vc_finish": (C.c_int, [P, P, C.POINTER(C.c_uint64)]),
        "vc_reset": (C.c_int, [P]),
        "vc_device_counts": (P, [P]),
        "vc_bind_outputs": (C.c_int, [P, P, P]),
        "vc_device_tally": (P, [P]),
        "vc_stream": (P, [P]),
        "vc_set_timing": (C.c_int, [P, C.c_int]),
        "vc_kernel_ms": (C.c_int, [P, C.POINTER(C.c_float)]),
        "vc_table_info": (C.c_int, [P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_uint64)]),
        "vc_count_file": (C.c_int, [P, C.c_char_p, C.c_int, C.c_int, C.POINTER(FileStats)]),
        "vc_count_file_range": (C.c_int, [P, C.c_char_p, C.c_uint64, C.c_uint64, C.c_int, C.c_int,
                                          C.POINTER(FileStats), C.POINTER(RangeInfo)]),
        "vc_scan_file_range": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_uint64,
                                         C.c_uint64, C.POINTER(FileStats), C.POINTER(RangeInfo), P, C.c_size_t,
                                         P, C.c_size_t]),
        "vc_ingest_profile": (C.c_uint64, [P]),
        "vc_ingest_profile_ex": (C.c_uint64, [P, C.c_int]),
        "vc_scan_file": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.POINTER(FileStats), P, C.c_size_t,
                                   P, C.c_size_t]),
        "vc_scan_file_parallel": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                            C.POINTER(FileStats), P, C.c_size_t, P, C.c_size_t]),
        "vc_scan_records": (C.c_int64, [C.c_char_p, P, C.c_int64]),
        "vc_gz_inflate_parallel": (C.c_int64, [C.c_char_p, C.c_int, C.c_uint64, P, C.c_uint64, P]),
        "vc_gz_inflate_zlib": (C.c_int64, [C.c_char_p, P, C.c_uint64]),
        "vc_gz_crc32": (C.c_uint32, [C.c_uint32, P, C.c_uint64]),
        "vc_gz_crc32_combine": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint64]),
        "vc_gz_share_scan": (C.c_int, [C.c_char_p, C.c_uint64, C.c_uint64, C.c_int, C.c_uint64,
                                       C.POINTER(GzShareInfo), P]),
        "vc_count_gz_share": (C.c_int, [P, C.c_char_p, C.c_int, C.c_uint64, P, C.c_uint64, C.c_int, C.c_int,
                                        C.POINTER(FileStats), C.POINTER(RangeInfo), C.POINTER(GzShareCrc)]),
        "vc_scan_gz_share": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_uint64, P, C.c_uint64, C.c_int, C.c_int,
                                       C.POINTER(FileStats), C.POINTER(RangeInfo), C.POINTER(GzShareCrc),
                                       P, C.c_size_t, P, C.c_size_t]),
        "vc_gz_share_open": (C.c_int, [P, C.c_char_p, C.c_uint64, C.c_uint64, C.c_int, C.c_uint64, C.c_uint64,
                                       C.POINTER(GzShareInfo), P, C.POINTER(P)]),
        "vc_count_gz_share_held": (C.c_int, [P, P, C.c_int, P, C.c_uint64, C.c_int, C.c_int, C.POINTER(FileStats),
                                             C.POINTER(RangeInfo), C.POINTER(GzShareCrc)]),
        "vc_scan_gz_share_held": (C.c_int, [P, C.c_int, C.c_int, P, C.c_uint64, C.c_int, C.c_int,
                                            C.POINTER(FileStats), C.POINTER(RangeInfo), C.POINTER(GzShareCrc),
                                            P, C.c_size_t, P, C.c_size_t]),
        "vc_gz_share_close": (None, [P]),
        "vc_reserve_file_ingest": (C.c_int, [P, C.c_int]),
        "vc_fasta_load": (C.c_int, [C.c_char_p, C.POINTER(P)]),
        "vc_fasta_count": (C.c_int, [P]),
        "vc_fasta_name": (C.c_char_p, [P, C.c_int]),
        "vc_fasta_seq": (P, [P, C.c_int, C.POINTER(C.c_uint32)]),
        "vc_fasta_data": (C.c_int, [P, C.POINTER(P), C.POINTER(C.c_size_t), C.POINTER(P), C.POINTER(P)]),
        "vc_fasta_free": (None, [P]),
        "vc_set_nt4_decode": (C.c_int, [P, C.c_int]),
        "vc_count_candidates": (C.c_int, [C.c_int, P, C.c_size_t, P, P, C.c_uint64, P, C.c_size_t, P,
                                          C.c_int]),
        "vc_kc_create": (C.c_int, [C.POINTER(P), C.c_int, C.c_uint64, C.c_int]),
        "vc_kc_set_partition": (C.c_int, [P, C.c_uint32, C.c_uint32]),
        "vc_kc_slots": (C.c_uint64, [P]),
        "vc_kc_histogram": (C.c_int, [P, P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "vc_kc_histogram2": (C.c_int, [P, P, C.c_uint32, C.c_uint64, C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_uint64)]),
        "vc_kc_track_first": (C.c_int, [P, C.c_int]),
        "vc_yak_bloom_select": (C.c_int, [P, C.c_int, C.c_int, C.c_int]),
        "vc_vafset_create": (C.c_int, [C.POINTER(P)]),
        "vc_vafset_free": (None, [P]),
        "vc_vafset_add": (C.c_int, [P, C.c_char_p]),
        "vc_vafset_add_many": (C.c_int, [P, P, C.c_int, C.c_int, C.POINTER(C.c_int), P]),
        "vc_vafset_add_arrays": (C.c_int, [P, C.c_char_p, P, P, C.c_int]),
        "vc_vafset_count": (C.c_int, [P]),
        "vc_vafset_name": (C.c_char_p, [P, C.c_int]),
        "vc_vafset_snps": (C.c_int, [P, C.c_int]),
        "vc_corr_matrix": (C.c_int, [P, C.c_int, C.c_int, P, C.c_int, C.POINTER(C.c_float)]),
        "vc_corr_matrix_raw": (C.c_int, [P, P, P, C.c_int, C.c_size_t, C.c_int, C.c_int, P, C.c_int,
                                         C.POINTER(C.c_float)]),
        "vc_corr_write": (C.c_int, [P, P, C.c_char_p]),
        "vc_corr_tree": (C.c_int, [P, P, C.c_char_p]),
        "vc_synth_reads": (C.c_int, [P, P, P, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64,
                                     C.c_double, P, P, C.c_uint32, P]),
        "vc_debug_decode": (C.c_int, [P, C.c_size_t, P, P, C.c_uint64, P, P]),
        "vc_strerror": (C.c_char_p, [C.c_int]),
        "vc_version": (C.c_int, []),
        "vc_build_id": (C.c_char_p, []),
    }
    older = "VAFC_LIB" in os.environ      # A/B against an older build: bind what it has
    for name, (res, args) in sig.items():
        if older and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def tree_build_id(root: str = None) -> str:
    """The build id of the sources in this tree (the Makefile's BUILD_ID): the
    first 16 hex digits of sha256 over every file of kmer-cnt_amd/csrc in name
    order, then include/vafc.h."""
    import hashlib
    csrc = os.path.join(_HERE, "csrc")
    root = root or os.path.dirname(_HERE)
    h = hashlib.sha256()
    for fn in sorted(os.listdir(csrc)):
        p = os.path.join(csrc, fn)
        if os.path.isfile(p):
            with open(p, "rb") as f:
                h.update(f.read())
    with open(os.path.join(root, "include", "vafc.h"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def binary_build_id(path: str):
    """The "VAFC_BUILD_ID=<hex>" string embedded in a built binary (read from
    the file, not loaded), or None."""
    import re
    try:
        with open(path, "rb") as f:
            m = re.search(rb"VAFC_BUILD_ID=([0-9a-f]{16})", f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def check_build(paths=None) -> None:
    """Raise VafcError unless every product binary carries the tree's build id."""
    want = tree_build_id()
    lib_dir = os.path.join(_HERE, "lib")
    paths = paths or [os.path.join(lib_dir, f) for f in BINARIES]
    bad = [(os.path.basename(p), binary_build_id(p)) for p in paths if binary_build_id(p) != want]
    if bad:
        raise VafcError("stale or missing build: the tree's sources hash to %s, but %s; "
                        "rebuild with make -C kmer-cnt_amd/csrc" % (
                            want, ", ".join("%s has %s" % (n, i) for n, i in bad)))


BINARIES = ("libvafc.so", "vaf-counter", "snp-pattern-gen", "kc-c4", "yak-count", "correlation-matrix")


def _ck(rc, what):
    if rc != VC_OK:
        raise VafcError(what, rc)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(P)


# --------------------------------------------------------------------------
# pattern database
# --------------------------------------------------------------------------

class PatternDB:
    """patterns.txt records (vaf-counter.c:92-108,149-184)."""

    def __init__(self, handle):
        self._h = handle

    @property
    def n(self) -> int:
        return lib().vc_patterns_count(self._h)

    def __len__(self):
        return self.n

    def record(self, i: int):
        chr_, rsid, rk, ak = C.c_char_p(), C.c_char_p(), C.c_char_p(), C.c_char_p()
        start, ref, alt = C.c_int(), C.c_char(), C.c_char()
        _ck(lib().vc_pattern_fields(self._h, i, C.byref(chr_), C.byref(start), C.byref(rsid),
                                    C.byref(ref), C.byref(alt), C.byref(rk), C.byref(ak)),
            "vc_pattern_fields")
        return (chr_.value.decode("latin-1"), start.value, rsid.value.decode("latin-1"),
                ref.value, alt.value, rk.value, ak.value)

    def keys(self, k: int):
        """(keys uint64[m], vals uint32[m], n_collisions) -- create_combined_kmer_map's content."""
        kp, vp, n, coll = P(), P(), C.c_size_t(), C.c_int()
        _ck(lib().vc_patterns_keys(self._h, k, C.byref(kp), C.byref(vp), C.byref(n), C.byref(coll)),
            "vc_patterns_keys")
        try:
            m = n.value
            keys = np.ctypeslib.as_array(C.cast(kp, C.POINTER(C.c_uint64)), (m,)).copy() if m else \
                np.zeros(0, np.uint64)
            vals = np.ctypeslib.as_array(C.cast(vp, C.POINTER(C.c_uint32)), (m,)).copy() if m else \
                np.zeros(0, np.uint32)
        finally:
            lib().vc_free(kp)
            lib().vc_free(vp)
        return keys, vals, coll.value

    def write_vaf(self, counts: np.ndarray, path: str) -> None:
        counts = np.ascontiguousarray(counts, dtype=np.uint32)
        assert counts.size >= 2 * self.n
        _ck(lib().vc_write_vaf(self._h, _ptr(counts), path.encode()), "vc_write_vaf")

    def close(self):
        if self._h:
            lib().vc_patterns_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_patterns(fn: str) -> PatternDB:
    """load_patterns (vaf-counter.c:149): raises VafcError(VC_EIO) if unreadable."""
    h = P()
    _ck(lib().vc_patterns_load(fn.encode(), C.byref(h)), "load_patterns(%s)" % fn)
    return PatternDB(h)


# --------------------------------------------------------------------------
# device k-mer map + counters
# --------------------------------------------------------------------------

class KmerMap:
    """The device-resident static key table + counts (kmer_cnt_t + pattern_t counters).

    ``devices`` (a list of device ids, repeats allowed) makes a multi-GPU
    counter (vc_create_multi): one table replica + counts per entry, host
    batches dealt round robin, one RCCL reduce in ``finish()``."""

    def __init__(self, k: int, keys: np.ndarray, vals: np.ndarray, n_patterns: int, device: int = 0,
                 devices=None):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        vals = np.ascontiguousarray(vals, dtype=np.uint32)
        self.k, self.n_patterns, self.device = k, int(n_patterns), device
        h = P()
        if devices:
            devs = np.ascontiguousarray(devices, dtype=np.int32)
            self.device = int(devs[0])
            _ck(lib().vc_create_multi(C.byref(h), k, _ptr(keys), _ptr(vals), keys.size, self.n_patterns,
                                      _ptr(devs), devs.size), "vc_create_multi")
        else:
            _ck(lib().vc_create(C.byref(h), k, _ptr(keys), _ptr(vals), keys.size, self.n_patterns, device),
                "vc_create")
        self._h = h
        self.n_collisions = 0

    def shards(self):
        """[(device, host batches counted)] per shard."""
        out = []
        for i in range(lib().vc_shard_count(self._h)):
            d, b = C.c_int(), C.c_uint64()
            _ck(lib().vc_shard_info(self._h, i, C.byref(d), C.byref(b)), "vc_shard_info")
            out.append((d.value, b.value))
        return out

    # -- counting -----------------------------------------------------------
    def count_block(self, seq: np.ndarray, offs: np.ndarray, lens: np.ndarray) -> None:
        seq = np.ascontiguousarray(seq, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        assert offs.size == lens.size
        _ck(lib().vc_count_block(self._h, _ptr(seq), seq.size, _ptr(offs), _ptr(lens), offs.size),
            "vc_count_block")

    def count_device(self, seq_ptr: int, seq_bytes: int, offs_ptr: int, lens_ptr: int,
                     n_reads: int, stream: int = 0) -> None:
        """Count HBM-resident reads on `stream` (a hipStream_t handle): 0 is HIP's
        null stream, i.e. torch's default stream, so reads written by torch on
        its current stream are ordered before the count when that handle is
        passed (torch.cuda.current_stream().cuda_stream); STREAM_CTX is the
        counter's own stream."""
        _ck(lib().vc_count_device(self._h, P(seq_ptr), seq_bytes, P(offs_ptr), P(lens_ptr),
                                  n_reads, P(stream) if stream else None), "vc_count_device")

    def reserve_file_ingest(self, n_thread: int = 4) -> None:
        """Allocate count_file's parallel-reader buffers now (vc_reserve_file_ingest);
        without it they are allocated by the reader's workers on first use."""
        _ck(lib().vc_reserve_file_ingest(self._h, n_thread), "vc_reserve_file_ingest")

    def count_file(self, fn: str, block_size: int = 10_000_000, n_thread: int = 4) -> FileStats:
        st = FileStats()
        rc = lib().vc_count_file(self._h, fn.encode(), block_size, n_thread, C.byref(st))
        if rc == VC_EIO:
            raise FileNotFoundError(fn)
        _ck(rc, "vc_count_file(%s)" % fn)
        return st

    def count_gz_share(self, fn: str, first_share: bool, start_bit: int, window, text_len: int,
                       block_size: int = 10_000_000, n_thread: int = 4):
        """One rank's share of a gzip file (vc_count_gz_share): (FileStats,
        RangeInfo in share coordinates, CRC accounting dict)."""
        st, ri, cr = FileStats(), RangeInfo(), GzShareCrc()
        w = None if window is None else np.ascontiguousarray(window, dtype=np.uint8)
        rc = lib().vc_count_gz_share(self._h, fn.encode(), 1 if first_share else 0, start_bit,
                                     None if w is None else _ptr(w), text_len, block_size, n_thread,
                                     C.byref(st), C.byref(ri), C.byref(cr))
        if rc == VC_EIO:
            raise FileNotFoundError(fn)
        _ck(rc, "vc_count_gz_share(%s)" % fn)
        return st, ri, cr.as_dict()

    def count_gz_share_held(self, share, first_share: bool, window, text_len: int, block_size: int = 10_000_000,
                            n_thread: int = 4):
        """count_gz_share from a held share (vc_count_gz_share_held): the
        scan's decoded chunks are streamed instead of inflated again.  The
        share is spent (close it afterwards)."""
        st, ri, cr = FileStats(), RangeInfo(), GzShareCrc()
        w = None if window is None else np.ascontiguousarray(window, dtype=np.uint8)
        rc = lib().vc_count_gz_share_held(self._h, share.handle(), 1 if first_share else 0,
                                          None if w is None else _ptr(w), text_len, block_size, n_thread,
                                          C.byref(st), C.byref(ri), C.byref(cr))
        _ck(rc, "vc_count_gz_share_held")
        return st, ri, cr.as_dict()

    def count_file_range(self, fn: str, begin: int, end: int, block_size: int = 10_000_000,
                         n_thread: int = 4):
        """One rank's byte range [begin, end) of a file (vc_count_file_range):
        (FileStats, RangeInfo); FileNotFoundError if it cannot be opened."""
        st, ri = FileStats(), RangeInfo()
        rc = lib().vc_count_file_range(self._h, fn.encode(), begin, min(end, NO_OFFSET), block_size, n_thread,
                                       C.byref(st), C.byref(ri))
        if rc == VC_EIO:
            raise FileNotFoundError(fn)
        _ck(rc, "vc_count_file_range(%s)" % fn)
        return st, ri

    def finish(self):
        """(counts uint32[2n], kmers_extracted) after all queued work."""
        counts = np.zeros(2 * self.n_patterns + 2, dtype=np.uint32)
        km = C.c_uint64()
        _ck(lib().vc_finish(self._h, _ptr(counts), C.byref(km)), "vc_finish")
        return counts[:2 * self.n_patterns], km.value

    def reset(self) -> None:
        _ck(lib().vc_reset(self._h), "vc_reset")

    def bind_outputs(self, counts_ptr: int = 0, tally_ptr: int = 0) -> None:
        _ck(lib().vc_bind_outputs(self._h, P(counts_ptr) if counts_ptr else None,
                                  P(tally_ptr) if tally_ptr else None), "vc_bind_outputs")

    @property
    def stream(self) -> int:
        return lib().vc_stream(self._h) or 0

    def set_timing(self, on: bool = True) -> None:
        _ck(lib().vc_set_timing(self._h, 1 if on else 0), "vc_set_timing")

    def kernel_ms(self) -> float:
        ms = C.c_float()
        _ck(lib().vc_kernel_ms(self._h, C.byref(ms)), "vc_kernel_ms")
        return ms.value

    def table_info(self):
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _ck(lib().vc_table_info(self._h, C.byref(a), C.byref(b), C.byref(c)), "vc_table_info")
        return {"n_keys": a.value, "slots": b.value, "filter_bytes": c.value}

    def close(self):
        if getattr(self, "_h", None):
            lib().vc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def create_combined_kmer_map(db: PatternDB, k: int, device: int = 0, devices=None) -> KmerMap:
    """create_combined_kmer_map (vaf-counter.c:198): keys -> static device table
    (one replica per entry of ``devices`` for a multi-GPU counter)."""
    keys, vals, coll = db.keys(k)
    if coll > 0:
        sys.stderr.write("[W::create_combined_kmer_map] Warning: %d k-mer collisions detected. "
                         "Some patterns may have overlapping k-mers.\n" % coll)
    m = KmerMap(k, keys, vals, db.n, device, devices)
    m.n_collisions = coll
    return m


def count_fastq_kmers(fn: str, k: int, n_thread: int, block_size: int, kmer_map: KmerMap,
                      db: PatternDB = None):
    """count_fastq_kmers (vaf-counter.c:550): silently skips an unopenable file."""
    assert k == kmer_map.k
    try:
        return kmer_map.count_file(fn, block_size, n_thread)
    except FileNotFoundError:
        return None


def scan_file(fn: str, k: int, block_size: int = 10_000_000, with_reads: bool = False):
    """Host-only reader + block loop (no device): (FileStats, reads or None)."""
    st = FileStats()
    if not with_reads:
        rc = lib().vc_scan_file(fn.encode(), k, block_size, C.byref(st), None, 0, None, 0)
        reads = None
    else:
        size = _text_size(fn) + 16
        seq = np.zeros(max(size * 4, 64), np.uint8)     # gz inflates; bounded by caller use
        lens = np.zeros(max(size, 16), np.uint32)
        rc = lib().vc_scan_file(fn.encode(), k, block_size, C.byref(st), _ptr(seq), seq.size,
                                _ptr(lens), lens.size)
        reads = []
        pos = 0
        for i in range(int(st.seqs)):
            n = int(lens[i])
            reads.append(seq[pos:pos + n].tobytes())
            pos += n
    if rc == VC_EIO:
        raise FileNotFoundError(fn)
    _ck(rc, "vc_scan_file")
    return st, reads


def _text_size(fn: str) -> int:
    """Bytes of the file's (decompressed) text."""
    with open(fn, "rb") as f:
        gz = f.read(2) == b"\x1f\x8b"
    if not gz:
        return os.path.getsize(fn)
    n = lib().vc_gz_inflate_zlib(fn.encode(), None, 0)
    return max(int(n), 0)


def gz_inflate_parallel(fn: str, threads: int = 4, chunk_bytes: int = 4 << 20):
    """The decompressed stream of a gzip file through the parallel inflater
    (vafc_gzip.h): (bytes, stats dict); None if the inflater declines the file."""
    st = np.zeros(6, np.uint64)
    n = lib().vc_gz_inflate_parallel(fn.encode(), threads, chunk_bytes, None, 0, _ptr(st))
    if n < 0:
        return None
    cap = int(n) + 1
    out = np.zeros(cap, np.uint8)
    n = lib().vc_gz_inflate_parallel(fn.encode(), threads, chunk_bytes, _ptr(out), cap, _ptr(st))
    keys = ("chunks", "accepted", "skipped", "fallback", "members", "crc_error")
    return out[:min(int(n), cap)].tobytes(), dict(zip(keys, (int(x) for x in st)))


def gz_inflate_zlib(fn: str) -> bytes:
    """The decompressed stream through zlib's gzread (the reference's reader)."""
    cap = _text_size(fn) + 1
    out = np.zeros(cap, np.uint8)
    n = lib().vc_gz_inflate_zlib(fn.encode(), _ptr(out), cap)
    if n < 0:
        raise FileNotFoundError(fn)
    return out[:int(n)].tobytes()


def scan_file_parallel(fn: str, k: int, block_size: int = 10_000_000, threads: int = 4,
                       piece_bytes: int = 8 << 20, with_reads: bool = False):
    """Host-only parallel reader of vc_count_file (no device): (FileStats, reads
    or None); the reads are those of scan_file, in order.  Plain files: pieces
    of piece_bytes parsed by `threads` workers; gzip: `threads` inflate workers
    on chunks of piece_bytes compressed bytes, one parsing thread."""
    st = FileStats()
    if not with_reads:
        rc = lib().vc_scan_file_parallel(fn.encode(), k, block_size, threads, piece_bytes, C.byref(st),
                                         None, 0, None, 0)
        reads = None
    else:
        size = _text_size(fn) + 16
        seq = np.zeros(max(size, 64), np.uint8)
        lens = np.zeros(max(size, 16), np.uint32)
        rc = lib().vc_scan_file_parallel(fn.encode(), k, block_size, threads, piece_bytes, C.byref(st),
                                         _ptr(seq), seq.size, _ptr(lens), lens.size)
        reads = []
        pos = 0
        for i in range(int(st.seqs)):
            n = int(lens[i])
            reads.append(seq[pos:pos + n].tobytes())
            pos += n
    if rc == VC_EIO:
        raise FileNotFoundError(fn)
    _ck(rc, "vc_scan_file_parallel")
    return st, reads


def scan_file_range(fn: str, k: int, begin: int, end: int, block_size: int = 10_000_000, threads: int = 4,
                    piece_bytes: int = 8 << 20, with_reads: bool = False):
    """Host-only: vc_count_file_range's reader over [begin, end) without a
    device: (FileStats, RangeInfo, reads or None)."""
    st, ri = FileStats(), RangeInfo()
    end = min(end, NO_OFFSET)
    if not with_reads:
        rc = lib().vc_scan_file_range(fn.encode(), k, block_size, threads, piece_bytes, begin, end, C.byref(st),
                                      C.byref(ri), None, 0, None, 0)
        reads = None
    else:
        size = _text_size(fn) + 16
        seq = np.zeros(max(size, 64), np.uint8)
        lens = np.zeros(max(size, 16), np.uint32)
        rc = lib().vc_scan_file_range(fn.encode(), k, block_size, threads, piece_bytes, begin, end, C.byref(st),
                                      C.byref(ri), _ptr(seq), seq.size, _ptr(lens), lens.size)
        reads = []
        pos = 0
        for i in range(int(st.seqs)):
            n = int(lens[i])
            reads.append(seq[pos:pos + n].tobytes())
            pos += n
    if rc == VC_EIO:
        raise FileNotFoundError(fn)
    _ck(rc, "vc_scan_file_range")
    return st, ri, reads


def gz_share_scan(fn: str, begin: int, end: int, threads: int = 4, chunk_bytes: int = 0):
    """vc_gz_share_scan: (GzShareInfo as a dict, the share's last 32 KiB as
    uint16 symbols)."""
    info = GzShareInfo()
    wsym = np.zeros(GZ_WSIZE, np.uint16)
    rc = lib().vc_gz_share_scan(fn.encode(), begin, min(end, NO_OFFSET), threads, chunk_bytes, C.byref(info),
                                _ptr(wsym))
    if rc == VC_EIO:
        raise FileNotFoundError(fn)
    _ck(rc, "vc_gz_share_scan(%s)" % fn)
    return {f: int(getattr(info, f)) for f, _ in info._fields_}, wsym


class GzShare:
    """A held share of a gzip stream (vc_gz_share_open): the scan's decoded
    chunks, kept for one count of the share.  close() frees them (a count
    spends the share but the handle still needs closing)."""

    def __init__(self, h):
        self._h = h

    def handle(self):
        if not self._h:
            raise VafcError("gz share already closed")
        return self._h

    def close(self):
        if self._h:
            lib().vc_gz_share_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gz_share_open(fn: str, begin: int, end: int, threads: int = 4, chunk_bytes: int = 0, hold_bytes: int = 0,
                  kmap=None):
    """vc_gz_share_open: gz_share_scan that keeps the share's decoded chunks
    (at most hold_bytes of buffers) for the count: (info dict, window
    symbols, GzShare or None when the share was not kept).  kmap: the
    KmerMap that will count the share (its GPU's NUMA node), or None."""
    info = GzShareInfo()
    wsym = np.zeros(GZ_WSIZE, np.uint16)
    h = P()
    rc = lib().vc_gz_share_open(None if kmap is None else kmap._h, fn.encode(), begin, min(end, NO_OFFSET), threads, chunk_bytes, hold_bytes,
                                C.byref(info), _ptr(wsym), C.byref(h))
    if rc == VC_EIO:
        raise FileNotFoundError(fn)
    _ck(rc, "vc_gz_share_open(%s)" % fn)
    return {f: int(getattr(info, f)) for f, _ in info._fields_}, wsym, (GzShare(h.value) if h.value else None)


def gz_window_after(wsym: np.ndarray, before: np.ndarray) -> np.ndarray:
    """The 32 KiB of text after a share from its symbols and the 32 KiB
    before it (include/vafc.h: 0x8000 | i is byte i of `before`)."""
    w = np.asarray(wsym, dtype=np.uint16)
    b = np.asarray(before, dtype=np.uint8)
    return np.where(w < 256, w, b[w & (GZ_WSIZE - 1)]).astype(np.uint8)


def gz_crc32_combine(crc1: int, crc2: int, len2: int) -> int:
    return int(lib().vc_gz_crc32_combine(crc1, crc2, len2))


def scan_gz_share(fn: str, k: int, first_share: bool, start_bit: int, window, text_len: int,
                  block_size: int = 10_000_000, threads: int = 4, with_reads: bool = False, cap: int = 0):
    """Host-only vc_scan_gz_share: (FileStats, RangeInfo, CRC dict, reads or None)."""
    st, ri, cr = FileStats(), RangeInfo(), GzShareCrc()
    w = None if window is None else np.ascontiguousarray(window, dtype=np.uint8)
    seq = lens = None
    if with_reads:
        n = max(cap or 2 * text_len + 4096, 64)
        seq = np.zeros(n, np.uint8)
        lens = np.zeros(max(n // 2, 16), np.uint32)
    rc = lib().vc_scan_gz_share(fn.encode(), k, 1 if first_share else 0, start_bit, None if w is None else _ptr(w),
                                text_len, block_size, threads, C.byref(st), C.byref(ri), C.byref(cr),
                                None if seq is None else _ptr(seq), 0 if seq is None else seq.size,
                                None if lens is None else _ptr(lens), 0 if lens is None else lens.size)
    if rc == VC_EIO:
        raise FileNotFoundError(fn)
    _ck(rc, "vc_scan_gz_share(%s)" % fn)
    reads = None
    if with_reads:
        reads, pos = [], 0
        for i in range(int(st.seqs)):
            m = int(lens[i])
            reads.append(seq[pos:pos + m].tobytes())
            pos += m
    return st, ri, cr.as_dict(), reads


def scan_gz_share_held(share, k: int, first_share: bool, window, text_len: int, block_size: int = 10_000_000,
                       threads: int = 4, with_reads: bool = False, cap: int = 0):
    """Host-only vc_scan_gz_share_held: scan_gz_share from a held share."""
    st, ri, cr = FileStats(), RangeInfo(), GzShareCrc()
    w = None if window is None else np.ascontiguousarray(window, dtype=np.uint8)
    seq = lens = None
    if with_reads:
        n = max(cap or 2 * text_len + 4096, 64)
        seq = np.zeros(n, np.uint8)
        lens = np.zeros(max(n // 2, 16), np.uint32)
    rc = lib().vc_scan_gz_share_held(share.handle(), k, 1 if first_share else 0, None if w is None else _ptr(w),
                                     text_len, block_size, threads, C.byref(st), C.byref(ri), C.byref(cr),
                                     None if seq is None else _ptr(seq), 0 if seq is None else seq.size,
                                     None if lens is None else _ptr(lens), 0 if lens is None else lens.size)
    _ck(rc, "vc_scan_gz_share_held")
    reads = None
    if with_reads:
        reads, pos = [], 0
        for i in range(int(st.seqs)):
            m = int(lens[i])
            reads.append(seq[pos:pos + m].tobytes())
            pos += m
    return st, ri, cr.as_dict(), reads


INGEST_PROFILE_KEYS = ("reader_s", "main_wait_s", "submit_s", "reparse_s", "parse_thread_s", "slot_wait_thread_s",
                       "acquire_thread_s", "read_thread_s", "read_bytes", "copy_thread_s", "copy_bytes",
                       "guess_thread_s", "worker_cpu_s", "worker_wall_s", "main_cpu_s", "threads", "copy_mode")


def ingest_profile() -> dict:
    """vc_ingest_profile_ex: where this thread's last pass through the parallel
    reader spent its time (seconds; *_thread_s summed over the workers; the
    parse split into the reads out of the source, the batched slot copies and
    the record guesses; worker CPU against wall seconds)."""
    out = np.zeros(len(INGEST_PROFILE_KEYS), np.float64)
    n = lib().vc_ingest_profile_ex(_ptr(out), len(out))
    d = {k: round(float(v), 4) for k, v in zip(INGEST_PROFILE_KEYS, out)}
    for k in ("read_bytes", "copy_bytes", "threads", "copy_mode"):
        d[k] = int(d[k])
    d["pieces"] = int(n)
    return d


def scan_records(fn: str, cap: int = 1 << 20) -> np.ndarray:
    """kseq_read return codes of every record of a file (host-only)."""
    rets = np.zeros(cap, np.int32)
    n = lib().vc_scan_records(fn.encode(), _ptr(rets), cap)
    if n == VC_EIO:
        raise FileNotFoundError(fn)
    return rets[:min(n, cap)]


def synth_reads(seq_ptr, offs_ptr, lens_ptr, first, n_reads, read_len, seed, f_snp,
                windows_ptr, dosage_ptr, n_snp, stream=0) -> None:
    """vafc_synth.gen_reads evaluated on the device (bench / tests)."""
    _ck(lib().vc_synth_reads(P(seq_ptr), P(offs_ptr), P(lens_ptr), first, n_reads, read_len, seed,
                             f_snp, P(windows_ptr) if n_snp else None,
                             P(dosage_ptr) if n_snp else None, n_snp,
                             P(stream) if stream else None), "vc_synth_reads")


def debug_decode(seq_ptr, seq_bytes, offs_ptr, lens_ptr, n_reads, codes_ptr, stream=0) -> None:
    _ck(lib().vc_debug_decode(P(seq_ptr), seq_bytes, P(offs_ptr), P(lens_ptr), n_reads,
                              P(codes_ptr), P(stream) if stream else None), "vc_debug_decode")


# --------------------------------------------------------------------------
# CLI mirror (vaf-counter.c:584-738)
# --------------------------------------------------------------------------

USAGE = (
    "Usage: vaf-counter [options] -p <patterns.txt> -o <output.vaf> <reads.fq> [reads2.fq ...]\n"
    "Options:\n"
    "  -k INT    k-mer length [%d]\n"
    "  -p FILE   input pattern file\n"
    "  -o FILE   output VAF file\n"
    "  -t INT    number of threads [%d]\n"
    "  -b INT    block size [%d]\n"
    "  -v        verbose mode (report performance statistics)\n")


def parse_args(argv):
    """ketopt(..., permute=1, "k:p:o:t:b:v") semantics: options may follow files."""
    opt = {"k": 21, "t": 4, "b": 10_000_000, "p": None, "o": None, "v": False}
    files, i = [], 0
    while i < len(argv):
        a = argv[i]
        if a == "--":
            files.extend(argv[i + 1:])
            break
        if len(a) >= 2 and a[0] == "-":
            j = 1
            while j < len(a):
                c = a[j]
                if c in "kpotb":
                    val = a[j + 1:] if j + 1 < len(a) else (argv[i + 1] if i + 1 < len(argv) else None)
                    if j + 1 >= len(a):
                        i += 1
                    if val is not None:
                        if c in "ktb":
                            try:
                                opt[c] = int(val)
                            except ValueError:
                                opt[c] = 0
                        else:
                            opt[c] = val
                    break
                if c == "v":
                    opt["v"] = True
                j += 1
        else:
            files.append(a)
        i += 1
    return opt, files


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    o, files = parse_args(argv)
    k = o["k"]
    if not o["p"] or not o["o"] or not files:
        sys.stderr.write(USAGE % (k, o["t"], o["b"]))
        return 1
    err = sys.stderr.write
    t_start = time.time()
    err("[M::main] Loading patterns...\n")
    t = time.time()
    try:
        db = load_patterns(o["p"])
    except VafcError:
        err("Error: failed to load pattern file\n")
        return 1
    err("[M::main] Loaded %d patterns in %.3f sec\n" % (db.n, time.time() - t))
    err("[M::main] Creating k-mer map...\n")
    try:
        devs = [int(x) for x in os.environ.get("VAFC_DEVICES", "").split(",") if x.strip()]
        kmap = create_combined_kmer_map(db, k, int(os.environ.get("VAFC_DEVICE", "0")), devs or None)
    except VafcError:
        err("Error: failed to create k-mer map\n")
        return 1
    err("[M::main] Counting k-mers in FASTQ files with %d threads...\n" % o["t"])
    t = time.time()
    bases = seqs = 0
    for fn in files:
        err("[M::main] Processing %s...\n" % fn)
        st = count_fastq_kmers(fn, k, o["t"], o["b"], kmap, db)
        if st is not None:
            bases += st.bases
            seqs += st.seqs
    counts, kmers = kmap.finish()
    t_count = time.time() - t
    tot = int(counts.astype(np.uint64).sum())
    avg = tot / (db.n if db.n > 0 else 1)
    err("[M::main] Writing VAF file...\n")
    try:
        db.write_vaf(counts, o["o"])
    except VafcError:
        err("Error: failed to open output file\n")
        return 1
    err("[M::main] Done. Average depth: %.2f\n" % avg)
    if o["v"]:
        err("  Bases processed:       %d (%.2f Mbases)\n" % (bases, bases / 1e6))
        err("  K-mers extracted:      %d (%.2f million)\n" % (kmers, kmers / 1e6))
        if t_count > 0:
            err("  Speed:                 %.2f Mbases/sec\n" % (bases / t_count / 1e6))
        err("  Total runtime:         %.3f sec\n" % (time.time() - t_start))
    kmap.close()
    db.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())


# --------------------------------------------------------------------------
# snp-pattern-gen
# --------------------------------------------------------------------------

def load_fasta(fn: str):
    """load_fasta (snp-pattern-gen.c:67-103): [(name, sequence bytes)]."""
    h = P()
    rc = lib().vc_fasta_load(fn.encode(), C.byref(h))
    if rc == VC_EIO:
        raise FileNotFoundError(fn)
    _ck(rc, "vc_fasta_load")
    try:
        out = []
        for i in range(lib().vc_fasta_count(h)):
            n = C.c_uint32()
            p = lib().vc_fasta_seq(h, i, C.byref(n))
            out.append((lib().vc_fasta_name(h, i), C.string_at(p, n.value) if n.value else b""))
        return out
    finally:
        lib().vc_fasta_free(h)


def count_candidate_kmers(k: int, seqs, keys, device: int = 0) -> np.ndarray:
    """count_candidate_kmers (snp-pattern-gen.c:159-190) on the GPU: for each of
    the distinct canonical keys, how often it occurs among the canonical
    k-mers of the sequences (u32)."""
    seqs = [bytes(s) for s in seqs]
    blob = np.frombuffer(b"".join(seqs), np.uint8) if any(seqs) else np.zeros(1, np.uint8)
    lens = np.array([len(s) for s in seqs], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens, dtype=np.uint64)[:-1]]).astype(np.uint64) if len(seqs) else \
        np.zeros(1, np.uint64)
    keys = np.ascontiguousarray(keys, np.uint64)
    counts = np.zeros(max(keys.size, 1), np.uint32)
    blob = np.ascontiguousarray(blob)
    _ck(lib().vc_count_candidates(k, _ptr(blob), int(sum(len(s) for s in seqs)), _ptr(offs), _ptr(lens),
                                  len(seqs), _ptr(keys), keys.size, _ptr(counts), device),
        "vc_count_candidates")
    return counts[:keys.size]


# --------------------------------------------------------------------------
# kc-c4 k-mer histogram
# --------------------------------------------------------------------------

class KmerHistogram(KmerMap):
    """kc-c4's kc_c4x_t (kc-c4.c:52-67) on the GPU: every canonical k-mer of the
    reads counted in one device hash table of ``slots`` 16-byte slots (0 = sized
    from free HBM).  count_block / count_device / count_file as for KmerMap;
    ``histogram()`` is print_hist's count vector (kc-c4.c:219-231)."""

    def __init__(self, k: int, slots: int = 0, device: int = 0):
        self.k, self.n_patterns, self.device = k, 0, device
        h = P()
        _ck(lib().vc_kc_create(C.byref(h), k, slots, device), "vc_kc_create")
        self._h = h
        self.n_collisions = 0

    @property
    def slots(self) -> int:
        return lib().vc_kc_slots(self._h)

    def set_partition(self, n_parts: int, part: int) -> None:
        """Count only hash slice ``part`` of ``n_parts`` (clears the table)."""
        _ck(lib().vc_kc_set_partition(self._h, n_parts, part), "vc_kc_set_partition")

    def histogram(self, n_bins: int = 256, min_count: int = 1):
        """(hist uint64[n_bins], distinct, kmers): hist[min(c, n_bins-1)] = keys
        counted c >= min_count times (kc-c4: 256 bins; yak-count: 1024).
        Raises VafcError(VC_EFULL) when the table ran out."""
        hist = np.zeros(n_bins, np.uint64)
        d, km = C.c_uint64(), C.c_uint64()
        _ck(lib().vc_kc_histogram2(self._h, _ptr(hist), n_bins, min_count, C.byref(d), C.byref(km)),
            "vc_kc_histogram2")
        return hist, d.value, km.value

    def track_first(self, on: bool = True) -> None:
        """Record first-occurrence stamps (yak -b pass 1); clears the table."""
        _ck(lib().vc_kc_track_first(self._h, 1 if on else 0), "vc_kc_track_first")

    def yak_bloom_select(self, pre: int, bf_shift: int, n_hash: int) -> None:
        """yak-count's Bloom filters replayed: keep the keys yak's pass 1 keeps,
        counts restart at 0, later counting only touches those keys."""
        _ck(lib().vc_yak_bloom_select(self._h, pre, bf_shift, n_hash), "vc_yak_bloom_select")


def kc_count_file(fn: str, k: int = 31, block_size: int = 10_000_000, n_thread: int = 4,
                  slots: int = 0, device: int = 0) -> np.ndarray:
    """count_file + print_hist's counts (kc-c4.c:181-231): hist uint64[256].
    A table too small for the distinct k-mers is re-run in hash slices."""
    h = KmerHistogram(k, slots, device)
    try:
        n_parts = 1
        while True:
            total = np.zeros(256, np.uint64)
            kmers, full = 0, False
            for part in range(n_parts):
                h.set_partition(n_parts, part)
                h.count_file(fn, block_size, n_thread)
                h.finish()
                try:
                    hist, _, kmers = h.histogram()
                except VafcError as e:
                    if e.code != VC_EFULL:
                        raise
                    full = True
                    break
                total += hist
            if not full:
                return total
            cap = h.slots * 7 // 10
            n_parts = max(n_parts * 2, -(-kmers // cap) if cap else 2)
            if n_parts > 1024:
                raise VafcError("k-mer table too small", VC_EFULL)
    finally:
        h.close()


def kc_main(argv=None) -> int:
    """kc-c4's main (kc-c4.c:236-265): prints ``i\tcount`` for i = 1..255."""
    import getopt
    argv = sys.argv[1:] if argv is None else argv
    k, p, b, t = 31, 10, 10_000_000, 4
    try:
        opts, args = getopt.gnu_getopt(argv, "k:p:b:t:")
    except getopt.GetoptError:
        opts, args = [], []
    for o, v in opts:
        if o == "-k":
            k = int(v)
        elif o == "-p":
            p = int(v)
        elif o == "-b":
            b = int(v)
        elif o == "-t":
            t = int(v)
    if not args:
        sys.stderr.write("Usage: kc-c4 [options] <in.fa>\nOptions:\n"
                         "  -k INT     k-mer size [%d]\n  -p INT     prefix length [%d]\n"
                         "  -b INT     block size [%d]\n  -t INT     number of worker threads [%d]\n"
                         % (k, p, b, t))
        return 1
    if p < 10:
        sys.stderr.write("ERROR: -p should be at least 10\n")
        return 1
    hist = kc_count_file(args[0], k, b, t, int(os.environ.get("VAFC_KC_SLOTS", "0")),
                         int(os.environ.get("VAFC_DEVICE", "0")))
    sys.stdout.write("".join("%d\t%d\n" % (i, hist[i]) for i in range(1, 256)))
    return 0


def yak_count_file(fn1: str, fn2: str = None, k: int = 31, pre: int = 10, bf_shift: int = 0, n_hash: int = 4,
                   chunk_size: int = 10_000_000, n_thread: int = 4, slots: int = 0, device: int = 0):
    """yak_count_file + yak_ch_shrink + yak_ch_hist (yak-count.c:440-452,
    268-288, 209-240): (hist uint64[1024], distinct k-mers after shrinking)."""
    fn2 = fn1 if fn2 is None else fn2
    two_pass = bf_shift > 0
    replay = two_pass and fn1 != fn2
    block = min(chunk_size, 0x7FFFFFFF)
    h = KmerHistogram(k, slots, device)
    try:
        n_parts = 1
        while True:
            total, tot, kmers, full = np.zeros(1024, np.uint64), 0, 0, False
            for part in range(n_parts):
                h.set_partition(n_parts, part)
                if replay:
                    h.track_first(True)
                h.count_file(fn1, block, n_thread)
                h.finish()
                try:
                    if replay:
                        h.yak_bloom_select(pre, bf_shift, n_hash)
                        h.count_file(fn2, block, n_thread)
                        h.finish()
                    hist, d, kmers = h.histogram(1024, 2 if two_pass else 1)
                except VafcError as e:
                    if e.code != VC_EFULL:
                        raise
                    full = True
                    break
                total += hist
                tot += d
            if not full:
                return total, tot
            cap = h.slots * 7 // 10
            n_parts = max(n_parts * 2, -(-kmers // cap) if cap else 2)
            if n_parts > 1024:
                raise VafcError("k-mer table too small", VC_EFULL)
    finally:
        h.close()


def yak_main(argv=None) -> int:
    """yak-count's main (yak-count.c:456-507): 1023 histogram lines."""
    import getopt
    argv = sys.argv[1:] if argv is None else argv
    k, pre, chunk, t, b, H = 31, 10, 10_000_000, 4, 0, 4
    try:
        opts, args = getopt.gnu_getopt(argv, "k:p:K:t:b:H:")
    except getopt.GetoptError:
        opts, args = [], []
    for o, v in opts:
        if o == "-k":
            k = int(v)
        elif o == "-p":
            pre = int(v)
        elif o == "-K":
            chunk = int(v)
        elif o == "-t":
            t = int(v)
        elif o == "-b":
            b = int(v)
        elif o == "-H":
            H = int(v)
    if not args:
        sys.stderr.write("Usage: yak-count [options] <in.fa> [in.fa]\nOptions:\n"
                         "  -k INT     k-mer size [%d]\n  -p INT     prefix length [%d]\n"
                         "  -b INT     set Bloom filter size to 2**INT bits; 0 to disable [%d]\n"
                         "  -H INT     use INT hash functions for Bloom filter [%d]\n"
                         "  -t INT     number of worker threads [%d]\n  -K INT     chunk size [100m]\n"
                         "Note: -b37 is recommended for human reads\n" % (k, pre, b, H, t))
        return 1
    if pre < 10:
        sys.stderr.write("ERROR: -p should be at least 10\n")
        return 1
    hist, tot = yak_count_file(args[0], args[1] if len(args) > 1 else None, k, pre, b, H, chunk, t,
                               int(os.environ.get("VAFC_KC_SLOTS", "0")), int(os.environ.get("VAFC_DEVICE", "0")))
    sys.stderr.write("[M::main] %d distinct k-mers after shrinking\n" % tot)
    sys.stdout.write("".join("%d\t%d\n" % (i, hist[i]) for i in range(1, 1024)))
    return 0


# ---------------------------------------------------------------------------
# correlation-matrix (correlation-matrix.c), the names
# of the reference's functions over vc_vafset / vc_corr_* in libvafc.so
# ---------------------------------------------------------------------------

class VafSamples:
    """The reference's sample_t array (correlation-matrix.c:11-16) as a vc_vafset."""

    def __init__(self):
        L = lib()
        h = P()
        _ck(L.vc_vafset_create(C.byref(h)), "vc_vafset_create")
        self._h = h

    def load_vaf_file(self, fn: str) -> None:
        """correlation-matrix.c:25-90; VafcError(VC_EIO) if the file cannot be opened."""
        _ck(lib().vc_vafset_add(self._h, fn.encode()), "load_vaf_file(%s)" % fn)

    def load_vaf_files(self, fns, n_threads: int = 8) -> list:
        """load_vaf_file over many files, read by n_threads threads and appended
        in order (vc_vafset_add_many).  Returns, per file added, whether the
        100,000-row cap truncated it.  VafcError(VC_EIO) at the first file that
        cannot be opened; the files before it stay added."""
        arr = (C.c_char_p * len(fns))(*[f.encode() for f in fns])
        trunc = np.zeros(max(len(fns), 1), np.uint8)
        added = C.c_int(0)
        rc = lib().vc_vafset_add_many(self._h, C.cast(arr, P), len(fns), n_threads, C.byref(added), _ptr(trunc))
        _ck(rc, "load_vaf_files(%s)" % (fns[added.value] if rc and added.value < len(fns) else ""))
        return [bool(t) for t in trunc[: added.value]]

    def add(self, name: str, vaf: np.ndarray, depth: np.ndarray) -> None:
        vaf = np.ascontiguousarray(vaf, np.float64)
        depth = np.ascontiguousarray(depth, np.int32)
        _ck(lib().vc_vafset_add_arrays(self._h, name.encode(), _ptr(vaf), _ptr(depth), vaf.size), "add")

    def __len__(self):
        return lib().vc_vafset_count(self._h)

    def name(self, i: int) -> str:
        return lib().vc_vafset_name(self._h, i).decode()

    def n_snps(self, i: int) -> int:
        return lib().vc_vafset_snps(self._h, i)

    def calculate_correlation_matrix(self, min_snps: int = 20, min_depth: int = 1, device: int = 0):
        """correlation-matrix.c:146-162 on the GPU; returns (n x n float64 matrix, kernel ms)."""
        n = len(self)
        corr = np.zeros((n, n), np.float64)
        ms = C.c_float()
        _ck(lib().vc_corr_matrix(self._h, min_snps, min_depth, _ptr(corr), device, C.byref(ms)),
            "calculate_correlation_matrix")
        return corr, ms.value

    def write_corr(self, corr: np.ndarray, fn: str) -> None:
        corr = np.ascontiguousarray(corr, np.float64)
        _ck(lib().vc_corr_write(self._h, _ptr(corr), fn.encode()), "write %s" % fn)

    def build_tree(self, corr: np.ndarray, fn: str) -> None:
        """correlation-matrix.c:190-257."""
        corr = np.ascontiguousarray(corr, np.float64)
        _ck(lib().vc_corr_tree(self._h, _ptr(corr), fn.encode()), "build_tree %s" % fn)

    def close(self):
        if getattr(self, "_h", None):
            lib().vc_vafset_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def correlation_matrix_raw(vaf: np.ndarray, depth: np.ndarray, n_snps=None, min_snps: int = 20,
                           min_depth: int = 1, device: int = 0):
    """Pairwise depth-aware Pearson of the rows of vaf/depth ([n_samples][stride]);
    sample i has n_snps[i] rows (default: all).  Returns (matrix, kernel ms)."""
    vaf = np.ascontiguousarray(vaf, np.float64)
    depth = np.ascontiguousarray(depth, np.int32)
    n, stride = vaf.shape
    ns = np.ascontiguousarray(np.full(n, stride) if n_snps is None else n_snps, np.int32)
    corr = np.zeros((n, n), np.float64)
    ms = C.c_float()
    _ck(lib().vc_corr_matrix_raw(_ptr(vaf), _ptr(depth), _ptr(ns), n, stride, min_snps, min_depth, _ptr(corr),
                                 device, C.byref(ms)), "vc_corr_matrix_raw")
    return corr, ms.value
