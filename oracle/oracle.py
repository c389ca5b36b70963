"""ctypes view of oracle/build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker.  The product never imports it.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "liboracle.so")
CLI = os.path.join(_HERE, "build", "vaf-counter-oracle")
REF_CLI = os.path.join(_HERE, "_ref", "vaf-counter")
REF_KMER_DUMP = os.path.join(_HERE, "_ref", "ref_kmer_dump")
P = C.c_void_p
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError("oracle not built: make -C oracle")
        L = C.CDLL(LIB)
        L.orc_open.restype = P
        L.orc_open.argtypes = [C.c_char_p, C.c_int]
        L.orc_open_keys.restype = P
        L.orc_open_keys.argtypes = [C.c_int, P, P, C.c_uint64]
        L.orc_close.argtypes = [P]
        L.orc_n_patterns.argtypes = [P]
        L.orc_n_collisions.argtypes = [P]
        L.orc_n_keys.restype = C.c_uint64
        L.orc_n_keys.argtypes = [P]
        L.orc_dump_pattern_keys.restype = C.c_uint64
        L.orc_dump_pattern_keys.argtypes = [P, P, P, C.c_uint64]
        L.orc_count_reads.restype = C.c_uint64
        L.orc_count_reads.argtypes = [P, P, P, P, C.c_uint64, P]
        L.orc_read_kmers.restype = C.c_uint64
        L.orc_read_kmers.argtypes = [C.c_int, P, C.c_uint32, P, C.c_uint64]
        L.orc_decode.argtypes = [P, C.c_uint32, P]
        L.orc_count_file.argtypes = [P, C.c_char_p, C.c_int, P, P, P, P]
        L.orc_scan_records.restype = C.c_int64
        L.orc_scan_records.argtypes = [C.c_char_p, P, C.c_int64]
        L.orc_fasta_records.restype = C.c_int64
        L.orc_fasta_records.argtypes = [C.c_char_p, P, C.c_size_t, P, C.c_int64, P, C.c_size_t]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(P)


class Oracle:
    """Pattern table + counting, restated on the CPU."""

    def __init__(self, k, pattern_fn=None, keys=None, vals=None):
        self.k = k
        if pattern_fn is not None:
            self.h = lib().orc_open(pattern_fn.encode(), k)
            if not self.h:
                raise FileNotFoundError(pattern_fn)
        else:
            keys = np.ascontiguousarray(keys, dtype=np.uint64)
            vals = np.ascontiguousarray(vals, dtype=np.uint32)
            self.h = lib().orc_open_keys(k, _p(keys), _p(vals), keys.size)

    @property
    def n_patterns(self):
        return lib().orc_n_patterns(self.h)

    @property
    def n_collisions(self):
        return lib().orc_n_collisions(self.h)

    def keys(self):
        n = lib().orc_n_keys(self.h)
        k = np.zeros(n, np.uint64)
        v = np.zeros(n, np.uint32)
        lib().orc_dump_pattern_keys(self.h, _p(k), _p(v), n)
        return k, v

    def count_reads(self, seq, offs, lens, n_patterns=None):
        n_patterns = self.n_patterns if n_patterns is None else n_patterns
        counts = np.zeros(2 * n_patterns + 2, np.uint32)
        seq = np.ascontiguousarray(seq, np.uint8)
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        km = lib().orc_count_reads(self.h, _p(seq), _p(offs), _p(lens), offs.size, _p(counts))
        return counts[:2 * n_patterns], km

    def count_file(self, fn, block, counts):
        b, s, km = C.c_uint64(), C.c_uint64(), C.c_uint64()
        rc = lib().orc_count_file(self.h, fn.encode(), block, _p(counts), C.byref(b), C.byref(s), C.byref(km))
        return rc, b.value, s.value, km.value

    def close(self):
        if self.h:
            lib().orc_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_kmers(k, read: bytes):
    a = np.frombuffer(bytes(read), np.uint8).copy() if len(read) else np.zeros(1, np.uint8)
    out = np.zeros(max(len(read), 1), np.uint64)
    n = lib().orc_read_kmers(k, _p(a), len(read), _p(out), out.size)
    return out[:n]


def decode(read: bytes):
    a = np.frombuffer(bytes(read), np.uint8).copy() if len(read) else np.zeros(1, np.uint8)
    out = np.zeros(max(len(read), 1), np.uint8)
    lib().orc_decode(_p(a), len(read), _p(out))
    return out[:len(read)]


def scan_records(fn, cap=1 << 20):
    rets = np.zeros(cap, np.int32)
    n = lib().orc_scan_records(fn.encode(), _p(rets), cap)
    if n < 0:
        raise FileNotFoundError(fn)
    return rets[:min(n, cap)]


def fasta_records(fn):
    """[(name, seq)] of every record until the first kseq_read < 0 (the loop of
    snp-pattern-gen's load_fasta, snp-pattern-gen.c:82-98)."""
    import gzip
    raw = open(fn, "rb").read()
    if raw[:2] == b"\x1f\x8b":
        raw = gzip.decompress(raw)
    cap = len(raw) + 16
    seq = np.zeros(cap, np.uint8)
    lens = np.zeros(cap, np.uint32)
    names = np.zeros(cap, np.uint8)
    n = lib().orc_fasta_records(fn.encode(), _p(seq), cap, _p(lens), cap, _p(names), cap)
    if n < 0:
        raise FileNotFoundError(fn)
    out, pos = [], 0
    nm = names.tobytes().split(b"\0")
    for i in range(n):
        L = int(lens[i])
        out.append((nm[i], seq[pos:pos + L].tobytes()))
        pos += L
    return out
