#!/usr/bin/env python3
"""Where a reader thread's time goes on the host (CPU only, tools only): a
plain pread loop over a page-cached FASTQ in 1 MB windows (the copy out of
the page cache alone) against the product's host-only parallel reader
(vc_scan_file_parallel: pread + record parse + sequence copy), 1..T threads.
    python tools/host_read_split.py FASTQ [threads ...]
    python tools/host_read_split.py --make N FASTQ [threads ...]   (writes N 150 bp reads first)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kmer-cnt_amd"))


def make_fastq(fn, n, L=150):
    """n random 150 bp reads as 4-line FASTQ (20-byte names, constant quality)."""
    import numpy as np
    rng = np.random.default_rng(1)
    hw = 20
    rec = hw + 1 + L + 1 + 2 + L + 1
    with open(fn, "wb") as f:
        for c0 in range(0, n, 1_000_000):
            m = min(1_000_000, n - c0)
            a = np.empty((m, rec), np.uint8)
            ids = np.char.zfill(np.arange(c0, c0 + m).astype(str), hw - 2)
            a[:, 0], a[:, 1] = ord("@"), ord("r")
            a[:, 2:hw] = np.frombuffer("".join(ids).encode(), np.uint8).reshape(m, hw - 2)
            a[:, hw] = 10
            a[:, hw + 1:hw + 1 + L] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, (m, L))]
            o = hw + 1 + L
            a[:, o], a[:, o + 1], a[:, o + 2] = 10, ord("+"), 10
            a[:, o + 3:o + 3 + L] = ord("I")
            a[:, o + 3 + L] = 10
            f.write(a.tobytes())


def main():
    import vafc
    args = sys.argv[1:]
    if args[0] == "--make":
        make_fastq(args[2], int(args[1]))
        args = args[2:]
    fn = args[0]
    threads = [int(x) for x in args[1:]] or [1, 4]
    size = os.path.getsize(fn)
    buf = bytearray(1 << 20)
    mv = memoryview(buf)
    fd = os.open(fn, os.O_RDONLY)
    t = time.perf_counter()
    off = 0
    while True:
        n = os.preadv(fd, [mv], off)
        if n <= 0:
            break
        off += n
    dt = time.perf_counter() - t
    os.close(fd)
    print("pread, 1 MB windows, 1 thread: %.2f GB/s (%.3f s)" % (size / dt / 1e9, dt))
    for th in threads:
        best = 1e9
        for _ in range(2):
            t = time.perf_counter()
            vafc.scan_file_parallel(fn, 21, 10_000_000, th, 32 << 20)
            best = min(best, time.perf_counter() - t)
        prof = vafc.ingest_profile()
        print("reader, %d thread(s): %.2f GB/s of text, %.3f parse thread-seconds" %
              (th, size / best / 1e9, prof["parse_thread_s"]))


if __name__ == "__main__":
    main()
