"""One process per GPU: the drop-in vaf-counter as a torchrun job.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        kmer-cnt_amd/vafc_dist.py [-v] -k 21 -p patterns.txt -o sample.vaf R1.fq R2.fq.gz ...

Same flags, messages, exit codes and .vaf as the reference's main
(vaf-counter.c:584-735) and the drop-in CLI.  Reads are independent units, so
the path shards with no data-path collective:

* every rank loads the patterns and builds its own replica of the static
  key table on its GPU (load_patterns / create_combined_kmer_map,
  vaf-counter.c:149-252);
* a plain FASTA/FASTQ file is split into N byte ranges, one per rank
  (vc_count_file_range): rank r counts the records whose header lies in its
  range, found from the record shape at the range's start as the parallel
  reader's pieces are.  The reference reads the file in one kseq stream under
  its block loop (vaf-counter.c:486-517, 550-582), so a split is exact only if
  every range began at the record where the previous one ended and no range
  met a truncated record (a -2 ends a block, and the file's end -- the third
  empty block -- depends on the blocks before it).  The ranks exchange their
  (first, next, errs) with one all-gather per file; if the chain does not
  hold, every rank restores its counts from before the file and rank
  i mod N counts file i whole, which is exactly vc_count_file.  Rank 0
  decides up front which files are split and their sizes (one all-gather),
  so every rank takes the same branch for every file;
* a gzip file is split into shares of its deflate stream (round 6,
  vafc_gzip.h): rank r decodes the blocks from the first dynamic block at or
  after byte A_r of the file without the history before them and keeps its
  last 32 KiB as symbols naming bytes of that unknown window; one all-gather
  gives every rank the windows (each follows from the one before, rank 0's
  history being empty), and every rank then counts its share's records from
  its known window.  The ranges chain as for plain files, and the members'
  CRC-32 checks are combined across the shares; anything else (a share that
  cannot be decoded blind, a failed check) falls back to rank i mod N
  counting file i whole.  Files that are neither are dealt whole, file i to
  rank i mod N;
* the per-rank uint32 count vectors and the tallies (valid k-mers, bases,
  sequences) are summed with ONE all-reduce each -- RCCL over xGMI with the
  "nccl" backend, gloo on CPU -- and rank 0 writes the .vaf and the -v report.
  uint32 counts travel as int32 tensors: two's-complement addition is
  addition modulo 2^32, so the sum is bit-identical to the reference's single
  set of uint32 counters with their relaxed atomic increments
  (vaf-counter.c:101-102,473-477), wrap-around included.

The counting timer is the reference's (first file open to counts final),
taken as the maximum over ranks after a barrier.  A rank whose counter fails
(HIP error, out of memory) tells the others through the per-file all-gather
or the agreement before the all-reduce, and every rank exits 1 -- no rank is
left waiting in a collective.  In-process multi-GPU (one process, several
devices, one RCCL reduce inside vc_finish) is the drop-in CLI's VAFC_DEVICES
(vc_create_multi); this module is the torchrun form, which is
also what bench.py runs at N > 1.  The per-rank counter is pluggable
(RankCounter): HipRankCounter is the product; the CPU tests run the same
driver with the oracle.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

NO_OFFSET = (1 << 64) - 1     # vc_range_info's UINT64_MAX ("none" / "the file ended")
EMPTY_RANGE = NO_OFFSET - 1   # a rank whose nominal byte range is empty (more ranks than bytes)

# --------------------------------------------------------------------------
# sharding and the count reduction
# --------------------------------------------------------------------------


def shard(n_items: int, rank: int, world: int):
    """Contiguous, balanced partition: (first, count) of rank's share."""
    base, extra = divmod(n_items, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def deal(items, rank: int, world: int):
    """Round-robin share of a list (item i to rank i mod world), in order."""
    return [x for i, x in enumerate(items) if i % world == rank]


def byte_range(size: int, rank: int, world: int):
    """Rank's nominal byte range [begin, end) of a size-byte file; the last
    range is open-ended (end = NO_OFFSET), so a file that grows is still read
    to its end, as the reference would."""
    begin = size * rank // world
    end = NO_OFFSET if rank == world - 1 else size * (rank + 1) // world
    return begin, end


def splittable(fn: str) -> bool:
    """A regular file that is not gzip (vc_count_file_range splits those only)."""
    try:
        if not os.path.isfile(fn):
            return False
        with open(fn, "rb") as f:
            return f.read(2) != b"\x1f\x8b"
    except OSError:
        return False


def gz_file(fn: str) -> bool:
    """A regular gzip file (split into shares of its deflate stream)."""
    try:
        if not os.path.isfile(fn):
            return False
        with open(fn, "rb") as f:
            return f.read(2) == b"\x1f\x8b"
    except OSError:
        return False


def gz_shares_chain(rows) -> bool:
    """rows[r] = (start_bit, end_bit, text_len, ok, ended, ...) of rank r's
    share scan (vc_gz_share_scan): the shares cover the stream exactly iff
    every scan is ok, the first non-empty share is rank 0's, each non-empty
    share starts at the previous non-empty share's end, and the last one ends
    the stream (include/vafc.h)."""
    if not rows or any(int(r[3]) != 1 for r in rows):
        return False
    ne = [r for r in rows if int(r[0]) != NO_OFFSET]
    if not ne or ne[0] is not rows[0]:
        return False
    for prev, cur in zip(ne, ne[1:]):
        if int(cur[0]) != int(prev[1]) or int(prev[4]) != 0:
            return False
    return int(ne[-1][4]) == 1


def gz_windows(rows, wsyms):
    """The 32 KiB of text before each rank's share: share 0's history is
    empty; the window after a share is its symbols resolved against the
    window before it (vafc.gz_window_after).  None for empty shares."""
    import vafc
    out = [None] * len(rows)
    before = np.zeros(vafc.GZ_WSIZE, np.uint8)
    prev = None
    for r, row in enumerate(rows):
        if int(row[0]) == NO_OFFSET:
            continue
        if prev is not None:
            before = vafc.gz_window_after(wsyms[prev], before)
        out[r] = before
        prev = r
    return out


def gz_crc_chain(crcs, combine) -> bool:
    """The CRC-32 accounting of the non-empty shares in order (dicts of
    vc_gz_share_crc): no member inside a share failed, every share's first
    member end checks with the tails of the shares before it
    (combine = zlib's crc32_combine), and the stream's last member closed.
    gzread checks the same members in one pass (vaf-counter.c:557)."""
    carry_crc, carry_len = 0, 0
    for c in crcs:
        if c["crc_error"] or not c["complete"]:
            return False
        if c["events"] > 0:
            crc = combine(carry_crc, c["head_crc"], c["head_len"])
            if crc != c["head_expect_crc"] or (carry_len + c["head_len"]) & 0xFFFFFFFF != c["head_expect_isize"]:
                return False
            carry_crc, carry_len = c["tail_crc"], c["tail_len"]
        else:
            carry_crc = combine(carry_crc, c["tail_crc"], c["tail_len"])
            carry_len += c["tail_len"]
    return carry_len == 0


GZ_CRC_FIELDS = ("events", "head_crc", "head_len", "head_expect_crc", "head_expect_isize", "tail_crc", "tail_len",
                 "crc_error", "complete")


def chain_holds(infos) -> bool:
    """infos[r] = (first, next, errs, stopped) of rank r's range, in rank order:
    the ranges counted exactly the file's reads iff no range met a truncated
    record and each range began where the previous one ended (vafc.h,
    vc_count_file_range).  Empty ranges (EMPTY_RANGE) count nothing and are
    passed over."""
    infos = [i for i in infos if int(i[0]) != EMPTY_RANGE]
    if not infos:
        return True
    if any(int(i[2]) != 0 for i in infos):
        return False
    if int(infos[0][0]) != 0 and int(infos[0][0]) != NO_OFFSET:
        return False
    for prev, cur in zip(infos, infos[1:]):
        if int(cur[0]) != int(prev[1]):
            return False
    return True


def counts_to_tensor(counts: np.ndarray, device="cpu"):
    import torch
    return torch.from_numpy(np.ascontiguousarray(counts, dtype=np.uint32).view(np.int32).copy()).to(device)


def tensor_to_counts(t) -> np.ndarray:
    return t.detach().cpu().numpy().astype(np.int32, copy=False).view(np.uint32)


def allreduce_counts(t, group=None):
    """In-place sum of an int32 (uint32 bit pattern) count tensor over all ranks."""
    import torch.distributed as dist
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def allreduce_u64(value: int, device="cpu", group=None) -> int:
    """Sum of one uint64 per rank (k-mers extracted, bases processed)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return int(t.item()) & 0xFFFFFFFFFFFFFFFF


def allreduce_max(value: float, device="cpu", group=None) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def allgather_u16(a: np.ndarray, world: int, device="cpu"):
    """[rank 0's array, rank 1's, ...] for equal-length uint16 arrays."""
    import torch
    import torch.distributed as dist
    # as int32 (gloo's all-gather has no 16-bit types)
    t = torch.from_numpy(np.asarray(a, dtype=np.uint16).astype(np.int32)).to(device)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.cpu().numpy().astype(np.uint16) for o in out]


def allgather_ints(values, world: int, device="cpu"):
    """[values of rank 0, values of rank 1, ...]: one all-gather of a few
    integers per rank (uint64 offsets travel as their int64 bit pattern)."""
    import torch
    import torch.distributed as dist
    v = np.asarray(values, dtype=np.uint64).view(np.int64)
    t = torch.from_numpy(v.copy()).to(device)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.cpu().numpy().view(np.uint64).tolist() for o in out]


# --------------------------------------------------------------------------
# per-rank counters
# --------------------------------------------------------------------------


class RankCounter:
    """What a rank counts with: count_range for its share of each file, then
    local_counts gives its count vector (a tensor on `device`, where the
    collective runs: the GPU with RCCL, "cpu" with gloo) and its k-mer tally.
    save / restore bracket a split file whose ranges turn out not to chain."""

    device = "cpu"

    def count_range(self, fn: str, begin: int, end: int, block: int, threads: int):
        """(ok, bases, seqs, (first, next, errs, stopped)) of the records of fn
        whose header lies in [first, end) (vafc.h vc_count_file_range); ok
        False if the file cannot be opened (skipped silently, as the reference
        does, vaf-counter.c:557).  begin = 0, end = NO_OFFSET: the whole file."""
        raise NotImplementedError

    def count_gz_share(self, fn: str, first_share: bool, start_bit: int, window, text_len: int, block: int,
                       threads: int):
        """(ok, bases, seqs, (first, next, errs, stopped), crc dict) of one
        share of a gzip file (vafc.h vc_count_gz_share): first / next in share
        coordinates; ok False if the file cannot be opened."""
        raise NotImplementedError

    # host bytes a gzip share's scan may keep for the count (0: the count
    # inflates the share again); see count_gz_share_held
    gz_hold_bytes = 0

    def count_gz_share_held(self, share, first_share: bool, window, text_len: int, block: int, threads: int):
        """count_gz_share from a share whose scan kept its decoded chunks
        (vafc.h vc_count_gz_share_held): one inflate pass instead of two."""
        raise NotImplementedError

    def gz_kmap(self):
        """The vafc.KmerMap a held share's scan is placed for (None: no placement)."""
        return None

    def save(self):
        """Remember the counts and the k-mer tally (before a split file)."""
        raise NotImplementedError

    def restore(self):
        """Return to the counts and tally of the last save()."""
        raise NotImplementedError

    def local_counts(self):
        """This rank's (counts tensor on self.device, kmers)."""
        raise NotImplementedError

    def table_info(self):
        """The key table's geometry for the -v report (vc_table_info)."""
        return {"n_keys": 0, "slots": 0, "filter_bytes": 0}

    def close(self):
        pass


class HipRankCounter(RankCounter):
    """The product: the k-mer map on this rank's GPU (vc_create), counting
    straight into a torch int32 tensor (vc_bind_outputs) that the RCCL
    all-reduce then sums in place -- no device-to-host copy before the
    collective."""

    def __init__(self, db, k: int, local_rank: int, backend: str):
        import torch
        import vafc
        self.torch = torch
        self.dev = torch.device("cuda", local_rank)
        keys, vals, _ = db.keys(k)
        # the map without create_combined_kmer_map's warning: run() prints it once, on rank 0
        self.map = vafc.KmerMap(k, keys, vals, db.n, local_rank)
        self.counts = torch.zeros(2 * db.n, dtype=torch.int32, device=self.dev)
        self.tally = torch.zeros(1, dtype=torch.int64, device=self.dev)
        # the zero fills run on torch's stream, the counting kernels on the
        # map's own stream: finish the fills before the first count
        torch.cuda.current_stream(self.dev).synchronize()
        self.map.bind_outputs(self.counts.data_ptr(), self.tally.data_ptr())
        self.device = self.dev if backend == "nccl" else "cpu"
        self._saved = None
        self.gz_hold_bytes = gz_hold_budget()

    def count_range(self, fn, begin, end, block, threads):
        try:
            st, ri = self.map.count_file_range(fn, begin, end, block, threads)
        except FileNotFoundError:
            return False, 0, 0, (NO_OFFSET, NO_OFFSET, 0, 0)
        return True, st.bases, st.seqs, (ri.first, ri.next, ri.errs, ri.stopped)

    def count_gz_share(self, fn, first_share, start_bit, window, text_len, block, threads):
        try:
            st, ri, crc = self.map.count_gz_share(fn, first_share, start_bit, window, text_len, block, threads)
        except FileNotFoundError:
            return False, 0, 0, (NO_OFFSET, NO_OFFSET, 0, 0), None
        return True, st.bases, st.seqs, (ri.first, ri.next, ri.errs, ri.stopped), crc

    def gz_kmap(self):
        return self.map

    def count_gz_share_held(self, share, first_share, window, text_len, block, threads):
        st, ri, crc = self.map.count_gz_share_held(share, first_share, window, text_len, block, threads)
        return True, st.bases, st.seqs, (ri.first, ri.next, ri.errs, ri.stopped), crc

    def save(self):
        # count_file_range returns after the map's stream is synchronised, so
        # the counts are final; the copies run on torch's stream and are
        # finished before the next count
        self._saved = (self.counts.clone(), self.tally.clone())
        self.torch.cuda.current_stream(self.dev).synchronize()

    def restore(self):
        self.counts.copy_(self._saved[0])
        self.tally.copy_(self._saved[1])
        self.torch.cuda.current_stream(self.dev).synchronize()

    def local_counts(self):
        self.map.finish()                     # the rank's batches are all counted (syncs its stream)
        t = self.counts if self.device != "cpu" else self.counts.cpu()
        return t, int(self.tally.item())

    def table_info(self):
        return self.map.table_info()

    def close(self):
        self.map.bind_outputs(0, 0)
        self.map.close()


# --------------------------------------------------------------------------
# the driver
# --------------------------------------------------------------------------


def _agree(ok: bool, world: int, device) -> bool:
    """True iff every rank is ok (so that no rank enters a collective alone)."""
    if world == 1:
        return ok
    import torch
    import torch.distributed as dist
    t = torch.tensor([0 if ok else 1], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item()) == 0


def _khashl_capacity(n: int) -> int:
    """The reference's hash table capacity for n patterns (3n rounded up to a
    power of two, at least 4), as the drop-in CLI reports it."""
    want = 3 * n
    bits = max(want.bit_length() - 1 + (1 if want & (want - 1) else 0), 2)
    return 1 << bits


def file_plan(files, rank: int, world: int, coll_device):
    """How each file is counted, decided by rank 0 and shared with one
    all-gather before the first file, so that no rank can take another branch
    (and another collective) for a file that changed meanwhile: [(kind,
    size)] with kind 1 for a regular plain file split into byte ranges, 2 for
    a regular gzip file split into shares of its stream (world > 1), 0 for a
    file dealt whole; size the file's length for kinds 1 and 2."""
    plan = []
    for fn in files:
        kind = (1 if splittable(fn) else (2 if gz_file(fn) else 0)) if world > 1 else 0
        size = -1
        if kind:
            try:
                size = os.path.getsize(fn)
            except OSError:
                kind = 0
        plan.append((kind, size if kind else NO_OFFSET))
    if world == 1:
        return [(a, b) for a, b in plan]
    flat = [x for ab in plan for x in ab] or [0]
    rows = allgather_ints(flat, world, coll_device)
    r0 = rows[0]
    return [(int(r0[2 * i]), int(r0[2 * i + 1])) for i in range(len(files))]


def count_files(files, counter, o, rank, world, err, coll_device):
    """The reference's per-file loop (vaf-counter.c:644-650) over the ranks:
    (ok, bases, seqs, fallbacks, per_file).  ok is False on every rank as soon
    as any rank's counter failed.  per_file[i] = (opened, bases, seqs,
    seconds) of file i over all ranks, for the -v line of count_fastq_kmers
    (vaf-counter.c:573-578; rank 0 prints them after the loop)."""
    bases = seqs = fallbacks = 0
    ok = True
    plan = file_plan(files, rank, world, coll_device)
    mine = [[0, 0, 0, 0] for _ in files]   # this rank's (opened, bases, seqs, microseconds) per file
    i = -1
    while i + 1 < len(files):
        i += 1
        fn = files[i]
        kind, size = plan[i]
        wave = _gz_wave(plan, i, world)
        if wave:
            # consecutive gzip files (R1.fq.gz R2.fq.gz): counted at once, each
            # by its own group of ranks, rather than one after another by all
            # of them -- fewer, larger shares, and none for a file that has a
            # rank to itself
            if rank == 0:
                for f in wave:
                    err("[M::main] Processing %s...\n" % files[f])
            groups = gz_groups([plan[f][1] for f in wave], world)
            g = next(g for g, (r0, n) in enumerate(groups) if r0 <= rank < r0 + n)
            f = wave[g]
            t_file = time.time()
            res = _count_gz_group(files[f], f, plan[f][1], groups[g][0], groups[g][1], counter, o, rank, world,
                                  err, coll_device)
            if res is None:
                ok = False
                break
            good, b, s, fell, local_ok = res
            fallbacks += fell
            ok = ok and local_ok
            bases += b
            seqs += s
            if good:
                mine[f] = [1, b, s, int(1e6 * (time.time() - t_file))]
            i = wave[-1]
            continue
        if rank == 0:
            err("[M::main] Processing %s...\n" % fn)
        t_file = time.time()
        if kind == 2:
            res = _count_gz_shares(fn, i, size, counter, o, rank, world, err, coll_device)
            if res is None:        # a rank failed inside a collective step: every rank stops
                ok = False
                break
            good, b, s, fell, local_ok = res
            fallbacks += fell
            ok = ok and local_ok
            bases += b
            seqs += s
            if good:
                mine[i] = [1, b, s, int(1e6 * (time.time() - t_file))]
            continue
        if kind == 1:
            begin, end = byte_range(size, rank, world)
            counter.save()
            failed = False
            try:
                if end <= begin:     # an empty share: nothing to count (chain_holds passes over it)
                    good, b, s, info = True, 0, 0, (EMPTY_RANGE, EMPTY_RANGE, 0, 0)
                else:
                    good, b, s, info = counter.count_range(fn, begin, end, o["b"], o["t"])
            except Exception as e:   # VafcError (HIP, memory): tell the other ranks first
                err("Error: counting failed on %s (%s)\n" % (fn, e))
                failed, good, b, s, info = True, False, 0, 0, (NO_OFFSET, NO_OFFSET, 0, 0)
            rows = allgather_ints(list(info) + [1 if good else 0, 1 if failed else 0], world, coll_device)
            if any(r[5] for r in rows):
                ok = False
                break
            if not any(r[4] for r in rows):   # the file vanished: skipped, as the reference does
                continue
            if chain_holds([r[:4] for r in rows]):
                bases += b
                seqs += s
                mine[i] = [1, b, s, int(1e6 * (time.time() - t_file))]
                continue
            # not an exact split (a truncated record, a mis-guessed boundary):
            # every rank forgets its share and rank i mod N counts the file
            # whole, so several such files spread over the ranks
            fallbacks += 1
            counter.restore()
            if i % world == rank:
                try:
                    good, b, s, _ = counter.count_range(fn, 0, NO_OFFSET, o["b"], o["t"])
                    if good:
                        bases += b
                        seqs += s
                        mine[i] = [1, b, s, int(1e6 * (time.time() - t_file))]
                except Exception as e:
                    err("Error: counting failed on %s (%s)\n" % (fn, e))
                    ok = False
            continue
        if i % world != rank:        # whole files (gzip, or one rank) dealt round robin
            continue
        try:
            good, b, s, _ = counter.count_range(fn, 0, NO_OFFSET, o["b"], o["t"])
        except Exception as e:
            err("Error: counting failed on %s (%s)\n" % (fn, e))
            ok = False
            continue
        if good:
            bases += b
            seqs += s
            mine[i] = [1, b, s, int(1e6 * (time.time() - t_file))]
    # every rank reaches this point (a failure in a split file breaks every
    # rank's loop together), so one all-gather gives rank 0 every file's totals
    if world > 1 and files:
        rows = allgather_ints([x for m in mine for x in m], world, coll_device)
        per_file = []
        for i in range(len(files)):
            parts = [r[4 * i:4 * i + 4] for r in rows]
            per_file.append((any(p[0] for p in parts), sum(p[1] for p in parts), sum(p[2] for p in parts),
                             max(p[3] for p in parts) * 1e-6))
    else:
        per_file = [(bool(m[0]), m[1], m[2], m[3] * 1e-6) for m in mine]
    return ok, bases, seqs, fallbacks, per_file


def _gz_wave(plan, i, world):
    """The files counted together from file i on (count_files): the run of
    consecutive gzip files (kind 2) starting there, at most one per rank;
    empty unless it holds two or more ($VAFC_GZ_WAVES=0: never, A/B)."""
    if os.environ.get("VAFC_GZ_WAVES") == "0":
        return []
    wave = []
    while i < len(plan) and plan[i][0] == 2 and len(wave) < world:
        wave.append(i)
        i += 1
    return wave if len(wave) >= 2 else []


def _count_gz_shares(fn, i, size, counter, o, rank, world, err, coll_device):
    """File i, a gzip file, over all the ranks: _count_gz_group with one group."""
    return _count_gz_group(fn, i, size, 0, world, counter, o, rank, world, err, coll_device)


def gz_groups(sizes, world: int):
    """Ranks per file for a wave of len(sizes) <= world gzip files counted at
    once (count_files): at least one rank each, the rest shared out by
    compressed size (largest remainder, ties to the earlier file); returns
    [(first rank, ranks)] in file order, covering ranks 0 .. world-1."""
    g = len(sizes)
    assert 1 <= g <= world
    w = [max(int(x), 1) for x in sizes]
    spare = world - g
    want = [spare * x / sum(w) for x in w]
    extra = [int(x) for x in want]
    for f in sorted(range(g), key=lambda f: (extra[f] - want[f], f))[:spare - sum(extra)]:
        extra[f] += 1
    out, r = [], 0
    for f in range(g):
        out.append((r, 1 + extra[f]))
        r += 1 + extra[f]
    return out


def _count_gz_group(fn, i, size, first, n, counter, o, rank, world, err, coll_device):
    """File i, a gzip file, over ranks first .. first+n-1 (include/vafc.h,
    vafc_gzip.h); the other ranks count other files of the same wave at the
    same time, and every rank takes part in the same three all-gathers.  One
    rank: the file whole.  Several: each scans its share of the stream, the
    shares' windows follow from the scans' symbols, each counts its share, and
    the ranges and CRC-32 accounting are checked as one chain.  Anything that
    does not chain (a share that cannot be decoded blind, a record split
    wrongly, a member that fails its check) is counted whole by rank
    first + i mod n instead, which is exactly vc_count_file.  Returns (opened,
    bases, seqs, fallbacks, ok) of this rank (ok False: its whole-file count
    failed; the other ranks go on, as for a file dealt whole), or None when a
    rank failed during the shares (all ranks stop)."""
    import vafc
    me = rank - first
    assert 0 <= me < n
    failed = False
    info = {"start_bit": NO_OFFSET, "end_bit": NO_OFFSET, "text_len": 0, "ok": 1, "ended": 0}
    wsym = np.zeros(vafc.GZ_WSIZE, np.uint16)
    hold = int(counter.gz_hold_bytes)
    share = None
    if n > 1:
        begin, end = byte_range(size, me, n)
        try:
            if end > begin and hold > 0:     # one inflate pass: the scan's chunks kept for the count
                info, wsym, share = vafc.gz_share_open(fn, begin, end, threads=o["t"], hold_bytes=hold,
                                                       kmap=counter.gz_kmap())
            elif end > begin:
                info, wsym = vafc.gz_share_scan(fn, begin, end, threads=o["t"])
        except FileNotFoundError:
            info["ok"] = 0
        except Exception as e:
            err("Error: counting failed on %s (%s)\n" % (fn, e))
            failed = True
    try:
        return _count_gz_group_scanned(fn, i, first, n, counter, o, rank, world, err, coll_device, info, wsym,
                                       share, failed)
    finally:
        if share is not None:
            share.close()


def _count_gz_group_scanned(fn, i, first, n, counter, o, rank, world, err, coll_device, info, wsym, share, failed):
    """_count_gz_group after this rank's scan (share: its held chunks, or None)."""
    import vafc
    me = rank - first
    leader = first + i % n
    rows = allgather_ints([info["start_bit"], info["end_bit"], info["text_len"], info["ok"], info["ended"],
                           1 if failed else 0], world, coll_device)
    if any(r[5] for r in rows):
        return None
    wsyms = allgather_u16(wsym, world, coll_device)
    grows = rows[first:first + n]

    def whole():
        """(good, bases, seqs, ok) of the whole-file count on this rank."""
        try:
            good, b, s, _ = counter.count_range(fn, 0, NO_OFFSET, o["b"], o["t"])
        except Exception as e:
            err("Error: counting failed on %s (%s)\n" % (fn, e))
            return False, 0, 0, False
        return (good, b, s, True) if good else (False, 0, 0, True)

    # the count: the file whole (one rank, or shares that do not chain: the
    # leader alone), else this rank's share
    split = n > 1 and gz_shares_chain(grows)
    good, b, s, rinfo, crc, local_ok = False, 0, 0, (EMPTY_RANGE, EMPTY_RANGE, 0, 0), None, True
    if not split:
        if rank == leader:
            good, b, s, local_ok = whole()
            failed = failed or (n == 1 and not local_ok)   # a lone rank's failure stops the wave
    else:
        windows = gz_windows(grows, wsyms[first:first + n])
        counter.save()
        good = True
        if int(grows[me][0]) != NO_OFFSET:
            try:
                if share is not None:
                    good, b, s, rinfo, crc = counter.count_gz_share_held(share, me == 0, windows[me],
                                                                         int(grows[me][2]), o["b"], o["t"])
                else:
                    good, b, s, rinfo, crc = counter.count_gz_share(fn, me == 0, int(grows[me][0]), windows[me],
                                                                    int(grows[me][2]), o["b"], o["t"])
            except Exception as e:
                err("Error: counting failed on %s (%s)\n" % (fn, e))
                failed = True
    cvals = [int((crc or {}).get(f, 0)) for f in GZ_CRC_FIELDS]
    res = allgather_ints(list(rinfo) + [1 if good else 0, 1 if failed else 0] + cvals, world, coll_device)
    if any(r[5] for r in res):
        return None
    if not split:
        return (good, b, s, 0 if n == 1 else 1, local_ok) if rank == leader else (False, 0, 0, 1, True)
    gres = res[first:first + n]
    nonempty = [r for r in range(n) if int(grows[r][0]) != NO_OFFSET]
    crcs = [dict(zip(GZ_CRC_FIELDS, (int(x) for x in gres[r][6:]))) for r in nonempty]
    if all(gres[r][4] for r in nonempty) and chain_holds([gres[r][:4] for r in range(n)]) and \
            gz_crc_chain(crcs, vafc.gz_crc32_combine):
        return good, b, s, 0, True
    counter.restore()
    if rank != leader:
        return False, 0, 0, 1, True
    good, b, s, local_ok = whole()
    return good, b, s, 1, local_ok


def gz_hold_budget() -> int:
    """Host bytes one rank's gzip share may keep between its scan and its
    count ($VAFC_GZ_HOLD, bytes; 0 turns holding off): by default a quarter
    of the available memory split over this node's ranks, at most 32 GiB.  A
    held share takes about 2 bytes per byte of FASTQ text (16-bit symbols,
    profiles/r06k_held.json); a share over the budget is inflated again."""
    env = os.environ.get("VAFC_GZ_HOLD")
    if env is not None:
        try:
            return max(int(env), 0)
        except ValueError:
            return 0
    avail = 0
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    avail = int(line.split()[1]) * 1024
                    break
    except OSError:
        return 0
    local_world = max(int(os.environ.get("LOCAL_WORLD_SIZE", "1")), 1)
    return min(avail // (4 * local_world), 32 << 30)


def rank_device(local: int, local_world: int, n_dev: int, backend: str, rehearsal: bool):
    """The GPU of local rank `local`: one per rank.  More ranks on this node
    than visible GPUs is refused (None): RCCL refuses duplicate GPUs, and a
    gloo run would silently put two ranks on one card under an N-GPU label.
    An explicit gloo rehearsal (VAFC_DIST_BACKEND=gloo, VAFC_REHEARSAL=1)
    wraps the ranks onto the GPUs there are."""
    if n_dev >= 1 and local_world <= n_dev and local < n_dev:
        return local
    if rehearsal and backend == "gloo" and n_dev >= 1:
        return local % n_dev
    return None


def run(argv, make_counter, rank: int = 0, world: int = 1, err=None, coll_device="cpu") -> int:
    """The reference's main over `world` ranks (torch.distributed initialised
    by the caller when world > 1).  make_counter(db, k) -> RankCounter;
    coll_device: where the status flags of the collectives live (the GPU with
    the nccl backend)."""
    import vafc
    err = err or sys.stderr.write
    o, files = vafc.parse_args(argv)
    k = o["k"]
    if not o["p"] or not o["o"] or not files:
        if rank == 0:
            err(vafc.USAGE % (k, o["t"], o["b"]))
        return 1
    t_start = time.time()
    if rank == 0:
        err("[M::main] Loading patterns...\n")
    t = time.time()
    try:
        db = vafc.load_patterns(o["p"])
    except vafc.VafcError:
        if rank == 0:
            err("Error: failed to load pattern file\n")
        return 1
    t_load = time.time() - t
    if rank == 0:
        err("[M::main] Loaded %d patterns in %.3f sec\n" % (db.n, t_load))
        err("[M::main] Creating k-mer map...\n")
    t = time.time()
    try:
        keys, vals, coll = db.keys(k)
    except vafc.VafcError:
        if rank == 0:
            err("Error: failed to create k-mer map\n")
        return 1
    if coll > 0 and rank == 0:
        err("[W::create_combined_kmer_map] Warning: %d k-mer collisions detected. "
            "Some patterns may have overlapping k-mers.\n" % coll)
    counter = None
    try:
        counter = make_counter(db, k)
    except vafc.VafcError as e:
        err("Error: failed to create k-mer map (%s)\n" % e)
    if not _agree(counter is not None, world, coll_device):
        if counter is not None:
            counter.close()
        db.close()
        return 1
    t_map = time.time() - t
    tinfo = counter.table_info()
    n_entries = int(tinfo.get("n_keys") or keys.size)
    if o["v"] and rank == 0:
        err("[V::main] Created k-mer map with %d entries in %.3f sec\n" % (n_entries, t_map))
    if rank == 0:
        err("[M::main] Counting k-mers in FASTQ files with %d threads...\n" % o["t"])
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    t = time.time()
    ok, bases, seqs, _, per_file = count_files(files, counter, o, rank, world, err, coll_device)
    if ok and o["v"] and rank == 0:
        for fn, (opened, b, sq, sec) in zip(files, per_file):
            if opened:   # count_fastq_kmers returns before its line for a file it cannot open
                err("[V::count_fastq_kmers] Processed %s: %d sequences, %d bases in %.2f sec (%.2f Mbases/sec)\n"
                    % (fn, sq, b, sec, b / sec / 1e6 if sec > 0 else 0.0))
    counts_t = None
    km = 0
    if ok:
        try:
            counts_t, km = counter.local_counts()
        except Exception as e:
            err("Error: counting failed (%s)\n" % e)
            ok = False
    if not _agree(ok, world, coll_device):
        if rank == 0:
            err("Error: counting failed\n")
        counter.close()
        db.close()
        return 1
    if world > 1:
        allreduce_counts(counts_t)
        km = allreduce_u64(km, counter.device)
        bases = allreduce_u64(bases, counter.device)
        seqs = allreduce_u64(seqs, counter.device)
    counts = tensor_to_counts(counts_t)
    t_count = time.time() - t
    if world > 1:
        t_count = allreduce_max(t_count, counter.device)
    counter.close()
    rc = 0
    if rank == 0:
        tot = int(counts.astype(np.uint64).sum())
        avg = tot / (db.n if db.n > 0 else 1)
        err("[M::main] Writing VAF file...\n")
        t = time.time()
        try:
            db.write_vaf(counts, o["o"])
        except vafc.VafcError:
            err("Error: failed to open output file\n")
            rc = 1
        t_write = time.time() - t
        if rc == 0:
            err("[M::main] Done. Average depth: %.2f\n" % avg)
        if rc == 0 and o["v"]:   # the reference's report, vaf-counter.c:686-729
            total = time.time() - t_start
            cap = _khashl_capacity(db.n)
            err("\n=== Performance Statistics ===\n")
            err("Total runtime:           %.3f sec\n" % total)
            err("  Pattern loading:       %.3f sec (%.1f%%)\n" % (t_load, 100.0 * t_load / total))
            err("  K-mer map creation:    %.3f sec (%.1f%%)\n" % (t_map, 100.0 * t_map / total))
            err("  K-mer counting:        %.3f sec (%.1f%%)\n" % (t_count, 100.0 * t_count / total))
            err("  Output writing:        %.3f sec (%.1f%%)\n" % (t_write, 100.0 * t_write / total))
            err("\nThroughput:\n")
            err("  Sequences processed:   %d\n" % seqs)
            err("  Bases processed:       %d (%.2f Mbases)\n" % (bases, bases / 1e6))
            err("  K-mers extracted:      %d (%.2f million)\n" % (km, km / 1e6))
            if t_count > 0:
                err("  Speed:                 %.2f Mbases/sec\n" % (bases / t_count / 1e6))
                err("  K-mer throughput:      %.2f million k-mers/sec\n" % (km / t_count / 1e6))
            err("\nMemory:\n")
            err("  Patterns:              %d\n" % db.n)
            err("  Hash table entries:    %d\n" % n_entries)
            err("  Hash table capacity:   %d\n" % cap)
            err("  Hash table load:       %.1f%%\n" % (100.0 * n_entries / cap))
            err("\nOptimizations:\n")
            err("  SIMD:                  MI355X HIP (gfx950), LDS prefilter %d KiB, device table %d slots\n"
                % (int(tinfo.get("filter_bytes", 0)) >> 10, int(tinfo.get("slots", 0))))
            err("  Threads:               %d workers\n" % o["t"])
            err("==============================\n")
    db.close()
    if world > 1:
        import torch
        import torch.distributed as dist
        flag = torch.tensor([rc], dtype=torch.int64, device=coll_device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)   # an output error on rank 0 fails every rank
        rc = int(flag.item())
    return rc


def main(argv=None) -> int:
    """torchrun entry: one rank per GPU, backend nccl (RCCL) by default
    (VAFC_DIST_BACKEND=gloo all-reduces on the host)."""
    argv = sys.argv[1:] if argv is None else argv
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    backend = os.environ.get("VAFC_DIST_BACKEND", "nccl")
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    n_dev = torch.cuda.device_count()
    dev = rank_device(local, local_world, n_dev, backend, os.environ.get("VAFC_REHEARSAL") == "1")
    if dev is None:
        sys.stderr.write("Error: local rank %d of %d but %d GPU(s) visible: one GPU per rank (a gloo rehearsal on "
                         "fewer GPUs needs VAFC_DIST_BACKEND=gloo VAFC_REHEARSAL=1)\n" % (local, local_world, n_dev))
        return 1
    local = dev
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    try:
        return run(argv, lambda db, k: HipRankCounter(db, k, local, backend), rank, world,
                   coll_device=torch.device("cuda", local) if backend == "nccl" else "cpu")
    finally:
        if world > 1:
            dist.destroy_process_group()


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    sys.exit(main())
