"""One process per GPU: the drop-in vaf-counter as a torchrun job.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        kmer-cnt_amd/vafc_dist.py [-v] -k 21 -p patterns.txt -o sample.vaf R1.fq.gz R2.fq.gz ...

Same flags, messages, exit codes and .vaf as the reference's main
(vaf-counter.c:584-735) and the drop-in CLI.  Reads are independent units, so
the path shards with no data-path collective:

* every rank loads the patterns and builds its own replica of the static
  key table on its GPU (load_patterns / create_combined_kmer_map,
  vaf-counter.c:149-252);
* input files are dealt round robin to the ranks (file i to rank i mod N) and
  counted whole with vc_count_file.  A file is the unit because the
  reference's block loop -- -b blocks in file order, a file ending at its
  third empty block (vaf-counter.c:486-517, kthread.c:97-128) -- is a property
  of one file's record sequence; splitting a file across processes would need
  that state passed between them;
* the per-rank uint32 count vectors and the tallies (valid k-mers, bases,
  sequences) are summed with ONE all-reduce each -- RCCL over xGMI with the
  "nccl" backend, gloo on CPU -- and rank 0 writes the .vaf and the -v report.
  uint32 counts travel as int32 tensors: two's-complement addition is
  addition modulo 2^32, so the sum is bit-identical to the reference's single
  set of uint32 counters with their relaxed atomic increments
  (vaf-counter.c:101-102,473-477), wrap-around included.

The counting timer is the reference's (first file open to counts final),
taken as the maximum over ranks after a barrier.  In-process multi-GPU (one
process, several devices, one RCCL reduce inside vc_finish) is the drop-in
CLI's VAFC_DEVICES (vc_create_multi); this module is the
torchrun form of the same reduction, which is also what bench.py runs at
N > 1.  The per-rank counter is pluggable (RankCounter): HipRankCounter is
the product; the CPU tests run the same driver with the oracle.
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

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


# --------------------------------------------------------------------------
# per-rank counters
# --------------------------------------------------------------------------


class RankCounter:
    """What a rank counts with: count_file for each of its files, then
    local_counts gives its count vector (a tensor on `device`, where the
    collective runs: the GPU with RCCL, "cpu" with gloo) and its k-mer tally."""

    device = "cpu"

    def count_file(self, fn: str, block: int, threads: int):
        """(ok, bases, seqs); ok False if the file cannot be opened (skipped
        silently, as the reference does, vaf-counter.c:557)."""
        raise NotImplementedError

    def local_counts(self):
        """This rank's (counts tensor on self.device, kmers)."""
        raise NotImplementedError

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
        self.map = vafc.create_combined_kmer_map(db, k, device=local_rank)
        self.counts = torch.zeros(2 * db.n, dtype=torch.int32, device=self.dev)
        self.tally = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.map.bind_outputs(self.counts.data_ptr(), self.tally.data_ptr())
        self.device = self.dev if backend == "nccl" else "cpu"

    def count_file(self, fn, block, threads):
        try:
            st = self.map.count_file(fn, block, threads)
        except FileNotFoundError:
            return False, 0, 0
        return True, st.bases, st.seqs

    def local_counts(self):
        self.map.finish()                     # the rank's batches are all counted (syncs its stream)
        t = self.counts if self.device != "cpu" else self.counts.cpu()
        return t, int(self.tally.item())

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
    if o["v"] and rank == 0:
        err("[V::main] Created k-mer map with %d entries in %.3f sec\n" % (keys.size, t_map))
    if rank == 0:
        err("[M::main] Counting k-mers in FASTQ files with %d threads...\n" % o["t"])
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    t = time.time()
    bases = seqs = 0
    mine = deal(list(range(len(files))), rank, world)
    for i in mine:
        fn = files[i]
        err("[M::main] Processing %s...\n" % fn)
        ok, b, s = counter.count_file(fn, o["b"], o["t"])
        if ok:
            bases += b
            seqs += s
    counts_t, km = counter.local_counts()
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
        if rc == 0 and o["v"]:
            total = time.time() - t_start
            err("\n=== Performance Statistics ===\n")
            err("Total runtime:           %.3f sec\n" % total)
            err("  K-mer counting:        %.3f sec (%.1f%%)\n" % (t_count, 100.0 * t_count / total))
            err("  Output writing:        %.3f sec (%.1f%%)\n" % (t_write, 100.0 * t_write / total))
            err("\nThroughput:\n")
            err("  Sequences processed:   %d\n" % seqs)
            err("  Bases processed:       %d (%.2f Mbases)\n" % (bases, bases / 1e6))
            err("  K-mers extracted:      %d (%.2f million)\n" % (km, km / 1e6))
            if t_count > 0:
                err("  Speed:                 %.2f Mbases/sec\n" % (bases / t_count / 1e6))
                err("  K-mer throughput:      %.2f million k-mers/sec\n" % (km / t_count / 1e6))
            err("  Ranks:                 %d (files dealt round robin, one all-reduce of the counts)\n" % world)
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
    local = local % max(torch.cuda.device_count(), 1)
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
