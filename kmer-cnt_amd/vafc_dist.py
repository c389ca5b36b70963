"""Multi-GPU plumbing for the vaf-counter hot path.

Reads are independent units, so the path shards with no data-path collective:
rank r counts its own shard of reads (a contiguous range of the read stream, or
its own files) into a per-GPU uint32 count vector, and ONE all-reduce sums the
vectors before rank 0 writes the .vaf.  With the "nccl" backend this is RCCL
over xGMI; on CPU (tests) it is gloo.

This module is only the one-process-per-GPU (torchrun) side used by bench.py
and tests/test_synth_dist.py.  The product path for the drop-in CLI is
in-process: vc_create_multi (include/vafc.h) holds one table replica and
count vector per device and reduces them with RCCL inside vc_finish
(DESIGN.md §6).

uint32 counts are carried as int32 tensors: two's-complement addition is
addition modulo 2^32, so the reduced vector is bit-identical to the
reference's single-process uint32 counters (vaf-counter.c:101-102,473-477),
including wrap-around.
"""
from __future__ import annotations

import numpy as np


def shard(n_items: int, rank: int, world: int):
    """Contiguous, balanced partition: (first, count) of rank's share."""
    base, extra = divmod(n_items, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


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
