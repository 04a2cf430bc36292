"""Multi-GPU sharding of record batches.

Records encode and decode independently, so a batch splits into contiguous record ranges,
one per GPU (one process per GPU), with no data-path collective.  The only cross-rank
step is on control data: the exclusive scan of the G per-shard byte totals that turns
each shard's local record offsets into offsets of the single global stream (G <= 8
integers, one all_gather).  Concatenating the shard streams in rank order then yields
exactly the stream a single encode of the whole batch produces.
"""
from __future__ import annotations

import numpy as np


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous record range [lo, hi) of `rank`: sizes differ by at most one record."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def shard_columns(var_cols, lo: int, hi: int):
    """Slice (bytes, offs[n+1]) string columns to records [lo, hi) with offsets rebased to 0."""
    out = []
    for b, o in var_cols:
        a, z = int(o[lo]), int(o[hi])
        out.append((b[a:z], (o[lo:hi + 1] - o[lo]).astype(np.uint64)))
    return out


def exclusive_scan(totals) -> list[int]:
    acc, out = 0, []
    for t in totals:
        out.append(acc)
        acc += int(t)
    return out


def global_base(local_total: int, group=None) -> tuple[int, int]:
    """(this rank's byte offset in the global stream, global total) via one all_gather of totals."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return 0, int(local_total)
    world = dist.get_world_size(group)
    backend = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    mine = torch.tensor([int(local_total)], dtype=torch.int64, device=dev)
    allt = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allt, mine, group=group)
    totals = [int(t.item()) for t in allt]
    return exclusive_scan(totals)[dist.get_rank(group)], sum(totals)
