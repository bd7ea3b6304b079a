"""Batch×head sharding across the GPUs of one node (one process per GPU).

The attention op is embarrassingly parallel over the flattened batch ``b``
(every (batch, head) slice is independent in forward and backward — the
reference's grid.y = b, flash_attention.cu:2176), and the batch dims are the
outermost in the channel-first layout ``[b][c][n]``.  So a rank's shard is a
contiguous slab of slices: a pointer offset, no copy, and NO collective on the
data path.  The only inter-rank traffic is control: a barrier and a max-reduce
of timings (gloo over host memory), used by bench.py.
"""

from __future__ import annotations

import os
from typing import Tuple


def dist_env() -> Tuple[int, int, int]:
    """(world_size, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(b: int, world: int, rank: int) -> Tuple[int, int]:
    """[start, stop) of the flattened batch slices owned by `rank` (balanced, contiguous;
    the first b % world ranks take one extra slice)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad world/rank {world}/{rank}")
    q, rem = divmod(int(b), world)
    start = rank * q + min(rank, rem)
    return start, start + q + (1 if rank < rem else 0)


def local_shard(t, seq_dims: int, world: int, rank: int):
    """View of this rank's slab of a channel-first tensor batch_shape + (C, *seq):
    the batch dims are flattened, then sliced [start:stop] (a view: no copy)."""
    batch = t.shape[:t.dim() - seq_dims - 1]
    b = 1
    for s in batch:
        b *= int(s)
    flat = t.reshape((b,) + tuple(t.shape[len(batch):]))
    start, stop = shard_range(b, world, rank)
    return flat[start:stop]


def max_over_ranks(values, group=None):
    """Element-wise max of a list of floats over all ranks (gloo/host tensors)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [float(x) for x in t]


def sum_over_ranks(values, group=None):
    """Element-wise sum of a list of floats over all ranks (gloo/host tensors)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return [float(x) for x in t]
