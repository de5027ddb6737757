"""Multi-GPU plumbing for the cleaning path.

C1/C2/C5 are "replicas only" and C4 is a batch of independent archives: one
process per GPU (torchrun), each cleaning its own archives, with no collective
on the data path.  The only cross-rank operation is the timing reduction of
bench.py (max over ranks).  The reference processes its archive list in one
loop (iterative_cleaner.py:59-62); ``shard`` splits that list across ranks.
"""
from __future__ import annotations

import os
from typing import Sequence, TypeVar

T = TypeVar("T")


def rank_world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (1 process: 0, 1, 0)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad RANK/WORLD_SIZE: %d/%d" % (rank, world))
    return rank, world, local


def shard(items: Sequence[T], rank: int, world: int) -> list[T]:
    """Round-robin share of ``items`` for ``rank`` (disjoint, covers every item once,
    keeps the reference's processing order within a rank)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world: %d/%d" % (rank, world))
    return list(items[rank::world])


def max_over_ranks(value: float, device=None) -> float:
    """MAX all-reduce of one float (bench timing); identity without a process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
