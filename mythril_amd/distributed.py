"""Multi-GPU witness search: one process per GPU.

The candidate index range of every query is split into contiguous per-rank
slices; each rank searches its slice for ALL queries in one launch (programs
are replicated — they are KBs), then ONE ``all_reduce(MIN)`` of an int64
vector (one entry per query) over ``torch.distributed`` combines the lowest
witness indices: backend ``nccl`` (= RCCL over xGMI on MI355X) with
device tensors, ``gloo`` for CPU tests.  8 B per query: latency-bound, so the
collective is negligible next to a search.  The winning rank's index is
materialised by whichever rank owns it; since candidates are a deterministic
function of the index, any rank can regenerate the witness without a transfer.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

NONE = (1 << 64) - 1   # MG_NONE: no witness (never a candidate index: mg_search rejects ranges past it)
_BIAS = 1 << 63


def _to_i64(v: Optional[int]) -> int:
    """u64 index -> int64 with the order preserved (x - 2^63), so MIN over the
    signed tensor is MIN over the unsigned indices; "none" is the largest."""
    u = NONE if v is None else int(v)
    if not 0 <= u <= NONE:
        raise ValueError(f"witness index out of u64 range: {u}")
    return u - _BIAS


def _from_i64(x: int) -> Optional[int]:
    u = int(x) + _BIAS
    return None if u == NONE else u


def shard_range(begin: int, count: int, rank: int, world: int) -> Tuple[int, int]:
    base, rem = divmod(count, world)
    start = begin + rank * base + min(rank, rem)
    return start, base + (1 if rank < rem else 0)


def allreduce_min(values: Sequence[Optional[int]], device: Optional[str] = None) -> List[Optional[int]]:
    import torch
    import torch.distributed as dist
    t = torch.tensor([_to_i64(v) for v in values], dtype=torch.int64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return [_from_i64(x) for x in t.tolist()]


def sharded_search(engine, queries, count: int, begin: int = 0, flags: Optional[int] = None,
                   device: Optional[str] = None):
    """Search [begin, begin+count) of every query across all ranks; returns the
    global lowest witness index per query (identical on every rank) and this
    rank's kernel statistics."""
    import torch.distributed as dist
    from . import isa
    rank, world = dist.get_rank(), dist.get_world_size()
    b, c = shard_range(begin, count, rank, world)
    flags = (isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT) if flags is None else flags
    dps = [engine.dev.load(q.program) for q in queries]
    try:
        found, st = engine.dev.search(dps, engine.seed, b, c, flags) if c > 0 else ([None] * len(queries), {})
    finally:
        for dp in dps:
            dp.free()
    return allreduce_min(found, device), st
