"""Shot sharding across ranks (one process per GPU, torch.distributed).

Shots are independent, so the only cross-rank traffic is bookkeeping: a
barrier around the timed region, the max of the per-rank elapsed times and the
sum of failure / convergence counts -- a few bytes, no data-path collective
(SURVEY §8(e)).  The Philox sampler is counter-based (key = seed, stream;
counter = shot index), so shot index ranges fully determine every rank's
inputs and the union over ranks equals a single-process run over the same
range.
"""
from __future__ import annotations

__all__ = ["step_shot0", "shard_range", "reduce_counts", "max_time", "barrier"]


def step_shot0(step: int, world: int, rank: int, per_rank: int) -> int:
    """First shot index of `rank` at weak-scaling step `step` (each step every
    rank decodes `per_rank` fresh shots: ranks interleave by step)."""
    return (step * world + rank) * per_rank


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) share of `total` shots for strong-scaling runs."""
    per = -(-total // world)
    lo = min(total, rank * per)
    return lo, min(total, lo + per)


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def reduce_counts(values, device=None):
    """Sum integer counters over ranks (identity when not distributed)."""
    import torch
    t = torch.as_tensor(values, dtype=torch.int64, device=device)
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(t)
    return t.cpu().tolist()


def max_time(seconds: float, device=None) -> float:
    import torch
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    d.all_reduce(t, op=d.ReduceOp.MAX)
    return float(t.item())


def barrier() -> None:
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.barrier()
