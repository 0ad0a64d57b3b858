"""Shot sharding across ranks (one process per GPU, torch.distributed).

Shots are independent, so the only cross-rank traffic is bookkeeping: a
barrier around the timed region, the max of the per-rank elapsed times and the
sum of failure / convergence counts -- a few bytes, no data-path collective
(the reference's fan-out is `Pool(cpu_count())` over shots,
misc/p_sweep.py:17-40, which exchanges only the per-worker failure counts).

Those few bytes live on the host, so the process group is `gloo` on every
path (GPU ranks and the CPU rehearsal alike) and every collective here takes a
CPU tensor: the code a CPU test runs is exactly the code an 8-GPU node runs.
Nothing of the decode crosses ranks, so no RCCL communicator is created.  The
Philox sampler is counter-based (key = seed, stream; counter = shot index), so
shot index ranges fully determine every rank's inputs and the union over ranks
equals a single-process run over the same range.
"""
from __future__ import annotations

__all__ = ["BOOKKEEPING_BACKEND", "init_process_group", "rank_device", "step_shot0", "shard_range",
           "reduce_counts", "max_time", "barrier", "gather_rows"]

# the backend of the bookkeeping group: host tensors only (see the module doc)
BOOKKEEPING_BACKEND = "gloo"


def init_process_group(**kw) -> None:
    """Join the bookkeeping group (env:// rendezvous: RANK / WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT, as torchrun sets them).  Gloo announces its
    connections on the process's stdout (C++ printf), which would land beside
    rank 0's one JSON line, so stdout is pointed at stderr while it connects."""
    import os
    import sys

    import torch.distributed as dist
    if dist.is_initialized():
        return
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        dist.init_process_group(BOOKKEEPING_BACKEND, **kw)
        barrier()  # every pair connected before stdout is restored
    finally:
        sys.stdout.flush()
        try:  # C stdio buffers too (the announcements are C++ prints)
            import ctypes
            ctypes.CDLL(None).fflush(None)
        except Exception:
            pass
        os.dup2(saved, 1)
        os.close(saved)


def rank_device(local_rank: int, device_count: int) -> int:
    """HIP device of a local rank: one GPU per rank; ranks beyond the visible
    devices share them round-robin (a 1-GPU box can rehearse N ranks)."""
    if device_count <= 0:
        raise RuntimeError("no HIP device visible")
    return int(local_rank) % int(device_count)


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


def _host(values, dtype):
    """A CPU tensor of `values` (device tensors are copied to the host first)."""
    import torch
    if isinstance(values, torch.Tensor):
        return values.detach().to("cpu", dtype)
    return torch.as_tensor(values, dtype=dtype)


def reduce_counts(values) -> list:
    """Sum integer counters over ranks (identity when not distributed)."""
    import torch
    t = _host(values, torch.int64).clone()
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(t)
    return t.tolist()


def max_time(seconds: float) -> float:
    """The maximum of `seconds` over ranks."""
    import torch
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return float(seconds)
    t = torch.tensor([float(seconds)], dtype=torch.float64)
    d.all_reduce(t, op=d.ReduceOp.MAX)
    return float(t.item())


def gather_rows(values) -> list:
    """Every rank's row of floats, in rank order (one all_gather of host words;
    [values] when not distributed): per-rank timings and device ordinals for
    rank 0's report."""
    import torch
    t = _host(values, torch.float64).clone().reshape(-1)
    d = _dist()
    if d is None or d.get_world_size() == 1:
        return [t.tolist()]
    out = [torch.zeros_like(t) for _ in range(d.get_world_size())]
    d.all_gather(out, t)
    return [o.tolist() for o in out]


def barrier() -> None:
    """Host barrier over the bookkeeping group: an all-reduce of one CPU word
    (dist.barrier() would pick a device by itself)."""
    import torch
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(torch.zeros(1, dtype=torch.int32))
