"""The multi-GPU bench's bookkeeping runs on the backend it will run on.

bench.py --gpus N (one process per GPU, the driver's 1/2/4/8-GPU runs) joins a
gloo group through exp_ldpc_amd.sharding and issues every collective through
its helpers on host words, so this CPU rehearsal exercises the same calls the
GPU ranks make (reference fan-out: misc/p_sweep.py:17-40, Pool workers whose
failure counts are summed on the host)."""
import ast
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_issues_no_collective_of_its_own():
    """bench.py calls no torch.distributed collective directly and never asks
    for nccl: the barrier, max-time and count reductions all go through
    sharding.py (host tensors, gloo)."""
    tree = ast.parse(open(os.path.join(REPO, "bench.py")).read())
    direct = {"all_reduce", "barrier", "all_gather", "broadcast", "reduce", "gather", "scatter"}
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute):
            base = node.func.value
            if isinstance(base, ast.Name) and base.id == "dist":
                assert node.func.attr not in direct | {"init_process_group"}, f"bench.py:{node.lineno} dist.{node.func.attr}"
        if isinstance(node, ast.Constant) and isinstance(node.value, str):
            assert "nccl" not in node.value.lower(), f"bench.py:{node.lineno} names nccl"
    from exp_ldpc_amd import sharding
    assert sharding.BOOKKEEPING_BACKEND == "gloo"


def test_rank_device_round_robin():
    from exp_ldpc_amd.sharding import rank_device
    assert [rank_device(r, 8) for r in range(8)] == list(range(8))
    assert [rank_device(r, 1) for r in range(3)] == [0, 0, 0]
    with pytest.raises(RuntimeError):
        rank_device(0, 0)


def _worker(rank, world, port, q):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from exp_ldpc_amd.sharding import barrier, init_process_group, max_time, reduce_counts
    init_process_group()
    assert dist.get_backend() == "gloo"
    barrier()
    # counts arrive as (device) tensors in bench.py: the helper moves them to the host
    counts = reduce_counts(torch.tensor([rank + 1, 10 * rank, 7], dtype=torch.int64))
    lst = reduce_counts([1, 2])
    t = max_time(0.5 + rank)
    barrier()
    if rank == 0:
        q.put((counts, lst, t))
    dist.destroy_process_group()


def test_sharding_helpers_two_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    counts, lst, t = q.get(timeout=10)
    assert counts == [3, 10, 14]
    assert lst == [2, 4]
    assert t == 1.5


def test_helpers_without_process_group():
    from exp_ldpc_amd.sharding import barrier, max_time, reduce_counts
    assert reduce_counts(torch.tensor([4, 5])) == [4, 5]
    assert max_time(2.0) == 2.0
    barrier()
