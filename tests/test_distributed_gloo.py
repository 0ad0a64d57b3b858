"""world_size-2 rehearsal of the multi-GPU path on CPU (gloo): ranks sample and
decode their own shot ranges (the CPU oracle stands in for the device here),
reduce failure counts and max elapsed time, and the totals equal a single-process
run over the same shots -- the property bench.py and p_sweep rely on."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, per_rank, steps, q):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from conftest import load_checks, load_code
    from exp_ldpc_amd.sharding import barrier, max_time, reduce_counts, step_shot0
    from oracle import load
    hx, hz = load_checks("hgp_12_3_4_s1234")
    lz = load_code("hgp_12_3_4_s1234").logicals.z
    orc = load()
    fails = conv = 0
    barrier()
    for s in range(steps):
        shot0 = step_shot0(s, world, rank, per_rank)
        syn, rd = orc.sample_storage(hz, 0, 0.02, 0.02, seed=11, stream=0, shot0=shot0, B=per_rank, nthreads=1)
        out = orc.decode(hz, 0.02 * 2 / 3, syn, method="ms", precision="f32", max_iter=30, ssf=True, gens=hx,
                         lz=lz, readout=rd, want_llr=False, nthreads=1, ssf_impl="fast")
        fails += int(out["fail"].sum())
        conv += int((out["status"] & 1).sum())
    total = reduce_counts([fails, conv])
    t = max_time(float(rank + 1))
    barrier()
    if rank == 0:
        q.put((total, t))
    dist.destroy_process_group()


def test_two_rank_sharding_equals_single_process(oracle_lib):
    from conftest import load_checks, load_code
    world, per_rank, steps = 2, 300, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per_rank, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    (fails, conv), t = q.get(timeout=10)
    assert t == 2.0  # max over ranks
    hx, hz = load_checks("hgp_12_3_4_s1234")
    lz = load_code("hgp_12_3_4_s1234").logicals.z
    total = world * per_rank * steps
    syn, rd = oracle_lib.sample_storage(hz, 0, 0.02, 0.02, seed=11, stream=0, shot0=0, B=total)
    out = oracle_lib.decode(hz, 0.02 * 2 / 3, syn, method="ms", precision="f32", max_iter=30, ssf=True, gens=hx,
                            lz=lz, readout=rd, want_llr=False, ssf_impl="fast")
    assert fails == int(out["fail"].sum())
    assert conv == int((out["status"] & 1).sum())
