"""Throughput benchmark: decoded syndrome shots/s + logical error rate on the
(3,4)-HGP n=225 code (BASELINE.json configs[1] = SURVEY §8(d) C2).

One step = one pass of the hot path over one batch per sweep point: for each
p in geomspace(1e-3, 1e-1, 9), decode B device-resident storage-experiment shots
(R = 0: H = Hz 108x225) with BP min-sum (fp32, max_iter 50, alpha_t = 1-2^-t)
+ small-set-flip on BP failures + fused logical-failure check.  Inputs for every
step are sampled on the device *before* the timed region (distinct shots per
step; on-device Philox sampler), so the timed region is decode only.

Multi-GPU (`torchrun --nproc-per-node N bench.py --gpus N`): one process per GPU;
shots are sharded by index (rank r decodes shot range r*B..), no data-path
collective; a barrier + synchronize brackets the timed region and rank 0 reports
the max time over ranks.  value = shots decoded by all ranks / that time.

The 9 sweep points are spread round-robin over --streams HIP streams (default
5), so a point's SSF kernel (latency-bound, few waves) and another point's BP
kernel (VALU-bound) overlap; kernel durations are then measured under that
overlap (`--streams 1` gives isolated kernel times).

Also reported: `roofline` for the BP kernel (algorithmic bytes per launch per
SURVEY §8(d): 334 B/shot of I/O + 16*E B per BP iteration, over the BP kernel's
average launch duration measured with HIP events the library records on the
launch stream immediately around it; the SSF kernel's time is listed beside), and
`cpu_baseline`: the CPU oracle (oracle/, a C port of the same algorithm, OpenMP)
timed on the host cores on a bounded sample of the same workload (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "decoded syndrome shots/sec + logical error rate, (3,4)-HGP n=225 @ 1/2/4/8 GPUs"
CODE = "hgp_12_3_4_s1234"
SEED = 20250221
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def wilson(k: int, n: int, z: float = 1.96):
    if n == 0:
        return (0.0, 1.0)
    ph = k / n
    den = 1 + z * z / n
    c = (ph + z * z / (2 * n)) / den
    h = z * math.sqrt(ph * (1 - ph) / n + z * z / (4 * n * n)) / den
    return (max(0.0, c - h), min(1.0, c + h))


def load_code():
    from exp_ldpc_amd.codes import read_quantum_code
    with open(os.path.join(REPO, "tests", "golden", f"{CODE}.qecc")) as f:
        return read_quantum_code(f, validate_stabilizer_code=True)


def latest_traffic():
    """Per-launch HBM bytes of the decode kernel from the newest committed PMC
    summary (profiles/*_pmc_summary.json, written by tools/pmc_summary.py)."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_summary.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            return json.load(f).get("decode_kernel_hbm_bytes_per_launch")
    except Exception:
        return None


def cpu_baseline(code, ps, args, gpu_ler):
    """Time the CPU oracle on a bounded sample of the same workload."""
    from oracle import load as load_oracle
    orc = load_oracle()
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    per_p = args.cpu_shots
    total = 0
    elapsed = 0.0
    fails = {}
    for pi, p in enumerate(ps):
        syn, rd = orc.sample_storage(hz, 0, p, p, seed=SEED, stream=pi, shot0=0, B=per_p, nthreads=threads)
        t0 = time.perf_counter()
        out = orc.decode(hz, 2 * p / 3, syn, method="ms", precision="f32", max_iter=50, ssf=True, gens=hx, lz=lz,
                         readout=rd, want_llr=False, nthreads=threads, ssf_impl="fast")
        elapsed += time.perf_counter() - t0
        total += per_p
        fails[f"{p:.6g}"] = int(out["fail"].sum())
    return {"value": total / elapsed, "unit": "shots/s", "cores": threads, "kind": "port",
            "sample": f"{per_p} shots at each of the {len(ps)} sweep points (same sampler/seed as the GPU run, "
                      f"shot indices 0..{per_p - 1}); decode only, sampling excluded; {elapsed:.1f} s of CPU work",
            "failures_per_point": fails}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1 << 18, help="shots per sweep point per step per GPU")
    ap.add_argument("--points", type=int, default=9)
    ap.add_argument("--p", type=float, action="append", help="decode only these p values (diagnostics)")
    ap.add_argument("--cpu-shots", type=int, default=200000, help="CPU-baseline shots per sweep point")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=5, help="HIP streams the sweep points are spread over")
    ap.add_argument("--heavy-first", action="store_true", help="launch the sweep points from the highest p down")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from exp_ldpc_amd.decoder import Decoder

    code = load_code()
    hz, hx, lz = code.checks.z, code.checks.x, code.logicals.z
    m, n = hz.shape
    E = int(hz.nnz)
    ps = np.geomspace(1e-3, 1e-1, args.points) if not args.p else np.array(args.p)
    B = args.batch
    nsteps = args.warmup + args.steps

    dec = Decoder(hz, 2 * ps[0] / 3, method="ms", precision="f32", max_iter=50, ms_scaling=0.0,
                  flip_sets=hx, logicals=lz, device=local)
    # one decoder graph per sweep point (priors differ), sharing nothing mutable
    decs = [dec] + [Decoder(hz, 2 * p / 3, method="ms", precision="f32", max_iter=50, flip_sets=hx, logicals=lz,
                            device=local) for p in ps[1:]]

    # ---- inputs: distinct shots for every (step, point), sampled on device ----
    syn = torch.empty((nsteps, len(ps), B, m), dtype=torch.uint8, device=dev)
    rd = torch.empty((nsteps, len(ps), B, n), dtype=torch.uint8, device=dev)
    for s in range(nsteps):
        for pi, p in enumerate(ps):
            shot0 = (s * world + rank) * B
            dec.sample_storage_device(0, p, p, SEED, pi, shot0, B, syn[s, pi], rd[s, pi])
    iters = torch.empty((nsteps, len(ps), B), dtype=torch.int32, device=dev)
    status = torch.empty((nsteps, len(ps), B), dtype=torch.uint8, device=dev)
    fail = torch.empty((nsteps, len(ps), B), dtype=torch.uint8, device=dev)
    ssf_steps = torch.empty((nsteps, len(ps), B), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    # sweep points round-robin over HIP streams, so one point's SSF kernel (few,
    # latency-bound waves) overlaps the next point's BP kernel (VALU-bound); each
    # point has its own decoder handle, hence its own queue and timing events
    main = torch.cuda.current_stream(dev)
    streams = [main] + [torch.cuda.Stream(dev) for _ in range(max(1, args.streams) - 1)]

    order = list(range(len(ps)))[::-1] if args.heavy_first else list(range(len(ps)))

    def step(s):
        ev = torch.cuda.Event()
        ev.record(main)
        for st in streams[1:]:
            st.wait_event(ev)
        for li, pi in enumerate(order):
            st = streams[li % len(streams)]
            decs[pi].decode_device(B, syn=syn[s, pi], readout=rd[s, pi], iters=iters[s, pi], status=status[s, pi],
                                   fail=fail[s, pi], ssf_steps=ssf_steps[s, pi], stream=st.cuda_stream)
        for st in streams[1:]:
            e2 = torch.cuda.Event()
            e2.record(st)
            main.wait_event(e2)

    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    # HIP events recorded by the library on the launch stream right before the
    # BP kernel, after it and after the SSF kernel of every timed call
    for d in decs:
        d.set_timing(args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, nsteps):
        step(s)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # ---- per-launch kernel times and algorithmic bytes ----
    bp_ms = np.zeros((args.steps, len(ps)))
    ssf_ms = np.zeros((args.steps, len(ps)))
    for pi, d in enumerate(decs):
        a, c = d.read_timing()
        bp_ms[:, pi] = a
        ssf_ms[:, pi] = c
    launch_ms = bp_ms
    it_sum = iters[args.warmup:].to(torch.int64).sum(dim=2).cpu().numpy()  # [steps, points]
    b_io = m + n + 1  # syndrome in + correction out + failure flag
    bytes_per_launch = b_io * B + 16 * E * it_sum  # [steps, points]
    achieved_gbs = float(bytes_per_launch.sum() / (launch_ms.sum() * 1e-3) / 1e9)

    fails = fail[args.warmup:].to(torch.int64).sum(dim=(0, 2))
    conv = (status[args.warmup:] & 1).to(torch.int64).sum(dim=(0, 2))
    itp = iters[args.warmup:].to(torch.float64).mean(dim=(0, 2))
    ssp = ssf_steps[args.warmup:].to(torch.float64).mean(dim=(0, 2))
    if world > 1:
        dist.all_reduce(fails)
        dist.all_reduce(conv)
    fails = fails.cpu().numpy()
    conv = conv.cpu().numpy()
    shots_per_point = args.steps * B * world

    if rank == 0:
        total_shots = shots_per_point * len(ps)
        value = total_shots / elapsed
        ler = {}
        for pi, p in enumerate(ps):
            lo, hi = wilson(int(fails[pi]), shots_per_point)
            ler[f"{p:.6g}"] = {"failures": int(fails[pi]), "shots": shots_per_point,
                               "ler": float(fails[pi] / shots_per_point), "wilson95": [lo, hi],
                               "bp_converged_frac": float(conv[pi] / shots_per_point),
                               "mean_bp_iters_rank0": float(itp[pi]),
                               "mean_ssf_steps_rank0": float(ssp[pi]),
                               "bp_kernel_ms_per_launch": float(bp_ms[:, pi].mean()),
                               "ssf_kernel_ms_per_launch": float(ssf_ms[:, pi].mean())}
        traffic = latest_traffic()
        result = {
            "metric": METRIC, "value": value, "unit": "shots/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: on-device Philox sampler of the storage experiment under depolarizing_noise(p, pm=p), "
                    "seed 20250221, distinct shots per step",
            "config": {"workload": "C2: (3,4)-HGP n=225 (biregular_hgp(12,3,4,seed=1234)), R=0 (H=Hz 108x225, E=756), "
                                   "p-sweep geomspace(1e-3,1e-1,9), BP min-sum fp32 max_iter=50 alpha_t=1-2^-t + SSF "
                                   "(Hx flip sets) + fused logical check",
                       "shots_per_point_per_step_per_gpu": B, "global_batch": B * len(ps) * world,
                       "parallelism": f"shot-sharded x{world}, no collective", "streams": args.streams},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "bp_ms_wave_kernel<float, 2, 4, 7, true, true, 2> (BP min-sum, fp32, lean outputs, queues BP failures)",
                         "avg_launch_ms": float(launch_ms.mean()),
                         "launches": int(launch_ms.size),
                         "ssf_kernel": "ssf_wave_kernel<2, 4, 2>", "ssf_avg_launch_ms": float(ssf_ms.mean()),
                         "timing": "HIP events recorded by the library on the launch stream around each kernel",
                         "algorithmic_bytes_per_launch": float(bytes_per_launch.mean()),
                         "bytes_model": "per shot: (m+n+1)=334 B I/O + 16*E=12096 B per BP iteration"},
            "ler": ler,
        }
        if not args.no_cpu_baseline and world == 1:
            result["cpu_baseline"] = cpu_baseline(code, ps, args, ler)
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
