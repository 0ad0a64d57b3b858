"""Throughput of the larger BASELINE configs on one MI355X (diagnostic; the
driver's headline bench is bench.py = config 2).

  c3    [[144,12,12]] bivariate-bicycle lift, BP min-sum (max_iter 50) + SSF
  c4    biregular_hgp(80,3,4,seed=2025), n = 10^4, BP min-sum (max_iter 50) + SSF
  c5    config 5 as named: PSL(2,16) Cayley-graph LP code
        lifted_product_code_pgl2(1,4,2,double_cover=False,seed=1), n = 53,040,
        R = 1 spacetime syndromes (48,960 x 130,560), BP min-sum max_iter 50,
        fold + logical check (k = 4080)
  c5r0  the same code at R = 0: BP min-sum max_iter 50 + SSF + logical check
  c5m   PSL(2,13) matrix lift, n = 49,140, R = 1 spacetime, BP min-sum (the
        round-1/2 stand-in for config 5, kept as an extra graph)

Every line is run at each --precision (default f32 and f64; ldpc decodes in
f64) and records it.  Shots are sampled on the device (storage experiment,
depolarizing_noise(p, pm=p)) before the timed region; the timed region decodes
them (fused fold + logical check where logicals are given).  Prints one JSON
line per (config, precision, p).

Usage: python tools/bench_configs.py [c3 c4 c5 c5r0 c5m] [--shots N] [--p P ...] [--precision f32 f64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

SEED = 20250221


def build_config(name):
    import scipy.sparse as sp
    from conftest import load_checks
    from exp_ldpc_amd import gf2
    if name == "c3":
        from exp_ldpc_amd.lifted import bivariate_bicycle_code
        code = bivariate_bicycle_code(12, 6, [(3, 0), (0, 1), (0, 2)], [(0, 3), (1, 0), (2, 0)], compute_logicals=True)
        return dict(hz=code.checks.z, hx=code.checks.x, lz=code.logicals.z, rounds=0, batch=1 << 18,
                    ps=[0.001, 0.003, 0.01], desc="[[144,12,12]] BB lift, R=0, BP ms max_iter 50 + SSF")
    if name == "c4":
        hx, hz = load_checks("hgp_80_3_4_s2025")
        _, lz = gf2.css_logicals(hx, hz)
        return dict(hz=hz, hx=hx, lz=lz, rounds=0, batch=1 << 17, max_shots=1 << 18, ps=[0.01, 0.03],
                    desc="biregular_hgp(80,3,4,seed=2025) n=10000, R=0, BP ms max_iter 50 + SSF")
    if name in ("c5", "c5r0"):
        from conftest import load_logicals
        hx, hz = load_checks("lp_pgl2_1_4_2_s1")
        _, lz = load_logicals("lp_pgl2_1_4_2_s1")
        if name == "c5":
            return dict(hz=hz, hx=None, lz=lz, rounds=1, batch=1 << 17, max_shots=1 << 18, ps=[0.001, 0.002, 0.005],
                        desc="PSL(2,16) Cayley LP n=53040 k=4080, R=1 spacetime (48960x130560), BP ms max_iter 50, "
                             "fold + logical check")
        return dict(hz=hz, hx=hx, lz=lz, rounds=0, batch=1 << 17, max_shots=1 << 18, ps=[0.001, 0.002, 0.005],
                    desc="PSL(2,16) Cayley LP n=53040 k=4080, R=0, BP ms max_iter 50 + SSF + logical check")
    if name == "c5m":
        from exp_ldpc_amd.lifted import psl2_lifted_product_code
        hz = psl2_lifted_product_code(13).checks.z
        return dict(hz=sp.csr_matrix(hz), hx=None, lz=None, rounds=1, batch=1 << 15, max_shots=1 << 15, ps=[0.002, 0.005],
                    desc="PSL(2,13) matrix lift n=49140, R=1 spacetime (39312x117936), BP ms max_iter 50")
    raise SystemExit(f"unknown config {name}")


def run(name, shots, ps_override, reps, batch=None, precision="f32"):
    import torch
    import scipy.sparse as sp
    from exp_ldpc_amd.decoder import Decoder
    from exp_ldpc_amd.spacetime import SpacetimeCode
    cfg = build_config(name)
    hz = sp.csr_matrix(cfg["hz"])
    m, n = hz.shape
    R = cfg["rounds"]
    H = sp.csr_matrix(SpacetimeCode(hz, R).spacetime_check_matrix) if R else hz
    shots = min(shots, cfg.get("max_shots", shots))
    B = min(batch or cfg["batch"], shots)
    nb = max(1, shots // B)
    dev = torch.device("cuda", 0)
    for p in (ps_override or cfg["ps"]):
        sampler = Decoder(hz, 2 * p / 3, method="ms", precision="f32", max_iter=50)
        dec = Decoder(H, 2 * p / 3, method="ms", precision=precision, max_iter=50, flip_sets=cfg["hx"],
                      logicals=cfg["lz"], n_data=n, fold_blocks=R + 1)
        syn = torch.empty((nb, B, H.shape[0]), dtype=torch.uint8, device=dev)
        rd = torch.empty((nb, B, n), dtype=torch.uint8, device=dev)
        for b in range(nb):
            sampler.sample_storage_device(R, p, p, SEED, 0, b * B, B, syn[b], rd[b])
        iters = torch.empty((nb, B), dtype=torch.int32, device=dev)
        status = torch.empty((nb, B), dtype=torch.uint8, device=dev)
        fail = torch.empty((nb, B), dtype=torch.uint8, device=dev)
        ssf = torch.empty((nb, B), dtype=torch.int32, device=dev)
        want_fail = cfg["lz"] is not None

        def one_pass():
            for b in range(nb):
                dec.decode_device(B, syn=syn[b], readout=rd[b] if want_fail else None, iters=iters[b],
                                  status=status[b], fail=fail[b] if want_fail else None, ssf_steps=ssf[b])
        one_pass()  # warmup
        torch.cuda.synchronize()
        dec.set_timing(nb * reps)
        t0 = time.perf_counter()
        for r in range(reps):
            one_pass()
            torch.cuda.synchronize()
            print(f"[{name} p={p}] pass {r + 1}/{reps} {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        bp_ms, ssf_ms = dec.read_timing()
        E = int(H.nnz)
        it_sum = float(iters.to(torch.int64).sum().item())
        io = H.shape[0] + n + 1
        tsz = 4 if precision == "f32" else 8
        bytes_per_pass = io * B * nb + 4 * tsz * E * it_sum  # 16 E (fp32) / 32 E (fp64) per shot-iteration
        kernel_s = bp_ms.sum() / 1e3 / reps
        total = nb * B * reps
        res = {
            "config": name, "desc": cfg["desc"], "precision": precision, "p": p, "shots": total, "shots_per_s": total / dt,
            "ms_per_pass": dt / reps * 1e3, "batch": B,
            "bp_converged_frac": float((status & 1).to(torch.float64).mean().item()),
            "mean_bp_iters": it_sum / (nb * B), "mean_ssf_steps": float(ssf.to(torch.float64).mean().item()),
            "ler": float(fail.to(torch.float64).mean().item()) if want_fail else None,
            "bp_kernel_ms_per_launch": float(bp_ms.mean()), "ssf_kernel_ms_per_launch": float(ssf_ms.mean()),
            "E": E, "algorithmic_GBps_bp_kernel": bytes_per_pass / kernel_s / 1e9,
            "group_kernel_env": os.environ.get("QDEC_GROUP_KERNEL", "default"),
            "lds_kernel_env": os.environ.get("QDEC_LDS_KERNEL", "default"),
        }
        print(json.dumps(res), flush=True)
        del syn, rd
        torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c3", "c4", "c5", "c5r0"])
    ap.add_argument("--shots", type=int, default=1 << 20, help="distinct shots per p (rounded to batches)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--p", type=float, action="append")
    ap.add_argument("--batch", type=int, default=None, help="shots per launch (default: per config)")
    ap.add_argument("--precision", nargs="+", choices=["f32", "f64"], default=["f32", "f64"])
    a = ap.parse_args()
    for c in a.configs:
        for prec in a.precision:
            run(c, a.shots, a.p, a.reps, a.batch, prec)


if __name__ == "__main__":
    main()
