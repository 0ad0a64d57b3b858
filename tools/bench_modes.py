"""Throughput of the batched decoder modes (the p_sweep harness path,
exp_ldpc_amd.experiment.BatchPipeline) on one MI355X, device OSD vs the host OSD
stage.  Diagnostic companion of bench.py (which measures BASELINE config 2).

Default workload = the reference script's defaults (scripts/p_sweep.py,
misc/p_sweep.py:57-78, _experiment.py:213-229): R = 1, decoder_mode bposd,
bp_method ps, max_iter = n = 225, osd_cs order 7, priors 2p/3, on the n = 225 code.

Usage: python tools/bench_modes.py [--shots N] [--p P ...] [--modes bposd,...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch
    from conftest import load_code
    from exp_ldpc_amd.decoder import Decoder
    from exp_ldpc_amd.experiment import BatchPipeline
    from exp_ldpc_amd.noise_model import depolarizing_noise
    from exp_ldpc_amd.storage_sim import build_storage_simulation
    ap = argparse.ArgumentParser()
    ap.add_argument("--shots", type=int, default=1 << 18)
    ap.add_argument("--batch", type=int, default=1 << 16)
    ap.add_argument("--p", type=float, action="append")
    ap.add_argument("--modes", default="bposd:1,bposd_hybrid:1,bposd_single_shot:1,bpssf:0")
    ap.add_argument("--bp_method", default="ps")
    ap.add_argument("--max_iter", type=int, default=225)
    ap.add_argument("--host-osd", action="store_true", help="also time the host OSD stage")
    ap.add_argument("--precision", default="f64", choices=["f32", "f64"],
                    help="BP message precision (default f64, as ldpc v1 and the harness default)")
    a = ap.parse_args()
    code = load_code("hgp_12_3_4_s1234")
    ps = a.p or [0.003, 0.01, 0.03]
    opts = {"max_iter": a.max_iter, "bp_method": a.bp_method, "ms_scaling_factor": 0, "osd_method": "osd_cs",
            "osd_order": 7}
    for spec in a.modes.split(","):
        mode, rounds = spec.split(":")
        rounds = int(rounds)
        for p in ps:
            noise = depolarizing_noise(p, p)
            sim = build_storage_simulation(rounds, noise, code)
            pipe = BatchPipeline(code, rounds, mode, opts, (2 * p / 3, 2 * p / 3), noise=noise,
                                 precision=a.precision)
            batches = [sim.sample_device(pipe.sampler_graph, a.batch, 20250221, 0, s) for s in
                       range(0, a.shots, a.batch)]
            variants = [("device_osd", None)]
            if a.host_osd and mode.startswith("bposd"):
                variants.append(("host_osd", property(lambda self: False)))
            for vname, patch in variants:
                orig = Decoder.osd_device_supported
                if patch is not None:
                    Decoder.osd_device_supported = patch
                try:
                    pipe.run(*batches[0])  # warmup
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    fails = conv = 0
                    for syn, rd in batches:
                        r = pipe.run(syn, rd)
                        fails += int(r.fail.sum())
                        conv += r.bp_converged
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                finally:
                    Decoder.osd_device_supported = orig
                n = a.batch * len(batches)
                print(json.dumps({"mode": mode, "rounds": rounds, "p": p, "variant": vname, "bp_method": a.bp_method,
                                  "precision": a.precision,
                                  "max_iter": a.max_iter, "shots": n, "shots_per_s": n / dt, "ler": fails / n,
                                  "bp_converged_frac": conv / n}), flush=True)


if __name__ == "__main__":
    main()
