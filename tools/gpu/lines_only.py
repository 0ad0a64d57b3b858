"""Run bench.py's extra config lines alone (diagnostics and PMC passes of one
launch shape).

Usage: python tools/gpu/lines_only.py [--c3] [--c5] [--c5-p P ...] [--c3-p P ...]
       [--shots N] [--out file.json]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--c3", action="store_true")
ap.add_argument("--c5", action="store_true")
ap.add_argument("--c3-p", type=float, action="append")
ap.add_argument("--c5-p", type=float, action="append")
ap.add_argument("--shots", type=int, default=0, help="shots per launch (0: the bench's)")
ap.add_argument("--c5-warm-full", action="store_true", help="warmup launch as large as the timed one (PMC)")
ap.add_argument("--out")
args = ap.parse_args()
dev = torch.device("cuda", 0)
res = {}
if args.c3:
    kw = {"shots": args.shots} if args.shots else {}
    res["c3"] = bench.c3_line(dev, ps=tuple(args.c3_p or (0.001, 0.003, 0.01)), **kw)
    for ln in res["c3"]["lines"]:
        print("c3", ln["p"], f"{ln['shots_per_s']:.4g} shots/s", f"triage {ln['triage_ms']:.3f} bp {ln['bp_kernel_ms']:.3f} "
              f"ssf {ln['ssf_kernel_ms']:.3f} ms", f"frac {ln['roofline']['frac']:.3f}", f"ler {ln['ler']:.3g}")
if args.c5:
    kw = {"shots": args.shots, "low_p_shots": args.shots} if args.shots else {}
    if args.c5_warm_full:  # the warmup launch as large as the timed one (one launch shape per PMC pass)
        kw["warm_shots"] = 1 << 30
    res["c5"] = bench.large_code_roofline(dev, ps=tuple(args.c5_p or (0.0005, 0.001, 0.005)), **kw)
    for ln in res["c5"]["lines"]:
        print("c5", ln["p"], f"{ln['shots_per_s']:.4g} shots/s", f"bp {ln['bp_kernel_ms']:.1f} ms",
              f"iters {ln['mean_bp_iters']:.2f}", f"frac {ln['roofline']['frac']:.3f}", f"ler {ln['ler']:.3g}")
if args.out:
    open(args.out, "w").write(json.dumps(res))
