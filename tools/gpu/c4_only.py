"""Run bench.py's config-4 line alone (diagnostics).

Usage: python tools/gpu/c4_only.py [out.json] [--prec f32] [--p 0.03 ...] [--shots N] [--lds-kernel 1]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out", nargs="?")
ap.add_argument("--prec", action="append")
ap.add_argument("--p", type=float, action="append")
ap.add_argument("--shots", type=int, default=1 << 19)
ap.add_argument("--lds-kernel", type=int, default=None, help="QD_OPT_LDS_KERNEL for every handle")
args = ap.parse_args()
if args.lds_kernel is not None:
    from exp_ldpc_amd import decoder
    decoder.DEFAULT_OPTIONS["lds_kernel"] = args.lds_kernel
r = bench.c4_line(torch.device("cuda", 0), shots=args.shots, ps=tuple(args.p or (0.005, 0.01, 0.03)),
                  precisions=tuple(args.prec or ("f64", "f32")))
if args.out:
    open(args.out, "w").write(json.dumps(r))
for ln in r["lines"]:
    print(ln["precision"], ln["p"], f"{ln['shots_per_s']:.0f} shots/s", f"bp {ln['bp_kernel_ms']:.2f} ms",
          f"ssf {ln['ssf_kernel_ms']:.2f} ms", f"frac {ln['roofline']['frac']:.3f}", ln["bp_kernel"][:40], ln["ssf_kernel"][:40])
