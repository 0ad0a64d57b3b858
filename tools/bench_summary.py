"""One-line summary of a bench.py JSON line (headline, variant, per-point
isolated kernel times, roofline) for GPU-session logs."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"]
var = d.get("variants") or [{}]
print(f"n_gpus {d['n_gpus']}  {d['dtype']} {d['value'] / 1e6:.2f} M/s  ms/step {d['ms_per_step']:.2f}"
      + (f"  {var[0].get('dtype')} {var[0]['value'] / 1e6:.2f} M/s" if var[0] else ""))
print(f"  kernel {r.get('kernel')}  pre {r.get('pre_kernel', '')}  ssf {r.get('ssf_kernel')}")
print(f"  lds frac {r['frac']:.3f}  hbm frac {r['hbm']['frac']:.4f}  iso step {r['isolated_step_ms']:.2f} ms  "
      f"ceilings {r.get('ceilings', {}).get('kernel')}")
print("  bp ", [round(x["bp_kernel_ms_isolated"], 3) for x in d["ler"].values()])
print("  ssf", [round(x["ssf_kernel_ms_isolated"], 3) for x in d["ler"].values()])
if "sample_and_decode" in d:
    print(f"  sample+decode {d['sample_and_decode']['value'] / 1e6:.2f} M/s")
if "large_code_roofline" in d:
    lc = d["large_code_roofline"]
    print(f"  C5 {lc['shots_per_s'] / 1e3:.1f} k/s  {lc['roofline']['achieved'] / 1e3:.2f} TB/s")
if "cpu_baseline" in d:
    print(f"  cpu {d['cpu_baseline']['value'] / 1e6:.3f} M/s on {d['cpu_baseline']['cores']} threads")
if "ler_overlap_all" in d:
    print("  overlap", d["ler_overlap_all"])
