"""Split a rocprofv3 kernel trace of `bench.py` into the bench's phases and
compare the isolated-phase kernel durations with the bench's own HIP-event
numbers.

Usage: python tools/rocprof_phases.py <run_kernel_trace.csv> <bench.json> [out.json]

bench.py launches, per sweep point and step, one BP kernel and one SSF kernel
of the headline precision in this order: warmup steps + timed steps (phase 1,
overlapped streams), isolated steps (phase 3, one stream), sampling + decode
steps (phase 4, one stream); the variant precision's kernels are a different
template instantiation: warmup + timed (phase 2), isolated (phase 3).  Dispatches
of one kernel name, sorted by start time, therefore split by count.  When the
overlapped phase runs the 3-waves-per-SIMD build (a distinct instantiation,
OCC = 3), that name is phase 1 and the default build holds phases 3 and 4.
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    b = json.load(open(bench))
    P = len(b["ler"])
    W, K = b["warmup"], b["steps"]
    iso = b["roofline"]["launches"] // P
    by = defaultdict(list)
    with open(trace) as fh:
        for r in csv.DictReader(fh):
            by[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    res = {"trace": trace, "bench": bench, "points": P, "warmup": W, "steps": K, "iso_steps": iso, "kernels": {}}
    head = "double" if b["dtype"] == "f64" else "float"
    for name, d in sorted(by.items()):
        if "qdec::" not in name:
            continue
        d.sort()
        ms = [(e - s) * 1e-6 for s, e in d]
        if "bp_ms_wave_kernel" in name or "ssf_wave_kernel" in name:
            headline = ("bp_ms_wave_kernel<" + head) in name
            ssf = "ssf_wave_kernel" in name
            # ssf kernels of both precisions share one name: headline phases first
            n1 = (W + K) * P
            phases = {}
            occ3 = headline and name.split(">(")[0].endswith(", 3")
            if occ3:  # the 3-waves-per-SIMD build runs only in the overlapped phase (12 waves per CU)
                phases["1_overlapped"] = ms
            elif headline and any(k != name and ("bp_ms_wave_kernel<" + head) in k and k.split(">(")[0].endswith(", 3")
                                  for k in by):  # its default build: isolated + sampling phases only
                phases["3_isolated"] = ms[:iso * P]
                phases["4_sample_decode"] = ms[iso * P:]
            elif headline or ssf:
                phases["1_overlapped"] = ms[:n1]
                phases["3_isolated"] = ms[n1:n1 + iso * P]
                rest = ms[n1 + iso * P:]
                if ssf and "variants" in b:  # variant phase 2 + its isolated phase follow... in launch order
                    # launch order: p1 (W+K)P, p2 (W+K)P, p3 head isoP, p3 var isoP, p4 K*P
                    phases = {"1_overlapped": ms[:n1], "2_variant_overlapped": ms[n1:2 * n1],
                              "3_isolated_headline": ms[2 * n1:2 * n1 + iso * P],
                              "3_isolated_variant": ms[2 * n1 + iso * P:2 * n1 + 2 * iso * P],
                              "4_sample_decode": ms[2 * n1 + 2 * iso * P:]}
                elif headline:
                    phases["4_sample_decode"] = rest
            else:
                phases["2_overlapped"] = ms[:n1]
                phases["3_isolated"] = ms[n1:n1 + iso * P]
            res["kernels"][name] = {k: {"dispatches": len(v), "avg_ms": sum(v) / len(v) if v else None,
                                        "sum_ms": sum(v)} for k, v in phases.items()}
        else:
            res["kernels"][name] = {"all": {"dispatches": len(ms), "avg_ms": sum(ms) / len(ms), "sum_ms": sum(ms)}}
    rf = b["roofline"]
    for name, ph in res["kernels"].items():
        if ("bp_ms_wave_kernel<" + head) in name and "3_isolated" in ph:
            r = ph["3_isolated"]["avg_ms"]
            res["compare"] = {"kernel": name, "bench_hip_event_avg_ms": rf["avg_launch_ms"], "rocprof_avg_ms": r,
                              "rel_diff": (r - rf["avg_launch_ms"]) / rf["avg_launch_ms"]}
    txt = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(txt)
    print(json.dumps(res.get("compare"), indent=1))


if __name__ == "__main__":
    main()
