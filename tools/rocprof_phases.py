"""Split a rocprofv3 kernel trace of `bench.py` by kernel and phase, and compare
the roofline kernel's isolated-phase durations with the bench's own HIP-event
numbers.

Usage: python tools/rocprof_phases.py <run_kernel_trace.csv> <bench.json> [out.json]

Per sweep point and step bench.py launches, in the headline precision, a shot
triage (ms_triage_kernel), a BP kernel and an SSF kernel: W + K overlapped steps
(phase 1), the variant precision's W + K (phase 2, other instantiations), the
isolated steps (phase 3, one stream, headline then variant) and K sampling +
decode steps (phase 4, one stream); then the single-launch lines (config 5,
config 4, the reference default), whose kernels are other instantiations.  The
f64 overlapped phase runs the 3-waves-per-SIMD build of the BP kernel (its own
name, template argument OCC = 3), so the roofline kernel -- the default build,
named by the bench line's `roofline.kernel` -- has exactly the isolated
launches first, then the sampling phase's.  Without the OCC = 3 build in the
trace the first (W + K) * P launches of that name are the overlapped phase and
are skipped.  Every other kernel is summarised over all its dispatches.
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
    rf = b["roofline"]
    P = len(b["ler"]["p"]) if "p" in b["ler"] else len(b["ler"])  # the stdout line or its side file
    W, K = b["warmup"], b["steps"]
    iso = rf["launches"] // P
    by = defaultdict(list)
    with open(trace) as fh:
        for r in csv.DictReader(fh):
            k = r["Kernel_Name"].strip()
            k = k[5:] if k.startswith("void ") else k  # rocprof prefixes templated kernels with their return type
            by[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    res = {"trace": trace, "bench": bench, "points": P, "warmup": W, "steps": K, "iso_steps": iso, "kernels": {}}

    def summ(v):
        return {"dispatches": len(v), "avg_ms": sum(v) / len(v) if v else None, "sum_ms": sum(v)}

    roof = rf.get("kernel", "")
    def targs(name):
        head = name.split("(")[0]
        return head.split("<", 1)[0], [t.strip() for t in head.split("<", 1)[1].rstrip(">").split(",")] \
            if "<" in head else []

    # the 3-waves-per-SIMD build of the roofline kernel: template argument OCC (7th) = 3
    occ3 = False
    if roof:
        fam, ra = targs(roof)
        if len(ra) >= 7:
            cand = ra[:6] + ["3"] + ra[7:]
            occ3 = any(targs(k) == (fam, cand) for k in by)
    for name, d in sorted(by.items()):
        if "qdec::" not in name:
            continue
        d.sort()
        ms = [(e - s) * 1e-6 for s, e in d]
        entry = {"all": summ(ms)}
        if roof and name.split("(")[0] == roof:
            skip = 0 if occ3 else (W + K) * P
            entry["3_isolated"] = summ(ms[skip:skip + iso * P])
            entry["4_sample_decode"] = summ(ms[skip + iso * P:])
        res["kernels"][name] = entry
    for name, e in res["kernels"].items():
        if roof and name.split("(")[0] == roof and "3_isolated" in e:
            r = e["3_isolated"]["avg_ms"]
            res["compare"] = {"kernel": name, "bench_hip_event_avg_ms": rf["avg_launch_ms"], "rocprof_avg_ms": r,
                              "rocprof_all_dispatches_avg_ms": e["all"]["avg_ms"],
                              "rel_diff": (r - rf["avg_launch_ms"]) / rf["avg_launch_ms"] if r else None}
    txt = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(txt)
    print(json.dumps(res.get("compare"), indent=1))


if __name__ == "__main__":
    main()
