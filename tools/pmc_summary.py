"""Summarise rocprofv3 PMC passes (tools/pmc.sh output) per kernel.

Usage: python tools/pmc_summary.py <pmc_dir> <out.json>

For every kernel: dispatch count, mean of each counter per dispatch.  HBM bytes
follow MI355X_MICROARCH.md § HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE is doubled on gfx950 (it tallies 128-B read requests at 64 B);
WRITE_SIZE is taken as is.  Our loads are not all 16-B-per-lane streaming
reads, for which the guide calibrated the factor, so the byte figure is an
estimate; ratios between kernel variants are exact.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short_name(k: str) -> str:
    k = k.strip()
    if k.startswith("void "):
        k = k[5:]
    return k


def family(k: str) -> str:
    return k.split("<")[0].split("(")[0].strip().split("::")[-1]


def main():
    src, out = sys.argv[1], sys.argv[2]
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for f in sorted(glob.glob(os.path.join(src, "pass*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short_name(row["Kernel_Name"])
                c = row["Counter_Name"]
                acc[k][c] += float(row["Counter_Value"])
                cnt[k][c] += 1
    kernels = {}
    for k in acc:
        means = {c: acc[k][c] / cnt[k][c] for c in acc[k]}
        d = {"dispatches": max(cnt[k].values()), "counters_per_dispatch": means}
        if "FETCH_SIZE" in means or "WRITE_SIZE" in means:
            rd = 2 * 1024 * means.get("FETCH_SIZE", 0.0)
            wr = 1024 * means.get("WRITE_SIZE", 0.0)
            d["hbm_read_bytes_per_dispatch"] = rd
            d["hbm_write_bytes_per_dispatch"] = wr
            d["hbm_bytes_per_dispatch"] = rd + wr
        kernels[k] = d
    bp = [k for k in kernels if family(k) in ("bp_wave_kernel", "bp_ms_wave_kernel", "bp_block_kernel")]
    ssf = [k for k in kernels if family(k) in ("ssf_wave_kernel", "ssf_block_kernel")]

    def pick(names):
        if not names:
            return None
        k = max(names, key=lambda k: kernels[k]["dispatches"])
        return k, kernels[k].get("hbm_bytes_per_dispatch")

    res = {
        "source": src,
        "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024 (MI355X_MICROARCH.md HBM)",
        "kernels": kernels,
    }
    if pick(bp):
        res["decode_kernel"], res["decode_kernel_hbm_bytes_per_launch"] = pick(bp)
    if pick(ssf):
        res["ssf_kernel"], res["ssf_kernel_hbm_bytes_per_launch"] = pick(ssf)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
