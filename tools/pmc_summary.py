"""Summarise rocprofv3 PMC passes (tools/pmc.sh output) per kernel.

Usage: python tools/pmc_summary.py <pmc_dir> <out.json> [key=value ...]
(key=value pairs go to the summary's "meta", e.g. c5_p=0.005: bench.py matches
a summary to the launch it describes by them)

Per kernel: dispatch count, the mean of every counter per dispatch, and derived
ceilings computed from counter sums over the kernel's dispatches, each against
the GRBM_GUI_ACTIVE of the same pass (every pass collects it):

  cycles        = GRBM_GUI_ACTIVE / 8             (summed over the 8 XCDs)
  clock_ghz     = cycles / dispatch time           (timestamps of the same pass)
  valu_issue_frac = SQ_INSTS_VALU * 2 / (256 CU * 4 SIMD * cycles)
                  (a wave64 VALU op issues over 2 cycles on a SIMD-32; f64 and
                  transcendental ops take longer, so for f64 kernels this is a
                  lower bound on VALU busy time)
  lds_frac      = SQ_LDS_IDX_ACTIVE / (256 CU * cycles)   (LDS-array cycles)
  lds_bank_conflict_ratio = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  hbm_bytes_per_dispatch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> B); FETCH_SIZE
                  doubled per MI355X_MICROARCH.md § HBM (gfx950 tallies 128-B
                  read requests at 64 B; calibrated for wide streaming loads,
                  so an estimate for other access shapes)
  hbm_frac      = hbm bytes / dispatch time / 8 TB/s
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

CUS, SIMDS, HBM_PEAK = 256, 4, 8.0e12


def short_name(k: str) -> str:
    k = k.strip()
    return k[5:] if k.startswith("void ") else k


def family(k: str) -> str:
    return k.split("<")[0].split("(")[0].strip().split("::")[-1]


def main():
    src, out = sys.argv[1], sys.argv[2]
    # per kernel, per pass: counter sums, GRBM sums, durations per dispatch
    csum = defaultdict(lambda: defaultdict(float))      # kernel -> counter -> sum over dispatches
    ccnt = defaultdict(lambda: defaultdict(int))
    pass_of = defaultdict(dict)                          # kernel -> counter -> pass dir
    grbm = defaultdict(lambda: defaultdict(float))      # kernel -> pass -> sum GRBM
    dur = defaultdict(lambda: defaultdict(dict))        # kernel -> pass -> dispatch -> ns
    for f in sorted(glob.glob(os.path.join(src, "pass*", "**", "*counter_collection.csv"), recursive=True)):
        pdir = os.path.relpath(f, src).split(os.sep)[0]
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short_name(row["Kernel_Name"])
                c = row["Counter_Name"]
                v = float(row["Counter_Value"])
                d = int(row["Dispatch_Id"])
                dur[k][pdir][d] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                if c == "GRBM_GUI_ACTIVE":
                    grbm[k][pdir] += v
                    continue
                csum[k][c] += v
                ccnt[k][c] += 1
                pass_of[k][c] = pdir
    kernels = {}
    for k in set(csum) | set(grbm):
        means = {c: csum[k][c] / ccnt[k][c] for c in csum[k]}
        ndisp = max([len(v) for v in dur[k].values()] + [0])
        d = {"dispatches": ndisp, "counters_per_dispatch": means}

        def cycles(c):
            p = pass_of[k].get(c)
            return grbm[k].get(p, 0.0) / 8.0 if p else 0.0

        def secs(c):
            p = pass_of[k].get(c)
            return sum(dur[k][p].values()) * 1e-9 if p else 0.0

        dv = {"formulas": "valu_issue_frac = SQ_INSTS_VALU*2/(256*4*GRBM_GUI_ACTIVE/8); "
                          "lds_frac = SQ_LDS_IDX_ACTIVE/(256*GRBM_GUI_ACTIVE/8); "
                          "lds_bank_conflict_ratio = SQ_LDS_BANK_CONFLICT/SQ_LDS_IDX_ACTIVE; "
                          "hbm bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024; clock = GRBM_GUI_ACTIVE/8/time"}
        anyp = next(iter(dur[k].values()), {})
        if anyp:
            dv["duration_ms"] = sum(anyp.values()) / len(anyp) * 1e-6
        if "SQ_INSTS_VALU" in csum[k] and cycles("SQ_INSTS_VALU") > 0:
            cyc = cycles("SQ_INSTS_VALU")
            dv["valu_issue_frac"] = csum[k]["SQ_INSTS_VALU"] * 2 / (CUS * SIMDS * cyc)
            dv["clock_ghz"] = cyc / secs("SQ_INSTS_VALU") / 1e9 if secs("SQ_INSTS_VALU") > 0 else None
        if "SQ_LDS_IDX_ACTIVE" in csum[k] and cycles("SQ_LDS_IDX_ACTIVE") > 0:
            dv["lds_frac"] = csum[k]["SQ_LDS_IDX_ACTIVE"] / (CUS * cycles("SQ_LDS_IDX_ACTIVE"))
            if "SQ_LDS_BANK_CONFLICT" in csum[k] and csum[k]["SQ_LDS_IDX_ACTIVE"] > 0:
                dv["lds_bank_conflict_ratio"] = csum[k]["SQ_LDS_BANK_CONFLICT"] / csum[k]["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in means or "WRITE_SIZE" in means:
            rd = 2 * 1024 * means.get("FETCH_SIZE", 0.0)
            wr = 1024 * means.get("WRITE_SIZE", 0.0)
            dv["hbm_read_bytes_per_dispatch"] = rd
            dv["hbm_write_bytes_per_dispatch"] = wr
            dv["hbm_bytes_per_dispatch"] = rd + wr
            t_rd = secs("FETCH_SIZE") / max(1, ccnt[k].get("FETCH_SIZE", 1))
            t_wr = secs("WRITE_SIZE") / max(1, ccnt[k].get("WRITE_SIZE", 1))
            if t_rd > 0 and t_wr > 0:
                dv["hbm_frac"] = (rd / t_rd + wr / t_wr) / HBM_PEAK
        d["derived"] = dv
        kernels[k] = d
    res = {"source": src, "kernels": kernels}
    meta = {}
    for kv in sys.argv[3:]:
        key, _, val = kv.partition("=")
        try:
            meta[key] = float(val)
        except ValueError:
            meta[key] = val
    if meta:
        res["meta"] = meta
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, v in sorted(kernels.items()):
        if family(k) in ("bp_ms_wave_kernel", "bp_wave_kernel", "bp_block_kernel", "ssf_wave_kernel",
                         "ssf_block_kernel", "bp_group_kernel", "bp_ms_lds_kernel", "bp_ms_lds64_kernel", "ssf_inc_block_kernel"):
            print(k[:100], v["dispatches"], {a: (round(b, 4) if isinstance(b, float) else None)
                                               for a, b in v["derived"].items() if a != "formulas"})


if __name__ == "__main__":
    main()
