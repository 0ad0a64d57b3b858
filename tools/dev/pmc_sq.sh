#!/bin/bash
# SQ counter passes only (no TCC) for kernel tuning. Usage: tools/dev/pmc_sq.sh <outdir> <bench args...>
set -e
OUT=$1; shift
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
            "SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $CTRS -d "$R/$OUT/pass$i" -o run --output-format csv -- python3 bench.py "$@" > "$R/$OUT/pass$i.log" 2>&1
done
python3 tools/pmc_summary.py "$R/$OUT" "$R/$OUT/summary.json" > /dev/null
python3 - "$R/$OUT/summary.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    if "qdec" in k and ("bp_" in k or "ssf" in k):
        print(k[:90], v["dispatches"])
        for c, x in sorted(v["counters_per_dispatch"].items()):
            print("   %-24s %.4g" % (c, x))
PY
