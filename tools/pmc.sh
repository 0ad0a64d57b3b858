#!/bin/bash
# PMC passes for the bench kernels (run on the GPU box from the repo root).
# Each pass is its own rocprofv3 run with --kernel-trace only (no sys/runtime
# trace domains) and every pass also collects GRBM_GUI_ACTIVE, so each counter
# has the cycle count of its own pass.  Usage: tools/pmc.sh <outdir> <bench args...>
set -eo pipefail
OUT=$1; shift
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
            "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $CTRS -d "$R/$OUT/pass$i" -o run --output-format csv -- python3 bench.py "$@" > "$R/$OUT/pass$i.log" 2>&1
  echo "pass $i done"
done
python3 tools/pmc_summary.py "$R/$OUT" "$R/$OUT/summary.json" ${PMC_META:-}
