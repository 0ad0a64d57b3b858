#!/bin/bash
# tools/pmc.sh's counter passes over any python command (diagnostics):
#   tools/pmc_cmd.sh <outdir> <script.py> [args...]
# Each pass is its own rocprofv3 run, --kernel-trace only, killed after 240 s.
set -eo pipefail
OUT=$1; shift
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
            ${PMC_HBM:+"FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"}; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $CTRS -d "$R/$OUT/pass$i" -o run --output-format csv -- python3 "$@" > "$R/$OUT/pass$i.log" 2>&1
  echo "pass $i done"
done
python3 tools/pmc_summary.py "$R/$OUT" "$R/$OUT/summary.json" ${PMC_META:-}
