#!/bin/bash
# PMC passes on the C4 config (LDS-resident BP kernel + SSF block kernel), p = 0.03.
set -eo pipefail
OUT=gpurun_out/pmc_${CFG:-c4}
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d "$R/$OUT/pass$i" -o run --output-format csv -- python3 tools/bench_configs.py ${CFG:-c4} --p ${P:-0.03} --shots ${SHOTS:-131072} --reps 1 > "$R/$OUT/pass$i.log" 2>&1
  echo "pass $i done"
done
python3 tools/pmc_summary.py "$R/$OUT" "$R/$OUT/summary.json"
