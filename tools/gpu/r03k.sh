#!/bin/bash
# SQ counters of the f64 BP kernel at p = 0.1 (isolated, one stream): 8 vs 12 waves per CU.
set -eo pipefail
export TMPDIR=/tmp
for C in 8 12; do
  QDEC_F64_WAVES_PER_CU=$C bash tools/dev/pmc_sq.sh gpurun_out/r03k/cap$C --p 0.1 --steps 1 --warmup 1 --iso-steps 1 --no-cpu-baseline --no-sample-phase --variant none --streams 1 --no-large-code > gpurun_out/r03k_cap$C.txt 2>&1 || { tail -30 gpurun_out/r03k_cap$C.txt; exit 1; }
  echo "== cap $C"; cat gpurun_out/r03k_cap$C.txt
done
mkdir -p gpurun_out/r03k/fifo
timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE -d gpurun_out/r03k/fifo -o run --output-format csv -- python3 bench.py --p 0.1 --steps 1 --warmup 1 --iso-steps 1 --no-cpu-baseline --no-sample-phase --variant none --streams 1 --no-large-code > gpurun_out/r03k/fifo.log 2>&1 || tail -5 gpurun_out/r03k/fifo.log
