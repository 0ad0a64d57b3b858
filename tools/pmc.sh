#!/bin/bash
# PMC passes for the decode kernel (run on the GPU box from the repo root).
# Each pass is its own rocprofv3 run with --kernel-trace only (no sys/runtime
# trace domains).  Usage: tools/pmc.sh <outdir> <bench args...>
set -e
OUT=$1; shift
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $CTRS -d "$R/$OUT/pass$i" -o run --output-format csv -- python3 bench.py "$@" > "$R/$OUT/pass$i.log" 2>&1
done
