#!/bin/bash
# Round 4, session f: PMC passes (tools/pmc.sh) of the compact path and of the
# one-pass kernel, same bench shape (isolated + overlapped phases, f64 only).
set -eo pipefail
O=gpurun_out/r04f
mkdir -p $O
export TMPDIR=/tmp
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none --steps 2 --warmup 1"
timeout -k 10 900 bash tools/pmc.sh $O/pmc_cmp $A > $O/pmc_cmp.log 2>&1 || { tail -20 $O/pmc_cmp.log; exit 1; }
QDEC_COMPACT=0 timeout -k 10 900 bash tools/pmc.sh $O/pmc_one $A > $O/pmc_one.log 2>&1 || { tail -20 $O/pmc_one.log; exit 1; }
echo done
