#!/bin/bash
# PMC passes (tools/pmc.sh) of the bench kernels at p = 0.1 only, f64 headline + f32 variant.
# Usage: tools/gpu_pmc_p01.sh <tag>
set -eo pipefail
TAG=${1:-pmc}
export TMPDIR=/tmp
timeout -k 10 900 bash tools/pmc.sh gpurun_out/$TAG --p 0.1 --steps 2 --warmup 1 --iso-steps 1 --no-cpu-baseline --no-sample-phase --streams 1 > gpurun_out/$TAG.txt 2>&1
cat gpurun_out/$TAG.txt
