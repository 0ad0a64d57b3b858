#!/bin/bash
# SQ PMC passes of the BP/SSF kernels at p = 0.1 (isolated), f32 and f64.
set -eo pipefail
export TMPDIR=/tmp
timeout -k 10 400 bash tools/dev/pmc_sq.sh gpurun_out/r02b/f32 --p 0.1 --steps 2 --warmup 1 --no-cpu-baseline --streams 1 --precision f32 > gpurun_out/r02b_f32.txt 2>&1
timeout -k 10 400 bash tools/dev/pmc_sq.sh gpurun_out/r02b/f64 --p 0.1 --steps 2 --warmup 1 --no-cpu-baseline --streams 1 --precision f64 > gpurun_out/r02b_f64.txt 2>&1
