#!/bin/bash
# Round 5, session y: full GPU suite with bp_ms_lds64_kernel as the automatic
# f64 kernel of config 4, then the C4 line alone (both precisions).
set -eo pipefail
O=gpurun_out/${1:-r05y}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 400 python tools/gpu/c4_only.py $O/c4.json > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
grep -v amdgpu.ids $O/c4.log
