#!/bin/bash
# Full GPU test suite + smoke (what the driver runs at round end).
set -eo pipefail
O=gpurun_out/full; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -2 $O/smoke.log
