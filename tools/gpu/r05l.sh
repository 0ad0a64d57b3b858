#!/bin/bash
# Round 5, session l: hypergraph-product kernel after the sign-op rewrite --
# parity, BP-only timing against the generic lean f64 path.
set -eo pipefail
O=gpurun_out/${1:-r05l}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_hgp.py -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u tools/gpu/hgp_time.py 0 10 > $O/hgp_time.log 2>&1 || { tail -20 $O/hgp_time.log; exit 1; }
cp gpurun_out/hgp_time.json $O/
cat $O/hgp_time.log
