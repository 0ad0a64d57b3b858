#!/bin/bash
# Round 5, session g: config-4 line after the by-qubit logical test (lz_t), and the
# large-code parity tests.
set -eo pipefail
O=gpurun_out/${1:-r05g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_codes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python -u tools/gpu/c4_only.py $O/c4.json > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
cat $O/c4.log
