#!/bin/bash
# Round 5, session m: C4 LDS kernel check pass by sign bits (+ row swizzle by
# bit 4) -- large-code parity, C4 f32 line; the hypergraph-product kernel's
# parity and BP-only timing.
set -eo pipefail
O=gpurun_out/${1:-r05m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_codes.py tests/test_gpu_hgp.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python -u tools/gpu/c4_only.py $O/c4.json --prec f32 > $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
cat $O/c4.log
timeout -k 10 300 python -u tools/gpu/hgp_time.py 0 > $O/hgp_time.log 2>&1 || { tail -20 $O/hgp_time.log; exit 1; }
cp gpurun_out/hgp_time.json $O/
cat $O/hgp_time.log
