#!/bin/bash
# Round 5, session h: A/B of the LDS-resident min-sum kernel's variable pass
# (A: libqdec_hip_a.so, one variable's reads in flight; B: the tree's library,
# software-pipelined by one variable), config-4 line each, then the large-code
# parity tests on B.
set -eo pipefail
O=gpurun_out/${1:-r05h}
mkdir -p $O
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_a.so timeout -k 10 400 python -u tools/gpu/c4_only.py $O/c4_a.json > $O/c4_a.log 2>&1 || { tail -20 $O/c4_a.log; exit 1; }
timeout -k 10 400 python -u tools/gpu/c4_only.py $O/c4_b.json > $O/c4_b.log 2>&1 || { tail -20 $O/c4_b.log; exit 1; }
grep -h f32 $O/c4_a.log $O/c4_b.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_codes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
