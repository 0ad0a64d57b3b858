#!/bin/bash
# Unrolled product-sum workgroup path: parity, then bposd at R = 2 / 3 (workgroup
# kernel, ps) with the previous library vs the current one.
set -eo pipefail
O=gpurun_out/ps; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py tests/test_gpu_large_codes.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
QDEC_LIB=$PWD/exp_ldpc_amd/_ab/libqdec_hip_prev.so timeout -k 10 300 python -u tools/bench_modes.py --modes bposd:2,bposd:3 --p 0.003 --p 0.01 > $O/prev.jsonl 2> $O/prev.err
timeout -k 10 300 python -u tools/bench_modes.py --modes bposd:2,bposd:3 --p 0.003 --p 0.01 > $O/new.jsonl 2> $O/new.err
cut -c1-200 $O/prev.jsonl $O/new.jsonl
