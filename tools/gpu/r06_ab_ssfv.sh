#!/bin/bash
# A/B of a variant library (QDEC_LIB) on both C4 lines, interleaved, then its
# large-code GPU tests.  Usage: r06_ab_ssfv.sh TAG VARIANT
set -eo pipefail
O=gpurun_out/$1; V=$2
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u tools/gpu/c4_only.py > $O/base_$r.log 2>&1
  echo "base $r"; grep "^f" $O/base_$r.log
  QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_$V.so timeout -k 10 300 python -u tools/gpu/c4_only.py > $O/${V}_$r.log 2>&1
  echo "$V $r"; grep "^f" $O/${V}_$r.log
done
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_$V.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_large_codes.py > $O/tests_$V.log 2>&1 || { tail -20 $O/tests_$V.log; exit 1; }
echo "tests $V"; tail -1 $O/tests_$V.log
