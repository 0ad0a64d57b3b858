#!/bin/bash
# A/B of the C4 f64 kernel: default library vs variants (QDEC_LIB), interleaved,
# then each variant's LDS-kernel parity tests.  Usage: r06_ab_c4v.sh TAG V1 [V2 ...]
set -eo pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u tools/gpu/c4_only.py --prec ${PREC:-f64} > $O/base_$r.log 2>&1
  echo "base $r"; grep ${PREC:-f64} $O/base_$r.log
  for V in "$@"; do
    QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_$V.so timeout -k 10 300 python -u tools/gpu/c4_only.py --prec ${PREC:-f64} > $O/${V}_$r.log 2>&1
    echo "$V $r"; grep ${PREC:-f64} $O/${V}_$r.log
  done
done
for V in "$@"; do
  QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_$V.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_large_codes.py -k "${TESTK:-lds64 or hgp10k_f64}" > $O/tests_$V.log 2>&1 || { tail -20 $O/tests_$V.log; exit 1; }
  echo "tests $V"; tail -1 $O/tests_$V.log
done
