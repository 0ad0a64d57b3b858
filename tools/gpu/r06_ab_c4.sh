#!/bin/bash
# A/B of the C4 f64 kernel: default library vs a variant (QDEC_LIB), interleaved.
set -eo pipefail
O=gpurun_out/${1:-r06h}; V=${2:-colreads}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u tools/gpu/c4_only.py --prec f64 > $O/base_$r.log 2>&1
  QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_$V.so timeout -k 10 300 python -u tools/gpu/c4_only.py --prec f64 > $O/${V}_$r.log 2>&1
  echo "base $r"; cat $O/base_$r.log | grep f64; echo "$V $r"; cat $O/${V}_$r.log | grep f64
done
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_$V.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_large_codes.py -k "lds64 or hgp10k_f64" > $O/tests_$V.log 2>&1 || { tail -20 $O/tests_$V.log; exit 1; }
tail -1 $O/tests_$V.log
