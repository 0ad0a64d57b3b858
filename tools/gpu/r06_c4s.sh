#!/bin/bash
# C4 f64 kernel round: LDS-kernel parity tests, the config-4 line, phase stamps.
set -eo pipefail
TAG=${1:-r06s}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_large_codes.py -k "lds64 or hgp10k_f64 or hgp10k_bp_f64" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python -u tools/gpu/c4_only.py $O/c4.json --prec f64 > $O/c4.log 2> $O/c4.err
cat $O/c4.log
if [ -f exp_ldpc_amd/libqdec_hip_stamps.so ]; then
  timeout -k 10 300 python -u tools/dev/stamps_c4.py 0.005 0.03 > $O/stamps.log 2>&1
  grep "p=" $O/stamps.log
fi
