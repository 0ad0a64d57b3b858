#!/bin/bash
# Round 5, session z: bp_ms_lds64_kernel A/B (a = committed, b = working tree),
# C4 f64 line, interleaved; then the lds64 parity tests on b.
set -eo pipefail
O=gpurun_out/${1:-r05z}
mkdir -p $O
L=$PWD/exp_ldpc_amd
for r in 1 2; do
  for v in a b; do
    lib=$L/libqdec_hip.so; [ $v = a ] && lib=$L/libqdec_hip_a.so
    QDEC_LIB=$lib timeout -k 10 300 python tools/gpu/c4_only.py $O/c4_${v}_$r.json --prec f64 --p 0.005 --p 0.03 > $O/c4_${v}_$r.log 2>&1 || { tail -20 $O/c4_${v}_$r.log; exit 1; }
    echo "$v $r"; grep -v amdgpu.ids $O/c4_${v}_$r.log
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_large_codes.py -k "lds64 or f64" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
