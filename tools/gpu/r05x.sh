#!/bin/bash
# Round 5, session x: bp_ms_lds64_kernel (f64 LDS-resident C4 kernel): parity,
# then C4 f64 timing against the slot-group kernel.
set -eo pipefail
O=gpurun_out/${1:-r05x}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_large_codes.py \
  -k "lds64" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
timeout -k 10 300 python tools/gpu/c4_only.py $O/c4_lds64.json --prec f64 --p 0.005 --p 0.01 --p 0.03 --lds-kernel 1 > $O/c4_lds64.log 2>&1 || { tail -20 $O/c4_lds64.log; exit 1; }
cat $O/c4_lds64.log | grep -v amdgpu.ids
timeout -k 10 300 python tools/gpu/c4_only.py $O/c4_group.json --prec f64 --p 0.005 --p 0.01 --p 0.03 > $O/c4_group.log 2>&1 || { tail -20 $O/c4_group.log; exit 1; }
cat $O/c4_group.log | grep -v amdgpu.ids
