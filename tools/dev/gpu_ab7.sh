#!/bin/bash
# Session-2 A/B batch: suite + benches (default, 8-wave SSF workgroups,
# deferred per-shot stores), LEAN parity on the deferred-store build, then the
# overlapped-phase occupancy A/B.
set -eo pipefail
bash tools/dev/gpu_ab3.sh ab7 w8o6 ds1
O=gpurun_out/ab7
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_ds1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lean or zero or occupancy or bp_ssf_parity" > $O/t_ds1.log 2>&1 || { tail -30 $O/t_ds1.log; exit 1; }
echo "ds1 parity: $(tail -1 $O/t_ds1.log)"
bash tools/dev/gpu_occ_ab.sh occ1
