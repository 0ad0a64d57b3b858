#!/bin/bash
# GPU check of the large-graph kernels: parity (auto selection and the shot-lane
# kernel forced), then configs 4-5 throughput.
set -eo pipefail
O=gpurun_out/lane; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_codes.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
QDEC_LANE_KERNEL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_large_codes.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests_lane.log 2>&1 || { tail -40 $O/tests_lane.log; exit 1; }
tail -1 $O/tests_lane.log
timeout -k 10 600 python -u tools/bench_configs.py c4 c5 > $O/configs.jsonl 2> $O/configs.err
python -c "
import json
for l in open('$O/configs.jsonl'):
    d=json.loads(l); print(d['config'], d['p'], d['batch'], '%.4g shots/s'%d['shots_per_s'], 'bp_ms %.2f GBps %.0f'%(d['bp_kernel_ms_per_launch'], d['algorithmic_GBps_bp_kernel']))"
