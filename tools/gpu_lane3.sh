#!/bin/bash
set -eo pipefail
O=gpurun_out/lane3; mkdir -p $O; export TMPDIR=/tmp
QDEC_LANE_KERNEL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_large_codes.py -x -q --timeout 300 --timeout-method thread > $O/lane_tests.log 2>&1 || { tail -40 $O/lane_tests.log; exit 1; }
tail -1 $O/lane_tests.log
QDEC_LANE_KERNEL=1 timeout -k 10 300 python -u tools/bench_configs.py c4 --reps 2 --batch 131072 --shots 262144 > $O/c4_lane.jsonl 2> $O/c4_lane.err
python -c "
import json
for l in open('$O/c4_lane.jsonl'):
    d=json.loads(l); print(d['config'], d['p'], '%.4g shots/s'%d['shots_per_s'], 'bp_ms %.1f GBps %.0f'%(d['bp_kernel_ms_per_launch'], d['algorithmic_GBps_bp_kernel']))"
