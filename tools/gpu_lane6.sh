#!/bin/bash
set -eo pipefail
O=gpurun_out/lane6; mkdir -p $O; export TMPDIR=/tmp
show() { python -c "
import json
for l in open('$1'):
    d=json.loads(l); print('$2', d['config'], d['p'], d['batch'], '%.4g shots/s'%d['shots_per_s'], 'bp_ms %.1f GBps %.0f'%(d['bp_kernel_ms_per_launch'], d['algorithmic_GBps_bp_kernel']))"; }
QDEC_LANE_KERNEL=1 QDEC_LANE_SCRATCH_MB=112000 timeout -k 10 500 python -u tools/bench_configs.py c5 --reps 2 --batch 32768 --shots 32768 > $O/c5_lane.jsonl 2> $O/e2.err
show $O/c5_lane.jsonl lane
