#!/bin/bash
set -eo pipefail
O=gpurun_out/lane4; mkdir -p $O; export TMPDIR=/tmp
show() { python -c "
import json
for l in open('$1'):
    d=json.loads(l); print('$2', d['config'], d['p'], d['batch'], '%.4g shots/s'%d['shots_per_s'], 'bp_ms %.1f GBps %.0f'%(d['bp_kernel_ms_per_launch'], d['algorithmic_GBps_bp_kernel']))"; }
QDEC_LANE_KERNEL=1 timeout -k 10 300 python -u tools/bench_configs.py c4 --reps 2 --batch 32768 --shots 131072 > $O/c4_lane_b32k.jsonl 2> $O/e1.err
show $O/c4_lane_b32k.jsonl lane
QDEC_LANE_KERNEL=1 QDEC_LANE_SCRATCH_MB=65536 timeout -k 10 400 python -u tools/bench_configs.py c5 --reps 2 --batch 8192 --shots 16384 > $O/c5_lane.jsonl 2> $O/e2.err
show $O/c5_lane.jsonl lane
timeout -k 10 400 python -u tools/bench_configs.py c5 --reps 2 --batch 8192 --shots 16384 > $O/c5_block.jsonl 2> $O/e3.err
show $O/c5_block.jsonl block
