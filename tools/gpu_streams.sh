#!/bin/bash
# Headline bench with the sweep points on 1/2/3 HIP streams, then the opt-in
# shot-lane kernel: parity + config-4 throughput.
set -eo pipefail
O=gpurun_out/streams; mkdir -p $O; export TMPDIR=/tmp
for S in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --streams $S > $O/bench_s$S.json 2> $O/bench_s$S.err
  python -c "import json; d=json.load(open('$O/bench_s$S.json')); print('streams $S', round(d['value']/1e6, 2), 'M shots/s', round(d['ms_per_step'], 3), 'ms/step')"
done
QDEC_LANE_KERNEL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_large_codes.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/lane_tests.log 2>&1 || { tail -40 $O/lane_tests.log; exit 1; }
tail -1 $O/lane_tests.log
QDEC_LANE_KERNEL=1 timeout -k 10 300 python -u tools/bench_configs.py c4 --reps 2 --batch 131072 --shots 262144 > $O/c4_lane.jsonl 2> $O/c4_lane.err
cut -c1-260 $O/c4_lane.jsonl
