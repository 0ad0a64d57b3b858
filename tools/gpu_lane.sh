#!/bin/bash
# GPU check of the large-graph kernels: parity with the opt-in shot-lane kernel,
# then config-4 throughput with and without it.
set -eo pipefail
O=gpurun_out/lane2; mkdir -p $O; export TMPDIR=/tmp
QDEC_LANE_KERNEL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_large_codes.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
QDEC_LANE_KERNEL=1 timeout -k 10 300 python -u tools/bench_configs.py c4 --reps 2 >> $O/configs.jsonl 2>> $O/configs.err
QDEC_LANE_KERNEL=1 timeout -k 10 300 python -u tools/bench_configs.py c4 --reps 2 --batch 131072 --shots 262144 >> $O/configs.jsonl 2>> $O/configs.err
timeout -k 10 300 python -u tools/bench_configs.py c4 --reps 2 --batch 131072 --shots 262144 >> $O/configs.jsonl 2>> $O/configs.err
cat $O/configs.jsonl | cut -c1-300
