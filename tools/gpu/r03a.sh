#!/bin/bash
# Round 3, first pass: large-code GPU tests (config 5 as named, slot-group
# kernel), then config-5 throughput at f32 / f64.
set -eo pipefail
O=gpurun_out/r03a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_large_codes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/large_tests.log 2>&1 || { tail -40 $O/large_tests.log; exit 1; }
tail -3 $O/large_tests.log
timeout -k 10 600 python -u tools/bench_configs.py c5 c5r0 --shots 262144 --reps 2 > $O/bench_c5.jsonl 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
cat $O/bench_c5.jsonl
