#!/bin/bash
# LDS-resident min-sum kernel: large-code parity tests, then C4 throughput.
set -eo pipefail
O=gpurun_out/lds
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_codes.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python tools/bench_configs.py c4 --shots 262144 --reps 2 > $O/c4.jsonl 2> $O/c4.err
cat $O/c4.jsonl
