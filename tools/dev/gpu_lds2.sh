#!/bin/bash
set -eo pipefail
O=gpurun_out/lds2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_large_codes.py -x -q --timeout 120 --timeout-method thread -k "hgp10k or lds" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/bench_configs.py c4 --shots 262144 --reps 2 --p 0.03 > $O/c4.jsonl 2> $O/c4.err
cat $O/c4.jsonl
bash tools/dev/pmc_c4.sh
