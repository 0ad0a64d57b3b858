#!/bin/bash
# Workgroup-kernel changes: parity (small and large codes), then config 5
# (PSL(2,13) lift, R = 1 spacetime graph) with one 2^15-shot launch per pass.
set -eo pipefail
O=gpurun_out/c5; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_codes.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python -u tools/bench_configs.py c5 --reps 2 > $O/c5.jsonl 2> $O/c5.err
cut -c1-420 $O/c5.jsonl
timeout -k 10 600 python -u tools/bench_configs.py c4 --reps 2 --batch 131072 --shots 262144 > $O/c4_block.jsonl 2> $O/c4_block.err
cut -c1-420 $O/c4_block.jsonl
