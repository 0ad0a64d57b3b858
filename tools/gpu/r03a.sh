#!/bin/bash
# Round 3, first pass: large-code GPU tests (config 5 as named, slot-group
# kernel), config-5 throughput at f32 / f64, the new parity tests (bench LEAN
# kernels at all 9 points, bposd_hybrid end to end), HBM calibration passes.
set -eo pipefail
O=gpurun_out/r03a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_large_codes.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/large_tests.log 2>&1 || { tail -40 $O/large_tests.log; exit 1; }
tail -3 $O/large_tests.log
timeout -k 10 600 python -u tools/bench_configs.py c5 c5r0 --shots 262144 --reps 2 > $O/bench_c5.jsonl 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
cat $O/bench_c5.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py -m gpu -x -v --timeout 300 --timeout-method thread -k "lean_kernels or hybrid_matches" > $O/new_tests.log 2>&1 || { tail -40 $O/new_tests.log; exit 1; }
tail -3 $O/new_tests.log
timeout -k 10 700 bash tools/dev/gpu_calib.sh r03a/calib
