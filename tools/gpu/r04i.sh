#!/bin/bash
# Round 4, session h: vectorised triage tiles; compact tests, the full GPU
# suite, bench, kernel trace.
set -eo pipefail
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "compact or lean or bench or misaligned" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
A="--no-cpu-baseline --no-large-code --no-sample-phase"
timeout -k 10 300 python bench.py $A > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py $A --variant none --steps 2 --streams 1 > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
echo done
