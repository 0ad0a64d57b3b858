#!/bin/bash
# Round 5, session c: SSF toggle rows read in one round trip -- SSF / compact
# parity tests, short bench (headline + isolated kernels only).
set -eo pipefail
O=gpurun_out/${1:-r05c}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "ssf or bench_lean or compact" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-large-code --no-sample-phase --no-c4 --no-reference-default \
    > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json
