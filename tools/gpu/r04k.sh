#!/bin/bash
# Round 4, session k: compact kernel with LDS-DMA chunk staging and the inlined
# zero-row fix-up: compact/lean tests, stamps, bench.
set -eo pipefail
O=gpurun_out/r04k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "compact or lean or bench or misaligned" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/dev/stamps_cmp.py 0.001 0.0032 0.01 0.1 > $O/stamps_f64.log 2>&1 || { tail -20 $O/stamps_f64.log; exit 1; }
grep "^p=" $O/stamps_f64.log
STAMP_PREC=f32 timeout -k 10 300 python tools/dev/stamps_cmp.py 0.001 0.1 > $O/stamps_f32.log 2>&1 || { tail -20 $O/stamps_f32.log; exit 1; }
grep "^p=" $O/stamps_f32.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-large-code --no-sample-phase > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json
