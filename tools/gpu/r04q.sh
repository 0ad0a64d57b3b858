#!/bin/bash
# Round 4, session q: triage iteration 1 with table prefetch, tile gate, LDS logical rows.
# Compact + lean parity tests, then interleaved A/B bench (QDEC_TRIAGE_IT1=0
# vs on), then a kernel trace of the default path.
set -eo pipefail
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "compact or lean or bench or misaligned or triage" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none"
for V in 1 2; do
  for L in off on; do
    if [ $L = off ]; then E=0; else E=1; fi
    QDEC_TRIAGE_IT1=$E timeout -k 10 300 python bench.py $A > $O/bench_$L$V.json 2> $O/bench_$L$V.err || { tail -20 $O/bench_$L$V.err; exit 1; }
    echo "== $L$V"; python tools/bench_summary.py $O/bench_$L$V.json | grep -v kernel
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py $A --steps 2 --streams 1 > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
echo done
