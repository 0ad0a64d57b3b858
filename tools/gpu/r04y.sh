#!/bin/bash
# Round 4, session y: overlapped-phase occupancy of the f64 compact kernel:
# 12 waves per CU (3-per-SIMD build, the default) vs 16 (the same build, a larger grid),
# 3x interleaved, headline only.
set -eo pipefail
O=gpurun_out/r04y
mkdir -p $O
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none --iso-steps 1"
for V in 1 2 3; do
  for W in 12 8; do
    timeout -k 10 300 python bench.py $A --wave-occupancy $W > $O/bench_w$W-$V.json 2> $O/bench_w$W-$V.err || { tail -20 $O/bench_w$W-$V.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_w$W-$V.json')); print('w$W-$V %.2f M/s %.3f ms/step' % (d['value']/1e6, d['ms_per_step']))"
  done
done
