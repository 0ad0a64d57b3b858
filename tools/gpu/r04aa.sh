#!/bin/bash
# Round 4, session aa: hardware queues per process for the 9-stream headline:
# HIP's default (4 on this pool) vs GPU_MAX_HW_QUEUES=9 / 16, interleaved.
set -eo pipefail
O=gpurun_out/r04aa
mkdir -p $O
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none --iso-steps 1"
for V in 1 2 3; do
  for Q in 4 9 16; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py $A > $O/bench_q$Q-$V.json 2> $O/bench_q$Q-$V.err || { tail -20 $O/bench_q$Q-$V.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_q$Q-$V.json')); print('q$Q-$V %.2f M/s %.3f ms/step' % (d['value']/1e6, d['ms_per_step']))"
  done
done
