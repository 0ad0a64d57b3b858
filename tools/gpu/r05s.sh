#!/bin/bash
# Round 5, session s: with the end-of-region join -- hardware queues per
# process (4, the pool default, vs 9 and 16) and the overlapped phase's f64
# occupancy (12 waves per CU, the default, vs 8), interleaved.
set -eo pipefail
O=gpurun_out/${1:-r05s}
mkdir -p $O
ARGS="--no-cpu-baseline --no-c4 --no-reference-default --no-large-code --no-sample-phase --variant none"
for r in 1 2; do
  for q in 4 9 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py $ARGS > $O/q${q}_$r.json 2> $O/q${q}_$r.err || { tail -5 $O/q${q}_$r.err; exit 1; }
  done
  timeout -k 10 300 python bench.py $ARGS --wave-occupancy 8 > $O/occ8_$r.json 2> $O/occ8_$r.err || { tail -5 $O/occ8_$r.err; exit 1; }
done
for f in $O/q*_*.json $O/occ8_*.json; do python -c "
import json; b=json.load(open('$f')); print('$f', round(b['value']/1e6,2), round(b['ms_per_step'],2))"; done
