#!/bin/bash
# Headline bench: stream count and launch order sweep (no CPU baseline).
set -eo pipefail
O=gpurun_out/sweep; mkdir -p $O; export TMPDIR=/tmp
for S in 3 5 7 9; do
  for H in "" "--heavy-first"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --streams $S $H > $O/b_$S$H.json 2> $O/b_$S$H.err
    python -c "import json; d=json.load(open('$O/b_$S$H.json')); print('streams $S $H', round(d['value']/1e6, 2), 'M shots/s', round(d['ms_per_step'], 3), 'ms/step')"
  done
done
