#!/bin/bash
# Round 5, session q: the streams schedule joined every step (default) against
# joined only at the end of the timed region (--step-join end), interleaved.
set -eo pipefail
O=gpurun_out/${1:-r05q}
mkdir -p $O
ARGS="--no-cpu-baseline --no-c4 --no-reference-default --no-large-code --no-sample-phase"
for r in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > $O/step_$r.json 2> $O/step_$r.err || { tail -5 $O/step_$r.err; exit 1; }
  timeout -k 10 300 python bench.py $ARGS --step-join end > $O/end_$r.json 2> $O/end_$r.err || { tail -5 $O/end_$r.err; exit 1; }
done
for f in $O/step_1.json $O/end_1.json $O/step_2.json $O/end_2.json; do python -c "
import json; b=json.load(open('$f')); v=b['variants'][0] if b.get('variants') else {}
print('$f', round(b['value']/1e6,2), round(b['ms_per_step'],2), 'f32', round(v.get('value',0)/1e6,2))"; done
