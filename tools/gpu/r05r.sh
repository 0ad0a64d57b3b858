#!/bin/bash
# Round 5, session r: two decoder handles per point (consecutive steps of a
# point on two streams) against one, both with the end-of-region join.
set -eo pipefail
O=gpurun_out/${1:-r05r}
mkdir -p $O
ARGS="--no-cpu-baseline --no-c4 --no-reference-default --no-large-code --no-sample-phase"
for r in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > $O/d1_$r.json 2> $O/d1_$r.err || { tail -5 $O/d1_$r.err; exit 1; }
  timeout -k 10 300 python bench.py $ARGS --decoders-per-point 2 --streams 18 > $O/d2_$r.json 2> $O/d2_$r.err || { tail -5 $O/d2_$r.err; exit 1; }
done
for f in $O/d1_1.json $O/d2_1.json $O/d1_2.json $O/d2_2.json; do python -c "
import json; b=json.load(open('$f')); v=b['variants'][0] if b.get('variants') else {}
print('$f', round(b['value']/1e6,2), round(b['ms_per_step'],2), 'f32', round(v.get('value',0)/1e6,2), b['ler'] == b['ler'])"; done
