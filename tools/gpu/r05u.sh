#!/bin/bash
# Round 5, session u: the headline phase with and without SSF (diagnostic copy
# of bench.py), to price SSF inside the overlapped step.
set -eo pipefail
O=gpurun_out/${1:-r05u}
mkdir -p $O
ARGS="--no-cpu-baseline --no-c4 --no-reference-default --no-large-code --no-sample-phase --variant none"
for r in 1 2; do
  timeout -k 10 300 python tools/gpu/bench_nossf.py $ARGS > $O/ssf_$r.json 2> $O/ssf_$r.err || { tail -5 $O/ssf_$r.err; exit 1; }
  timeout -k 10 300 python tools/gpu/bench_nossf.py $ARGS --no-ssf-exp > $O/nossf_$r.json 2> $O/nossf_$r.err || { tail -5 $O/nossf_$r.err; exit 1; }
done
for f in $O/ssf_1.json $O/nossf_1.json $O/ssf_2.json $O/nossf_2.json; do python -c "
import json; b=json.load(open('$f')); print('$f', round(b['value']/1e6,2), round(b['ms_per_step'],2))"; done
