#!/bin/bash
# Price SSF inside the overlapped step: headline with and without SSF, interleaved.
set -eo pipefail
O=gpurun_out/${1:-r06i}
mkdir -p $O
A="--no-c3 --no-c4 --no-large-code --no-reference-default --no-cpu-baseline --variant none --iso-steps 1 --no-sample-phase"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py $A --detail-out $O/d_ssf_$r.json > $O/ssf_$r.json 2> $O/ssf_$r.err
  timeout -k 10 300 python -u bench.py $A --no-ssf-exp --detail-out $O/d_nossf_$r.json > $O/nossf_$r.json 2> $O/nossf_$r.err
  for k in ssf nossf; do python -c "import json; d=json.load(open('$O/${k}_$r.json')); print('$k', d['value']/1e6, d['ms_per_step'])"; done
done
