#!/bin/bash
# Headline step with SSF on per-point streams at default vs BP streams at high
# priority (bench.py --stream-priority), interleaved.
set -eo pipefail
O=gpurun_out/${1:-r06p}
mkdir -p $O
F="--no-cpu-baseline --no-large-code --no-c4 --no-reference-default --no-c3 --no-sample-phase --variant none --steps 10"
for r in 1 2; do
  for cfg in "base:" "split:--ssf-streams 1" "split_prio:--ssf-streams 1 --stream-priority 1" "prio:--stream-priority 1"; do
    name=${cfg%%:*}; flags=${cfg#*:}
    timeout -k 10 300 python -u bench.py $F $flags --detail-out $O/${name}_$r.detail.json > $O/${name}_$r.json 2> $O/${name}_$r.err
    python -c "import json,sys; d=json.load(open('$O/${name}_$r.json')); print('$name $r', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms')"
  done
done
