#!/bin/bash
# Variations of the split-SSF + BP-priority schedule (bench.py), interleaved.
set -eo pipefail
O=gpurun_out/${1:-r06p2}
mkdir -p $O
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
F="--no-cpu-baseline --no-large-code --no-c4 --no-reference-default --no-c3 --no-sample-phase --variant none --steps 10"
for r in 1 2; do
  for cfg in "base:" "sp:--ssf-streams 1 --stream-priority 1" "sp_s3:--ssf-streams 1 --stream-priority 1 --streams 3" \
             "sp_desc:--ssf-streams 1 --stream-priority 1 --point-order desc" "sp_occ8:--ssf-streams 1 --stream-priority 1 --wave-occupancy 8" \
             "sp_s5:--ssf-streams 1 --stream-priority 1 --streams 5"; do
    name=${cfg%%:*}; flags=${cfg#*:}
    timeout -k 10 300 python -u bench.py $F $flags --detail-out $O/${name}_$r.detail.json > $O/${name}_$r.json 2> $O/${name}_$r.err
    python -c "import json,sys; d=json.load(open('$O/${name}_$r.json')); print('$name $r', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], 'ms')"
  done
done
