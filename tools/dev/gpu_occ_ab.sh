#!/bin/bash
# A/B of the overlapped phase's f64 wave-kernel occupancy (bench --wave-occupancy).
set -eo pipefail
O=gpurun_out/${1:-occ}; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for w in 12 8; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sample-phase --variant none --no-large-code --steps 4 --wave-occupancy $w > $O/bench_w$w$r.json 2> $O/bench_w$w$r.err
python -c "import json; d=json.load(open('$O/bench_w$w$r.json')); print('waves $w', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
done
done
