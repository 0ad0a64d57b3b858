#!/bin/bash
set -eo pipefail
bash tools/gpu_quick.sh r02l
for prec in f64 f32; do
for sch in "--schedule pipeline" "--schedule streams --streams 5"; do
timeout -k 10 120 python bench.py $sch --steps 5 --iso-steps 1 --no-cpu-baseline --no-sample-phase --variant none --precision $prec > gpurun_out/sch.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/sch.json')); print('$prec $sch', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
done
done
