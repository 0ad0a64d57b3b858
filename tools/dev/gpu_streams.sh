#!/bin/bash
set -eo pipefail
for prec in f64 f32; do
for s in 5 7 9 12; do
timeout -k 10 120 python bench.py --streams $s --steps 5 --iso-steps 1 --no-cpu-baseline --no-sample-phase --variant none --precision $prec > gpurun_out/st.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/st.json')); print('$prec streams $s', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
done
done
