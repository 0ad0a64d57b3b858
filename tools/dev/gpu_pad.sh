#!/bin/bash
set -eo pipefail
for v in "" _nopad; do
for s in 1 5 9; do
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip$v.so timeout -k 10 120 python bench.py --streams $s --steps 5 --iso-steps 1 --no-cpu-baseline --no-sample-phase --variant none --precision f64 > gpurun_out/pad.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/pad.json')); print('lib$v streams $s', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
done
done
