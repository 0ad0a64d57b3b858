#!/bin/bash
set -eo pipefail
bash tools/gpu_quick.sh r02j
for v in "" _occ5 _occ6; do
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip$v.so timeout -k 10 120 python bench.py --p 0.1 --p 0.0562341 --steps 2 --iso-steps 2 --no-cpu-baseline --no-sample-phase --variant none --precision f32 --streams 1 > gpurun_out/ssf$v.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/ssf$v.json')); print('lib$v ssf', [round(v['ssf_kernel_ms_isolated'],3) for v in d['ler'].values()], 'fails', [v['failures'] for v in d['ler'].values()])"
done
