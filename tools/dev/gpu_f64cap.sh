#!/bin/bash
set -eo pipefail
bash tools/gpu_quick.sh r02i
timeout -k 10 120 python bench.py --p 0.1 --p 0.001 --p 0.03 --steps 2 --iso-steps 2 --no-cpu-baseline --no-sample-phase --variant none --precision f64 --streams 1 > gpurun_out/cap_def.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/cap_def.json')); print('default', [round(v['bp_kernel_ms_isolated'],3) for v in d['ler'].values()])"
