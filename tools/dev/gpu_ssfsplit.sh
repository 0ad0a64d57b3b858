#!/bin/bash
set -eo pipefail
bash tools/gpu_quick.sh r02p
for ns in 0 1; do
QDEC_SSF_NOSPLIT=$ns timeout -k 10 120 python bench.py --p 0.1 --p 0.0562341 --p 0.0316228 --steps 2 --iso-steps 2 --no-cpu-baseline --no-sample-phase --variant none --precision f32 --streams 1 > gpurun_out/ssfs.json 2>/dev/null
python -c "import json; d=json.load(open('gpurun_out/ssfs.json')); print('nosplit $ns ssf', [round(v['ssf_kernel_ms_isolated'],3) for v in d['ler'].values()], [v['failures'] for v in d['ler'].values()])"
done
