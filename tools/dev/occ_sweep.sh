#!/bin/bash
# Occupancy sweep of the BP kernel at p = 0.1 (QDEC_MAX_BLOCKS_PER_CU caps blocks per CU).
set -eo pipefail
for prec in f64 f32; do
  for cap in 0 12 8 4; do
    QDEC_MAX_BLOCKS_PER_CU=$cap timeout -k 10 120 python bench.py --p 0.1 --steps 2 --iso-steps 2 --no-cpu-baseline --no-sample-phase --variant none --precision $prec --streams 1 > gpurun_out/occ_${prec}_${cap}.json 2>/dev/null
    python -c "import json; d=json.load(open('gpurun_out/occ_${prec}_${cap}.json')); print('$prec cap $cap bp ms', round(d['roofline']['avg_launch_ms'],3))"
  done
done
