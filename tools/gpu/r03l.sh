#!/bin/bash
# Headline sweep: f64 waves per CU (8 / 12) x streams (3 / 5 / 9), interleaved.
set -eo pipefail
O=gpurun_out/r03l
mkdir -p $O
for rep in 1 2; do
  for S in 9 5 3; do
    for C in 8 12; do
      QDEC_F64_WAVES_PER_CU=$C timeout -k 10 300 python bench.py --no-cpu-baseline --variant none --no-sample-phase --no-large-code --iso-steps 1 --streams $S > $O/b_${C}_${S}_$rep.json 2> $O/b_${C}_${S}_$rep.err || { tail -20 $O/b_${C}_${S}_$rep.err; exit 1; }
      python -c "import json; d=json.load(open('$O/b_${C}_${S}_$rep.json')); print('cap $C streams $S rep $rep: %.2f M/s  %.2f ms/step' % (d['value']/1e6, d['ms_per_step']))"
    done
  done
done
