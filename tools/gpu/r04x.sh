#!/bin/bash
# Round 4, session x: the multi-rank bench path rehearsed with 4 ranks on the
# box's one GPU (gloo bookkeeping group, real HIP decode).
set -eo pipefail
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 500 python bench.py --gpus 4 --steps 2 --no-cpu-baseline --no-large-code --no-sample-phase > $O/bench_4ranks.json 2> $O/bench_4ranks.err || { tail -30 $O/bench_4ranks.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_4ranks.json')); print('4 ranks on 1 GPU:', d['n_gpus'], '%.2f M/s' % (d['value']/1e6), d['scaling'], d['config']['parallelism'], d['steps'])"
