#!/bin/bash
set -eo pipefail
O=gpurun_out/streams2; mkdir -p $O; export TMPDIR=/tmp
for S in 3 4 5 9; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --streams $S > $O/bench_s$S.json 2> $O/bench_s$S.err
  python -c "import json; d=json.load(open('$O/bench_s$S.json')); print('streams $S', round(d['value']/1e6, 2), 'M shots/s', round(d['ms_per_step'], 3), 'ms/step', 'bp_ms', round(d['roofline']['avg_launch_ms'],3), 'ssf_ms', round(d['roofline']['ssf_avg_launch_ms'],3))"
done
