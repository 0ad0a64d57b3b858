#!/bin/bash
# Kernel timeline of the overlapped headline phase (rocprofv3 kernel trace),
# plus an A/B of the sweep points' launch order.
set -eo pipefail
O=gpurun_out/${1:-tl}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-sample-phase --variant none --no-large-code --steps 3 --iso-steps 1 > $O/prof_bench.json 2> $O/prof.err
echo traced
for r in 1 2; do
for order in asc desc; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sample-phase --variant none --no-large-code --steps 4 --point-order $order > $O/bench_$order$r.json 2> $O/bench_$order$r.err
python -c "import json,sys; d=json.load(open('$O/bench_$order$r.json')); print('$order', round(d['value']/1e6,2), round(d['ms_per_step'],2))"
done
done
