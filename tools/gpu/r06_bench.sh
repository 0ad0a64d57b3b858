#!/bin/bash
# Default bench (the driver's command) with its side file, then the rocprofv3
# kernel-trace summary of the same command.  Usage: tools/gpu/r06_bench.sh <tag>
set -eo pipefail
TAG=${1:-r06a}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --detail-out $O/bench_detail.json > $O/bench.json 2> $O/bench.err
python -c "import json,sys; s=open('$O/bench.json').read().strip(); d=json.loads(s); print(len(s), 'B line;', d['value']/1e6, 'M shots/s;', d['roofline']['frac'], d.get('configs',{}).keys())"
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --detail-out $O/bench_detail_prof.json > $O/bench_prof.json 2> $O/bench_prof.err
  find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/rocprof_kernel_stats.csv \;
fi
