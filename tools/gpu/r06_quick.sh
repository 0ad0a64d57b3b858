#!/bin/bash
# Quick round: the bench-path GPU tests, then one default bench (no extra configs).
set -eo pipefail
TAG=${1:-r06d}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_packed.py tests/test_gpu_compact.py} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} --no-c4 --no-large-code --no-reference-default --no-cpu-baseline --variant none --detail-out $O/detail_$r.json > $O/bench_$r.json 2> $O/bench_$r.err
python - <<PY
import json; d=json.load(open('$O/bench_$r.json')); r=d['roofline']
dd=json.load(open('$O/detail_$r.json')); pp=dd['roofline']['per_point']
print(d['value']/1e6, 'M/s', d['ms_per_step'], 'bp', r['avg_launch_ms'], 'ssf', r['ssf_avg_launch_ms'], 'iso', r['isolated_step_ms'], 'c3', d['configs']['c3']['shots_per_s'])
print('triage us', [round(pp[str(i)]['triage_ms']*1000,1) for i in range(9)])
print('bp ms', [round(pp[str(i)]['bp_ms'],3) for i in range(9)])
PY
done
