#!/bin/bash
# Packed-input round: the new GPU tests + the parity tests of the bench path,
# then the bench with packed and with byte inputs (A/B, same box).
set -eo pipefail
TAG=${1:-r06b}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_packed.py tests/test_gpu_parity.py tests/test_gpu_compact.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for inp in packed bytes packed bytes; do
  timeout -k 10 300 python -u bench.py --inputs $inp --no-c4 --no-large-code --no-reference-default --no-cpu-baseline --detail-out $O/detail_$inp.json > $O/bench_$inp.json 2> $O/bench_$inp.err
  python -c "import json; d=json.load(open('$O/bench_$inp.json')); r=d['roofline']; print('$inp', d['value']/1e6, 'M/s', d['ms_per_step'], 'triage', r['triage']['avg_launch_ms'], 'iso', r['isolated_step_ms'], 'c3', d['configs']['c3']['shots_per_s'])"
done
