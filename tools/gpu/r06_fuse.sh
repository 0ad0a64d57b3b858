#!/bin/bash
# Fused-SSF round: GPU tests of the bench path (packed inputs, parity, compact),
# then bench A/B: fused vs queued SSF, packed inputs, twice each interleaved.
set -eo pipefail
TAG=${1:-r06c}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_packed.py tests/test_gpu_parity.py tests/test_gpu_compact.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for fz in 1 0 1 0; do
  timeout -k 10 300 python -u bench.py --ssf-fuse $fz --no-c4 --no-large-code --no-reference-default --no-cpu-baseline --variant none --detail-out $O/detail_$fz.json > $O/bench_$fz.json 2> $O/bench_$fz.err
  python -c "import json; d=json.load(open('$O/bench_$fz.json')); r=d['roofline']; print('fuse=$fz', d['value']/1e6, 'M/s', d['ms_per_step'], 'bp', r['avg_launch_ms'], 'triage', r['triage']['avg_launch_ms'], 'ssf', r['ssf_avg_launch_ms'], 'iso', r['isolated_step_ms'], 'c3', d['configs']['c3']['shots_per_s'], d['ler']['failures'])"
done
timeout -k 10 300 python -u bench.py --inputs bytes --no-c4 --no-large-code --no-reference-default --no-cpu-baseline --variant none --detail-out $O/detail_bytes.json > $O/bench_bytes.json 2> $O/bench_bytes.err
python -c "import json; d=json.load(open('$O/bench_bytes.json')); r=d['roofline']; print('bytes', d['value']/1e6, 'M/s', d['ms_per_step'], 'triage', r['triage']['avg_launch_ms'], 'iso', r['isolated_step_ms'])"
