#!/bin/bash
# Split-SSF round: parity tests of the double-buffered SSF queues, then the
# headline with SSF on a stream per point vs on the point's stream (A/B x2).
set -eo pipefail
O=gpurun_out/${1:-r06j}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "split or stream or bench_lean" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--no-c3 --no-c4 --no-large-code --no-reference-default --no-cpu-baseline --variant none --iso-steps 1 --no-sample-phase"
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 300 python -u bench.py $A --ssf-streams $v --detail-out $O/d_$v_$r.json > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err
    python -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('ssf-streams=$v', d['value']/1e6, d['ms_per_step'], [d['ler']['failures'][i] for i in (0,4,8)])"
  done
done
