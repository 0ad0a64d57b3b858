#!/bin/bash
# Round 5, session v: SSF early exit (empty workgroups return before loading
# the tables). Parity of the SSF paths first, then an interleaved A/B of the
# headline phase: a = library before the change, b = with it.
set -eo pipefail
O=gpurun_out/${1:-r05v}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_compact.py tests/test_gpu_large_codes.py > $O/pytest.log 2>&1 \
  || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
ARGS="--no-cpu-baseline --no-c4 --no-reference-default --no-large-code --no-sample-phase --variant none"
for r in 1 2 3; do
  QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_a.so timeout -k 10 300 python bench.py $ARGS > $O/a_$r.json 2> $O/a_$r.err || { tail -5 $O/a_$r.err; exit 1; }
  timeout -k 10 300 python bench.py $ARGS > $O/b_$r.json 2> $O/b_$r.err || { tail -5 $O/b_$r.err; exit 1; }
done
timeout -k 10 300 python tools/gpu/bench_nossf.py $ARGS --no-ssf-exp > $O/nossf.json 2> $O/nossf.err || { tail -5 $O/nossf.err; exit 1; }
for f in $O/a_1.json $O/b_1.json $O/a_2.json $O/b_2.json $O/a_3.json $O/b_3.json $O/nossf.json; do python -c "
import json; b=json.load(open('$f')); print('$f', round(b['value']/1e6,2), round(b['ms_per_step'],2))"; done
