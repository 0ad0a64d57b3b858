#!/bin/bash
# Round 5, session o: A/B of the f64 wave-kernel layout -- the production
# sequential anneals (A: libqdec_hip.so) against the joint anneal of lane order,
# row positions and state slots (B: libqdec_hip_joint.so, 12 M moves); wave
# kernel parity under B, then two interleaved bench runs of each.
set -eo pipefail
O=gpurun_out/${1:-r05o}
mkdir -p $O
B=$PWD/exp_ldpc_amd/libqdec_hip_joint.so
QDEC_LIB=$B timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_joint.log 2>&1 || { tail -30 $O/gpu_tests_joint.log; exit 1; }
tail -1 $O/gpu_tests_joint.log
ARGS="--no-cpu-baseline --no-c4 --no-reference-default --no-large-code --no-sample-phase"
for r in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > $O/a_$r.json 2> $O/a_$r.err || { tail -5 $O/a_$r.err; exit 1; }
  QDEC_LIB=$B timeout -k 10 300 python bench.py $ARGS > $O/b_$r.json 2> $O/b_$r.err || { tail -5 $O/b_$r.err; exit 1; }
done
python - <<'PY'
import json, sys
O = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r05o"
PY
for f in $O/a_1.json $O/b_1.json $O/a_2.json $O/b_2.json; do python -c "
import json,sys; b=json.load(open('$f')); r=b['roofline']
print('$f', round(b['value']/1e6,2), 'iso', round(r['isolated_step_ms'],2), 'avg', round(r['avg_launch_ms'],3), [round(v['bp_ms'],3) for v in r['per_point'].values()][-3:])"; done
