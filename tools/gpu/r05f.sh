#!/bin/bash
# Round 5, session f: A/B of the heavy-first compact list (libqdec_hip_noheavy.so:
# every listed shot light), then the evidence of the main library (r05e.sh:
# full GPU suite, smoke, default bench with the C4 / reference-default lines,
# rocprofv3 kernel trace + stats, PMC passes).
set -eo pipefail
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "ssf or bench_lean or compact" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ARGS="--no-cpu-baseline --no-large-code --no-sample-phase --no-c4 --no-reference-default --variant none"
for i in 1 2; do
  for v in main noheavy; do
    if [ $v = main ]; then L=""; else L=$PWD/exp_ldpc_amd/libqdec_hip_noheavy.so; fi
    QDEC_LIB=$L timeout -k 10 300 python bench.py $ARGS > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err || { tail -20 $O/ab_${v}_$i.err; exit 1; }
    echo "== $v $i"; python tools/bench_summary.py $O/ab_${v}_$i.json
  done
done
bash tools/gpu/r05e.sh r05f/ev
