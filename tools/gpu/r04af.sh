#!/bin/bash
# Round 4, session af: the iteration-1 tile gate: default (>= 8 shots of
# syndrome weight <= 12) vs A (>= 2 shots of weight <= 20), interleaved x2.
set -eo pipefail
O=gpurun_out/r04af
mkdir -p $O
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none"
for V in 1 2; do
  for L in on A; do
    LIB=$PWD/exp_ldpc_amd/libqdec_hip.so
    if [ $L = A ]; then LIB=$PWD/exp_ldpc_amd/libqdec_hip_A.so; fi
    QDEC_LIB=$LIB timeout -k 10 300 python bench.py $A > $O/bench_$L$V.json 2> $O/bench_$L$V.err || { tail -20 $O/bench_$L$V.err; exit 1; }
    echo "== $L$V"; python tools/bench_summary.py $O/bench_$L$V.json | grep -v kernel | head -2
  done
done
