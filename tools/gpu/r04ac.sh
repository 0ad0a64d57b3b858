#!/bin/bash
# Round 4, session ac: SSF kernel register budget: 5 waves per SIMD (default,
# <= 96 VGPRs, ~10 dwords spilled) vs 4 (A: -DQDEC_SSF_OCC=4, 111 VGPRs, no
# spill), interleaved x3; isolated SSF per point + headline.
set -eo pipefail
O=gpurun_out/r04ac
mkdir -p $O
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none"
for V in 1 2 3; do
  for L in on A; do
    LIB=$PWD/exp_ldpc_amd/libqdec_hip.so
    if [ $L = A ]; then LIB=$PWD/exp_ldpc_amd/libqdec_hip_A.so; fi
    QDEC_LIB=$LIB timeout -k 10 300 python bench.py $A > $O/bench_$L$V.json 2> $O/bench_$L$V.err || { tail -20 $O/bench_$L$V.err; exit 1; }
    echo "== $L$V"; python tools/bench_summary.py $O/bench_$L$V.json | grep -v kernel
  done
done
