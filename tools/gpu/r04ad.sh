#!/bin/bash
# Round 4, session ad: triage register budget: default (164 VGPRs, 3 waves per
# SIMD) vs A (-DQDEC_TRIAGE_UB=8 -DQDEC_TRIAGE_OCC=4: 128 VGPRs, 4 per SIMD,
# 6 dwords spilled).  Kernel traces (isolated launches) + headline x2.
set -eo pipefail
O=gpurun_out/r04ad
mkdir -p $O
export TMPDIR=/tmp
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none"
for L in on A; do
  LIB=$PWD/exp_ldpc_amd/libqdec_hip.so
  if [ $L = A ]; then LIB=$PWD/exp_ldpc_amd/libqdec_hip_A.so; fi
  QDEC_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$L -o run --output-format csv -- python3 bench.py $A --steps 2 --streams 1 > $O/prof_$L.json 2> $O/prof_$L.err || { tail -20 $O/prof_$L.err; exit 1; }
done
for V in 1 2; do
  for L in on A; do
    LIB=$PWD/exp_ldpc_amd/libqdec_hip.so
    if [ $L = A ]; then LIB=$PWD/exp_ldpc_amd/libqdec_hip_A.so; fi
    QDEC_LIB=$LIB timeout -k 10 300 python bench.py $A > $O/bench_$L$V.json 2> $O/bench_$L$V.err || { tail -20 $O/bench_$L$V.err; exit 1; }
    echo "== $L$V"; python tools/bench_summary.py $O/bench_$L$V.json | grep -v kernel | head -2
  done
done
