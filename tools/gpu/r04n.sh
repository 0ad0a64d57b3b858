#!/bin/bash
# Round 4, session n: A/B/C, interleaved, same box: A = commit 97db563 (chunk
# entries prefetched into registers), B = current (LDS-DMA chunk staging,
# counted hand-off wait, 8-entry chunks, inlined zero-row fix-up in the f64
# 2-wave build), C = B without the inlined fix-up.
set -eo pipefail
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none"
for V in 1 2; do
  for L in A B C; do
    if [ $L = B ]; then LIB=$PWD/exp_ldpc_amd/libqdec_hip.so; else LIB=$PWD/exp_ldpc_amd/libqdec_hip_$L.so; fi
    QDEC_LIB=$LIB timeout -k 10 300 python bench.py $A > $O/bench_$L$V.json 2> $O/bench_$L$V.err || { tail -20 $O/bench_$L$V.err; exit 1; }
    echo "== $L$V"; python tools/bench_summary.py $O/bench_$L$V.json | grep -v kernel
  done
done
