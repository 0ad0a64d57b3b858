#!/bin/bash
# Round 4, session d: LDS padding of the compact kernel (even placement of the
# capped f64 grid) A/B: padded (default), unpadded, one-pass; interleaved.
set -eo pipefail
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none"
for V in 1 2; do
  timeout -k 10 300 python bench.py $A > $O/bench_pad$V.json 2> $O/bench_pad$V.err || { tail -20 $O/bench_pad$V.err; exit 1; }
  python tools/bench_summary.py $O/bench_pad$V.json
  QDEC_CMP_LDS_PAD=0 timeout -k 10 300 python bench.py $A > $O/bench_nopad$V.json 2> $O/bench_nopad$V.err || { tail -20 $O/bench_nopad$V.err; exit 1; }
  python tools/bench_summary.py $O/bench_nopad$V.json
  QDEC_COMPACT=0 timeout -k 10 300 python bench.py $A > $O/bench_one$V.json 2> $O/bench_one$V.err || { tail -20 $O/bench_one$V.err; exit 1; }
  python tools/bench_summary.py $O/bench_one$V.json
done
