#!/bin/bash
# Round 4, session c: A/B of the compact-list path against the one-pass kernel
# (QDEC_COMPACT=0), interleaved, same box; then the 2-rank bench line.
set -eo pipefail
O=gpurun_out/r04c
mkdir -p $O
export TMPDIR=/tmp
A="--no-cpu-baseline --no-large-code --no-sample-phase"
for V in 1 2; do
  timeout -k 10 300 python bench.py $A > $O/bench_cmp$V.json 2> $O/bench_cmp$V.err || { tail -20 $O/bench_cmp$V.err; exit 1; }
  python tools/bench_summary.py $O/bench_cmp$V.json
  QDEC_COMPACT=0 timeout -k 10 300 python bench.py $A > $O/bench_one$V.json 2> $O/bench_one$V.err || { tail -20 $O/bench_one$V.err; exit 1; }
  python tools/bench_summary.py $O/bench_one$V.json
done
timeout -k 10 300 python bench.py --gpus 2 --steps 3 $A > $O/bench_2ranks.json 2> $O/bench_2ranks.err || { tail -30 $O/bench_2ranks.err; exit 1; }
python tools/bench_summary.py $O/bench_2ranks.json
