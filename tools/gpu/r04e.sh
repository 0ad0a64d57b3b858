#!/bin/bash
# Round 4, session e: kernel trace of the compact path (triage vs BP kernel
# durations per launch) and of the one-pass kernel, isolated-phase shapes.
set -eo pipefail
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none --steps 2 --warmup 1 --streams 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/cmp -o run --output-format csv -- python3 bench.py $A > $O/cmp.json 2> $O/cmp.err || { tail -20 $O/cmp.err; exit 1; }
QDEC_COMPACT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/one -o run --output-format csv -- python3 bench.py $A > $O/one.json 2> $O/one.err || { tail -20 $O/one.err; exit 1; }
ls -R $O | head -30
