#!/bin/bash
# Round 4, session g: compact-kernel placement A/B (f64 at <= 2 waves per SIMD
# by a pinned VGPR count vs the unpinned build vs the one-pass kernel), the
# compact parity tests, and a kernel trace (triage vs BP durations).
set -eo pipefail
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "compact or lean or bench" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--no-cpu-baseline --no-large-code --no-sample-phase --variant none"
for V in 1 2; do
  timeout -k 10 300 python bench.py $A > $O/bench_pin$V.json 2> $O/bench_pin$V.err || { tail -20 $O/bench_pin$V.err; exit 1; }
  python tools/bench_summary.py $O/bench_pin$V.json | grep -v kernel
  QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_nopin.so timeout -k 10 300 python bench.py $A > $O/bench_nopin$V.json 2> $O/bench_nopin$V.err || { tail -20 $O/bench_nopin$V.err; exit 1; }
  python tools/bench_summary.py $O/bench_nopin$V.json | grep -v kernel
  QDEC_COMPACT=0 timeout -k 10 300 python bench.py $A > $O/bench_one$V.json 2> $O/bench_one$V.err || { tail -20 $O/bench_one$V.err; exit 1; }
  python tools/bench_summary.py $O/bench_one$V.json | grep -v kernel
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py $A --steps 2 --streams 1 > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
echo done
