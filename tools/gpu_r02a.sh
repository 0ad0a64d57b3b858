#!/bin/bash
# Round-2 first look: GPU tests, f32/f64 single-stream benches, rocprof stats.
set -eo pipefail
O=gpurun_out/r02a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo tests done
timeout -k 10 300 python bench.py --streams 1 --no-cpu-baseline --precision f32 > $O/bench_f32_s1.json 2> $O/bench_f32_s1.err
echo f32 done
timeout -k 10 300 python bench.py --streams 1 --no-cpu-baseline --precision f64 > $O/bench_f64_s1.json 2> $O/bench_f64_s1.err
echo f64 done
timeout -k 10 300 python bench.py --streams 5 --no-cpu-baseline --precision f64 > $O/bench_f64_s5.json 2> $O/bench_f64_s5.err
echo f64 s5 done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --streams 1 --no-cpu-baseline --precision f64 > $O/prof_bench.json 2> $O/prof.err
echo prof done
