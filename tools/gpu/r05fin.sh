#!/bin/bash
# Round 5, final tree (f64 LDS-resident C4 kernel): full GPU suite, smoke,
# default bench, rocprofv3 kernel trace + stats of the same command.
set -eo pipefail
O=gpurun_out/${1:-r05fin}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
python tools/rocprof_phases.py $O/prof/run_kernel_trace.csv $O/prof_bench.json $O/rocprof_phases.json
cp $O/prof/run_kernel_stats.csv $O/rocprof_kernel_stats.csv
