#!/bin/bash
# Round 4, session b: the compact-list path (new tests first), then the GPU
# suite, smoke, default bench, the multi-rank bench path rehearsed with 2 ranks
# on the box's one GPU (gloo bookkeeping, real HIP decode), rocprof of the bench.
set -eo pipefail
O=gpurun_out/r04b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "compact or lean or bench" > $O/compact_tests.log 2>&1 || { tail -60 $O/compact_tests.log; exit 1; }
tail -1 $O/compact_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json
timeout -k 10 400 python bench.py --gpus 2 --steps 3 --no-cpu-baseline --no-large-code --no-sample-phase > $O/bench_2ranks.json 2> $O/bench_2ranks.err || { tail -30 $O/bench_2ranks.err; exit 1; }
python tools/bench_summary.py $O/bench_2ranks.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
python tools/rocprof_phases.py $O/prof/run_kernel_trace.csv $O/prof_bench.json $O/rocprof_phases.json
echo done
