#!/bin/bash
# One GPU-box evidence session: GPU tests, smoke, default bench, rocprof kernel
# trace + stats of the same command (split into the bench's phases), PMC passes.
# Usage (from the repo root on the box): tools/gpu_round.sh <tag>
# Every GPU step has its own time limit; the first failure ends the script.
set -eo pipefail
TAG=${1:-r02}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
echo bench done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/prof_bench.json 2> $O/prof.err
python tools/rocprof_phases.py $O/prof/run_kernel_trace.csv $O/prof_bench.json $O/rocprof_phases.json
timeout -k 10 1200 bash tools/pmc.sh $O/pmc --no-cpu-baseline > $O/pmc.log 2>&1
tail -5 $O/pmc.log
