#!/bin/bash
# One GPU-box session: build check, GPU tests, smoke, bench, rocprof summary,
# PMC passes.  Usage (from the repo root on the box): tools/gpu_round.sh <tag>
# Every GPU step has its own time limit; the first failure ends the script.
set -eo pipefail
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/prof_bench.json 2> $O/prof.err
timeout -k 10 900 tools/pmc.sh $O/pmc --steps 2 --no-cpu-baseline
python tools/pmc_summary.py $O/pmc $O/pmc_summary.json
