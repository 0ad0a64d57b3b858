#!/bin/bash
# Quick GPU check: GPU tests then a bench run without the CPU baseline.
# Usage: tools/gpu_quick.sh <tag> [bench args...]
set -eo pipefail
TAG=${1:-quick}; shift || true
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err
python - "$O/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value %.4g shots/s  ms/step %.3f  frac %.3f" % (d["value"], d["ms_per_step"], d["roofline"]["frac"]))
for p, v in d["ler"].items():
    print(p, "ler %.5f conv %.4f it %.2f ssf %.2f bp_ms %.3f ssf_ms %.3f" % (v["ler"], v["bp_converged_frac"], v["mean_bp_iters_rank0"], v.get("mean_ssf_steps_rank0", -1), v["bp_kernel_ms_per_launch"], v["ssf_kernel_ms_per_launch"]))
PY
