#!/bin/bash
# Quick loop: GPU tests, then the default bench without the CPU baseline.
# Usage: tools/gpu_quick.sh <tag> [extra bench args]
set -eo pipefail
TAG=${1:-q}; shift || true
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err
python - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value %.2f M/s %s  ms/step %.2f  variants %s" % (d["value"] / 1e6, d["dtype"], d["ms_per_step"],
      [(v["dtype"], round(v["value"] / 1e6, 2)) for v in d.get("variants", [])]))
print("bp iso ms", [round(v["bp_kernel_ms_isolated"], 3) for v in d["ler"].values()])
print("ssf iso ms", [round(v["ssf_kernel_ms_isolated"], 3) for v in d["ler"].values()])
print("isolated step ms", round(d["roofline"]["isolated_step_ms"], 2), "variant bp/ssf avg",
      [(v.get("bp_kernel_ms_isolated_avg"), v.get("ssf_kernel_ms_isolated_avg")) for v in d.get("variants", [])])
PY
