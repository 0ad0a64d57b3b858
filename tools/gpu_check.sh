#!/bin/bash
# Quick evidence session: GPU tests, smoke, default bench.
# Usage (repo root on the box): tools/gpu_check.sh <tag>
set -eo pipefail
TAG=${1:-chk}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value']/1e6, 'M shots/s', d['roofline'].get('avg_launch_ms'), [ (k, v.get('value')) for k,v in d.get('variants',{}).items()] if isinstance(d.get('variants'),dict) else d.get('variants'))"
