#!/bin/bash
# Round 5, session a: table-driven SSF kernel (ssf_lut_kernel) -- SSF / compact
# parity tests, then a short bench with per-point isolated SSF times.
set -eo pipefail
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compact.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "ssf or bench_lean or compact" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py --steps 5 --no-cpu-baseline --no-large-code --no-sample-phase > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/bench_summary.py $O/bench.json 2>/dev/null || python -c "
import json; d=json.load(open('$O/bench.json')); print(d['value']/1e6, 'M shots/s')
for k,r in d['ler'].items(): print(k, round(r['bp_kernel_ms_isolated'],3), round(r['ssf_kernel_ms_isolated'],3), r['overlaps_cpu_f64'] if 'overlaps_cpu_f64' in r else '')
"
