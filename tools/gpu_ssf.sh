#!/bin/bash
# SSF wave kernel: parity vs the oracle, phase timers, per-launch times, headline bench.
set -eo pipefail
O=gpurun_out/ssf; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 240 python -u tools/dev/stamps.py 0.03 0.1 > $O/stamps.log 2>&1
grep SSF $O/stamps.log
timeout -k 10 240 python -u tools/dev/ssf_time.py > $O/ssf_time.log 2>&1
cat $O/ssf_time.log | grep -v Warn
timeout -k 10 300 python bench.py --no-cpu-baseline --streams 1 > $O/bench_s1.json 2> $O/bench_s1.err
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_s5.json 2> $O/bench_s5.err
python -c "
import json
for s in (1, 5):
    d = json.load(open('$O/bench_s%d.json' % s)); print('streams', s, round(d['value'] / 1e6, 2), 'M shots/s', round(d['ms_per_step'], 3), 'ms/step')
"
