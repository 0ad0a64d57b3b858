#!/bin/bash
# Round-end evidence: tests, smoke, bench + rocprof + PMC (gpu_round.sh), then the
# larger configs and the C2 secondary (R = 1 hybrid) line.
set -eo pipefail
TAG=${1:-r01e}
bash tools/gpu_round.sh $TAG
O=gpurun_out/$TAG
tail -1 $O/gpu_tests.log
tail -1 $O/smoke.log
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value']/1e6, 'M shots/s', d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'])"
timeout -k 10 900 python -u tools/bench_configs.py c3 c4 c5 > $O/configs.jsonl 2> $O/configs.err
cut -c1-200 $O/configs.jsonl
timeout -k 10 600 python -u tools/bench_modes.py --modes bpssf_hybrid:1,bpssf:1 --bp_method ms --max_iter 50 --p 0.001 --p 0.01 --p 0.03 --p 0.1 > $O/modes_c2_r1.jsonl 2> $O/modes.err
cut -c1-260 $O/modes_c2_r1.jsonl
