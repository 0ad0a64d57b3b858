#!/bin/bash
# Round-6 evidence: GPU suite, smoke, default bench (+ side file), rocprofv3
# kernel-trace stats of the same command and its phase split, PMC of the
# headline kernels, C5 (decoding point and bandwidth point), C3 and C4 f64.
# Usage: tools/gpu/r06_final.sh <tag> [skip-tests|tests] [no-pmc]
set -eo pipefail
TAG=${1:-r06fin}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -2 $O/smoke.log
fi
timeout -k 10 400 python -u bench.py --detail-out $O/bench_detail.json > $O/bench.json 2> $O/bench.err
python -c "import json; s=open('$O/bench.json').read().strip(); d=json.loads(s); print(len(s), 'B;', d['value']/1e6, 'M/s', d['ms_per_step'], 'frac', d['roofline']['frac'], d.get('configs',{}).get('c5'))"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --detail-out $O/bench_detail_prof.json > $O/bench_prof.json 2> $O/bench_prof.err
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/rocprof_kernel_stats.csv \;
python3 tools/rocprof_phases.py $(find $O/prof -name "*kernel_trace.csv" | head -1) $O/bench_detail_prof.json $O/rocprof_phases.json > $O/rocprof_phases.log 2>&1 || echo "phases split failed"
echo "rocprof done"
# two ranks on the one GPU (rank r uses device r mod visible devices): the N > 1
# launch path and its one JSON line (not a scaling figure)
timeout -k 10 400 python -u bench.py --gpus 2 --no-cpu-baseline --detail-out $O/bench_2ranks_detail.json > $O/bench_2ranks.json 2> $O/bench_2ranks.err
python -c "import json; d=json.load(open('$O/bench_2ranks.json')); print('2 ranks:', d['n_gpus'], d['value']/1e6, 'M/s', d['ranks_seen'])"
[ "${3:-}" = "no-pmc" ] && exit 0
PMC_META="" bash tools/pmc.sh $O/pmc_bench --no-c4 --no-large-code --no-reference-default --no-c3 --no-cpu-baseline --steps 2
PMC_HBM=1 PMC_META="c5_p=0.005 c5_shots=65536" bash tools/pmc_cmd.sh $O/pmc_c5_p005 tools/gpu/lines_only.py --c5 --c5-p 0.005 --c5-warm-full
PMC_HBM=1 PMC_META="c5_p=0.001 c5_shots=65536" bash tools/pmc_cmd.sh $O/pmc_c5_p001 tools/gpu/lines_only.py --c5 --c5-p 0.001 --c5-warm-full
PMC_HBM=1 bash tools/pmc_cmd.sh $O/pmc_c3 tools/gpu/lines_only.py --c3
bash tools/pmc_cmd.sh $O/pmc_c4 tools/gpu/c4_only.py --prec f64 --p 0.01 --shots 131072
echo "pmc done"
