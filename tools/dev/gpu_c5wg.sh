#!/bin/bash
set -eo pipefail
O=gpurun_out/c5wg
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_codes.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python tools/bench_configs.py c5 --shots 65536 --reps 2 > $O/c5.jsonl 2> $O/c5.err
cat $O/c5.jsonl
for w in 4 3; do
QDEC_BLOCK_WG_PER_CU=$w timeout -k 10 240 python tools/bench_configs.py c5 --p 0.005 --shots 65536 --reps 1 > $O/c5_w$w.jsonl 2> $O/c5_w$w.err
python -c "import json; d=json.loads(open('$O/c5_w$w.jsonl').readline()); print('wg/cu $w', round(d['shots_per_s']), round(d['bp_kernel_ms_per_launch'],1))"
done
CFG=c5 P=0.005 SHOTS=32768 bash tools/dev/pmc_c4.sh
