#!/bin/bash
# Round 3 diagnostics at both precisions: configs 3 and 4 (bench_configs), the
# C2 secondary line (R = 1 bpssf_hybrid, min-sum, 50 iterations) at f64 and f32.
set -eo pipefail
O=gpurun_out/r03g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_configs.py c3 c4 --shots 1048576 --reps 2 > $O/cfg_c3_c4.jsonl 2> $O/cfg.err || { tail -20 $O/cfg.err; exit 1; }
cat $O/cfg_c3_c4.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['config'], d['precision'], d['p'], '%.0f shots/s' % d['shots_per_s'], 'it %.1f' % d['mean_bp_iters'])"
for PREC in f64 f32; do
  timeout -k 10 300 python -u tools/bench_modes.py --modes bpssf_hybrid:1 --bp_method ms --max_iter 50 --p 0.001 --p 0.01 --p 0.03 --p 0.1 --precision $PREC > $O/modes_hybrid_$PREC.jsonl 2> $O/modes_$PREC.err || { tail -20 $O/modes_$PREC.err; exit 1; }
  cat $O/modes_hybrid_$PREC.jsonl
done
