#!/bin/bash
# Iteration-1 check state from the priors + zero-syndrome shortcut (f64): parity, then bench A/B against the QDEC_NO_ST1 build.
set -eo pipefail
O=gpurun_out/r03o
mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for V in new cmp new cmp; do
  unset QDEC_MS_LAYOUT_V1 QDEC_LIB
  
  [ $V = cmp ] && export QDEC_LIB=$R/exp_ldpc_amd/libqdec_hip_nost1.so
  timeout -k 10 300 python bench.py --no-cpu-baseline --variant f32 --no-sample-phase --no-large-code --iso-steps 2 > $O/bench_$V.json 2> $O/bench_$V.err || { tail -20 $O/bench_$V.err; exit 1; }
  python - $O/bench_$V.json $V <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
v = d["variants"][0]["value"] if d.get("variants") else 0
print("%-4s f64 %.2f M/s  f32 %.2f M/s" % (sys.argv[2], d["value"] / 1e6, v / 1e6),
      "bp", [round(x["bp_kernel_ms_isolated"], 3) for x in d["ler"].values()], "bp_sum %.2f" % sum(x["bp_kernel_ms_isolated"] for x in d["ler"].values()))
PY
done
