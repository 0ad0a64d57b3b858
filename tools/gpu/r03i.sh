#!/bin/bash
# f64 check-pass row loads (7 of 8 slots) A/B on the default bench, after parity.
set -eo pipefail
O=gpurun_out/r03i
mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for V in default rowfull default rowfull default rowfull; do
  if [ $V = default ]; then unset QDEC_LIB; else export QDEC_LIB=$R/exp_ldpc_amd/libqdec_hip_$V.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --variant none --no-sample-phase --no-large-code > $O/bench_$V.json 2> $O/bench_$V.err || { tail -20 $O/bench_$V.err; exit 1; }
  python - $O/bench_$V.json $V <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "value %.2f M/s  ms/step %.2f" % (d["value"] / 1e6, d["ms_per_step"]),
      "bp", [round(v["bp_kernel_ms_isolated"], 3) for v in d["ler"].values()], "bp_sum %.2f" % sum(v["bp_kernel_ms_isolated"] for v in d["ler"].values()))
PY
done
