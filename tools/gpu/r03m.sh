#!/bin/bash
# Layout A/B: state-write-aware slot anneal + f64 scatter floor 4 vs the round-2 layout (QDEC_MS_LAYOUT_V1).
set -eo pipefail
O=gpurun_out/r03m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for V in new v1 new v1; do
  if [ $V = v1 ]; then export QDEC_MS_LAYOUT_V1=1; else unset QDEC_MS_LAYOUT_V1; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --variant f32 --no-sample-phase --no-large-code --iso-steps 2 > $O/bench_$V.json 2> $O/bench_$V.err || { tail -20 $O/bench_$V.err; exit 1; }
  python - $O/bench_$V.json $V <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
v = d.get("variants", [{}])
v = v[0] if isinstance(v, list) and v else v
print(sys.argv[2], "f64 %.2f M/s" % (d["value"] / 1e6), "f32", {k: v.get(k) for k in ("value",) } if isinstance(v, dict) else v,
      "bp", [round(x["bp_kernel_ms_isolated"], 3) for x in d["ler"].values()], "bp_sum %.2f" % sum(x["bp_kernel_ms_isolated"] for x in d["ler"].values()))
PY
done
