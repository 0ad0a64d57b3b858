#!/bin/bash
# f64 wave kernel occupancy A/B: 8 (default) vs 12 waves per CU (166 VGPRs fit 3 per SIMD).
set -eo pipefail
O=gpurun_out/r03j
mkdir -p $O
export TMPDIR=/tmp
for C in 8 12 8 12; do
  QDEC_F64_WAVES_PER_CU=$C timeout -k 10 300 python bench.py --no-cpu-baseline --variant none --no-sample-phase --no-large-code > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
  python - $O/bench_$C.json $C <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("cap", sys.argv[2], "value %.2f M/s  ms/step %.2f" % (d["value"] / 1e6, d["ms_per_step"]),
      "bp", [round(v["bp_kernel_ms_isolated"], 3) for v in d["ler"].values()], "bp_sum %.2f" % sum(v["bp_kernel_ms_isolated"] for v in d["ler"].values()))
PY
done
