#!/bin/bash
# Wave-occupancy knob: parity (incl. the zero-syndrome and occupancy tests), then
# the default bench (12 f64 waves per CU in the overlapped phases) against --wave-occupancy 0.
set -eo pipefail
O=gpurun_out/r03p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for V in auto 0 auto 0; do
  A=""; [ $V = 0 ] && A="--wave-occupancy 0"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-sample-phase --no-large-code $A > $O/bench_$V.json 2> $O/bench_$V.err || { tail -20 $O/bench_$V.err; exit 1; }
  python - $O/bench_$V.json $V <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
v = d["variants"][0]["value"] if d.get("variants") else 0
print("%-4s f64 %.2f M/s  f32 %.2f M/s" % (sys.argv[2], d["value"] / 1e6, v / 1e6), d["config"]["wave_waves_per_cu"],
      "bp_sum %.2f" % sum(x["bp_kernel_ms_isolated"] for x in d["ler"].values()))
PY
done
