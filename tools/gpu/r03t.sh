#!/bin/bash
# SSF entry stage issued after the shot's steps: parity, bench twice, SSF stamps.
set -eo pipefail
O=gpurun_out/r03t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py tests/test_gpu_large_codes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for V in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-sample-phase --no-large-code > $O/bench_$V.json 2> $O/bench_$V.err || { tail -20 $O/bench_$V.err; exit 1; }
  python - $O/bench_$V.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("f64 %.2f M/s  f32 %.2f M/s" % (d["value"] / 1e6, d["variants"][0]["value"] / 1e6),
      "bp", [round(x["bp_kernel_ms_isolated"], 3) for x in d["ler"].values()],
      "ssf", [round(x["ssf_kernel_ms_isolated"], 3) for x in d["ler"].values()])
PY
done
timeout -k 10 300 python tools/dev/stamps.py 0.0316 0.1 > $O/stamps.log 2>&1 && grep SSF $O/stamps.log
