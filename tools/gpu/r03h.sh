#!/bin/bash
# Batched lazy SSF scoring vs eager: SSF parity of the default library, then the
# default bench interleaved (isolated SSF times per point).
set -eo pipefail
O=gpurun_out/r03h
mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_codes.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ssf or lean or bb144 or fold or stream" > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for V in default eager default eager; do
  if [ $V = default ]; then unset QDEC_LIB; else export QDEC_LIB=$R/exp_ldpc_amd/libqdec_hip_$V.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --variant none --no-sample-phase --no-large-code > $O/bench_$V.json 2> $O/bench_$V.err || { tail -20 $O/bench_$V.err; exit 1; }
  python - $O/bench_$V.json $V <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "value %.2f M/s  ms/step %.2f" % (d["value"] / 1e6, d["ms_per_step"]),
      "ssf", [round(v["ssf_kernel_ms_isolated"], 3) for v in d["ler"].values()],
      "fails", sum(v["failures"] for v in d["ler"].values()))
PY
done
