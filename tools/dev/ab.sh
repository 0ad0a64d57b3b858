#!/bin/bash
# A/B: GPU parity tests for both min-sum kernels, then bench each.
set -eo pipefail
O=gpurun_out/${1:-ab}; mkdir -p $O; shift || true
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ms or ssf or fold or hybrid or edge or irregular" > $O/t1.log 2>&1 || { tail -30 $O/t1.log; exit 1; }
tail -1 $O/t1.log
QDEC_MS_WAVES=2 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ms or ssf or fold or hybrid or edge or irregular" > $O/t2.log 2>&1 || { tail -30 $O/t2.log; exit 1; }
tail -1 $O/t2.log
for W in 1 2; do
QDEC_MS_WAVES=$W timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench$W.json 2> $O/bench$W.err
python - "$O/bench$W.json" $W <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("waves", sys.argv[2], "value %.4g shots/s  ms/step %.3f" % (d["value"], d["ms_per_step"]))
print("  bp_ms", " ".join("%.3f" % v["bp_kernel_ms_per_launch"] for v in d["ler"].values()))
PY
done
