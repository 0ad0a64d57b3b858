#!/bin/bash
# A/B of the wave BP staging depth (2 vs 1 shots ahead):
# SSF parity tests, then interleaved benches of both libraries.
set -eo pipefail
O=gpurun_out/${1:-ii}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_harness.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "ssf or lean or zero or occupancy or hybrid or fold or bp_parity or edge or irregular or timing or empty" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
for v in "" _d1; do
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sample-phase --variant none --no-large-code --steps 4 > $O/bench$v$r.json 2> $O/bench$v$r.err
python - $O/bench$v$r.json "lib$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "value %.2f M/s  ms/step %.2f" % (d["value"] / 1e6, d["ms_per_step"]), "bp iso", [round(v["bp_kernel_ms_isolated"], 3) for v in d["ler"].values()], "sum %.2f" % sum(v["bp_kernel_ms_isolated"] for v in d["ler"].values()))
PY
done
done
