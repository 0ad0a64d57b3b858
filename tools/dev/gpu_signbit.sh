#!/bin/bash
# A/B of the f64 sign-bit check pass (QDEC_MS_SIGNBIT): parity of the LEAN
# kernels, zero-row frequency, then interleaved benches of both libraries.
set -eo pipefail
O=gpurun_out/${1:-sb}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "lean or zero or occupancy or bp_ssf_parity or bp_parity" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
[ -n "$ZR" ] && timeout -k 10 300 python -u tools/dev/zero_rows.py > $O/zero_rows.log 2>&1
true
for r in 1 2; do
for v in "" _sb0; do
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sample-phase --variant none --no-large-code --steps 4 > $O/bench$v$r.json 2> $O/bench$v$r.err
python - $O/bench$v$r.json "lib$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "value %.2f M/s  ms/step %.2f" % (d["value"] / 1e6, d["ms_per_step"]), "bp iso", [round(v["bp_kernel_ms_isolated"], 3) for v in d["ler"].values()], "sum %.2f" % sum(v["bp_kernel_ms_isolated"] for v in d["ler"].values()))
PY
done
done
