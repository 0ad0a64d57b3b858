#!/bin/bash
# A/B: the library built without the AMDGPU atomic optimizer (its rewrite of the
# lane-0 counter atomics waits for the returned value at once, vmcnt(0)).
set -eo pipefail
O=gpurun_out/${1:-nao}; mkdir -p $O
export TMPDIR=/tmp
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_nao.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_nao.log 2>&1 || { tail -30 $O/gpu_tests_nao.log; exit 1; }
echo "nao suite: $(tail -1 $O/gpu_tests_nao.log)"
for r in 1 2; do
for v in "" _nao; do
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sample-phase --variant none --no-large-code --steps 4 > $O/bench$v$r.json 2> $O/bench$v$r.err
python - $O/bench$v$r.json "lib$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
L = d["ler"].values()
print(sys.argv[2], "value %.2f M/s  ms/step %.2f" % (d["value"] / 1e6, d["ms_per_step"]),
      "bp iso", [round(v["bp_kernel_ms_isolated"], 3) for v in L], "sum %.2f" % sum(v["bp_kernel_ms_isolated"] for v in L),
      "ssf iso sum %.2f" % sum(v["ssf_kernel_ms_isolated"] for v in L))
PY
done
done
