#!/bin/bash
# Full GPU suite on the default library, then interleaved benches of the
# default library and its A/B variants (libqdec_hip_<tag>.so), then a kernel
# timeline of the overlapped phase.  Usage: tools/dev/gpu_ab3.sh <out> <tag>...
set -eo pipefail
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
for v in "" "$@"; do
[ -n "$v" ] && v="_$v"
QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-sample-phase --variant none --no-large-code --steps 4 > $O/bench$v$r.json 2> $O/bench$v$r.err
python - $O/bench$v$r.json "lib$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
L = d["ler"].values()
print(sys.argv[2], "value %.2f M/s  ms/step %.2f" % (d["value"] / 1e6, d["ms_per_step"]),
      "bp iso", [round(v["bp_kernel_ms_isolated"], 3) for v in L], "sum %.2f" % sum(v["bp_kernel_ms_isolated"] for v in L),
      "ssf iso", [round(v["ssf_kernel_ms_isolated"], 3) for v in L], "sum %.2f" % sum(v["ssf_kernel_ms_isolated"] for v in L))
PY
done
done
bash tools/dev/gpu_timeline.sh ${O#gpurun_out/}_tl
