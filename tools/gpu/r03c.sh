#!/bin/bash
# Round 3, third pass: large-code parity on the restructured slot-group kernel,
# config 4/5 throughput (f32 / f64), and an A/B of the wave kernel's epilogue
# changes (queue reservation, LDS-read logicals) on the default bench.
set -eo pipefail
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python -u -m pytest tests/test_gpu_large_codes.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/large.log 2>&1 || { tail -40 $O/large.log; exit 1; }
tail -2 $O/large.log
timeout -k 10 600 python -u tools/bench_configs.py c5 c5r0 c4 --shots 262144 --reps 2 --p 0.001 --p 0.005 --p 0.03 > $O/cfg.jsonl 2> $O/cfg.err || { tail -20 $O/cfg.err; exit 1; }
python - $O/cfg.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["config"], d["precision"], d["p"], "%.0f shots/s" % d["shots_per_s"], "%.0f GB/s" % d["algorithmic_GBps_bp_kernel"], "it %.1f" % d["mean_bp_iters"])
PY
for V in default noqres oldfin; do
  if [ $V = default ]; then unset QDEC_LIB; else export QDEC_LIB=$R/exp_ldpc_amd/libqdec_hip_$V.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --variant none --no-sample-phase > $O/bench_$V.json 2> $O/bench_$V.err || { tail -20 $O/bench_$V.err; exit 1; }
  python - $O/bench_$V.json $V <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "value %.2f M/s  ms/step %.2f" % (d["value"] / 1e6, d["ms_per_step"]),
      "bp", [round(v["bp_kernel_ms_isolated"], 3) for v in d["ler"].values()],
      "ssf", [round(v["ssf_kernel_ms_isolated"], 3) for v in d["ler"].values()])
PY
done
