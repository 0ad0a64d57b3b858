#!/bin/bash
# A/B round: slot-group kernel 4 vs 8 waves per group (configs 5 / 4), lazy vs
# eager SSF scoring and row- vs buffer-clamped staging on the default bench;
# parity of the default library first.
set -eo pipefail
O=gpurun_out/r03e
mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_large_codes.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c5 or group or f64 or psl13 or bb144" > $O/large.log 2>&1 || { tail -40 $O/large.log; exit 1; }
tail -1 $O/large.log
for V in default eager bufclamp default eager; do
  if [ $V = default ]; then unset QDEC_LIB; else export QDEC_LIB=$R/exp_ldpc_amd/libqdec_hip_$V.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --variant none --no-sample-phase > $O/bench_$V.json 2> $O/bench_$V.err || { tail -20 $O/bench_$V.err; exit 1; }
  python - $O/bench_$V.json $V <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], "value %.2f M/s  ms/step %.2f" % (d["value"] / 1e6, d["ms_per_step"]),
      "bp", [round(v["bp_kernel_ms_isolated"], 3) for v in d["ler"].values()],
      "ssf", [round(v["ssf_kernel_ms_isolated"], 3) for v in d["ler"].values()],
      "fails", sum(v["failures"] for v in d["ler"].values()))
PY
done
for V in default gw8; do
  if [ $V = default ]; then unset QDEC_LIB; else export QDEC_LIB=$R/exp_ldpc_amd/libqdec_hip_$V.so; fi
  timeout -k 10 500 python -u tools/bench_configs.py c5 c5r0 --shots 262144 --batch 262144 --reps 1 --p 0.001 --p 0.005 > $O/cfg_$V.jsonl 2> $O/cfg_$V.err || { tail -20 $O/cfg_$V.err; exit 1; }
  timeout -k 10 300 python -u tools/bench_configs.py c4 --shots 262144 --reps 1 --p 0.005 --p 0.03 --precision f64 >> $O/cfg_$V.jsonl 2>> $O/cfg_$V.err || { tail -20 $O/cfg_$V.err; exit 1; }
  python - $O/cfg_$V.jsonl $V <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(sys.argv[2], d["config"], d["precision"], d["p"], "%.0f shots/s" % d["shots_per_s"], "%.0f GB/s" % d["algorithmic_GBps_bp_kernel"], "it %.1f" % d["mean_bp_iters"])
PY
done
