#!/bin/bash
# Round 3, second pass: full wave-kernel parity (queue reservation, LDS-read
# logicals), the default bench, slot-group step-width A/B on config 5, HBM
# calibration passes of the C2 BP kernel.
set -eo pipefail
O=gpurun_out/r03b
mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -40 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value %.2f M/s %s  ms/step %.2f  variants %s" % (d["value"] / 1e6, d["dtype"], d["ms_per_step"],
      [(v["dtype"], round(v["value"] / 1e6, 2)) for v in d.get("variants", [])]))
print("bp iso ms", [round(v["bp_kernel_ms_isolated"], 3) for v in d["ler"].values()])
print("ssf iso ms", [round(v["ssf_kernel_ms_isolated"], 3) for v in d["ler"].values()])
print("cpu", d.get("cpu_baseline", {}).get("value"), [v["value"] for v in d.get("cpu_baseline", {}).get("variants", [])])
PY
for V in default uc4uv4 uc8uv8; do
  if [ $V = default ]; then unset QDEC_LIB; else export QDEC_LIB=$R/exp_ldpc_amd/libqdec_hip_$V.so; fi
  timeout -k 10 300 python -u tools/bench_configs.py c5 c5r0 --shots 65536 --batch 65536 --reps 1 --p 0.001 --p 0.005 > $O/grp_$V.jsonl 2> $O/grp_$V.err || { tail -20 $O/grp_$V.err; exit 1; }
  python - $O/grp_$V.jsonl $V <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(sys.argv[2], d["config"], d["precision"], d["p"], "%.0f shots/s" % d["shots_per_s"], "%.0f GB/s" % d["algorithmic_GBps_bp_kernel"])
PY
done
unset QDEC_LIB
timeout -k 10 700 bash tools/dev/gpu_calib.sh r03b/calib
python - $O/calib <<'PY'
import json, sys
for v in ("default", "calib"):
    d = json.load(open(f"{sys.argv[1]}/{v}/summary.json"))
    for name, k in d["kernels"].items():
        if "bp_ms_wave" in name or "ssf_wave" in name:
            print(v, name[:60], k.get("dispatches"), {kk: k["derived"].get(kk) for kk in ("hbm_bytes_per_dispatch", "duration_ms")})
PY
