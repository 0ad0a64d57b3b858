#!/bin/bash
# PMC passes on the shot-lane kernel (config 4, p = 0.03, one batch).
set -eo pipefail
O=gpurun_out/lane_pmc; mkdir -p $O; export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
# lane kernel auto-selected at 2^17 shots per launch
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_FLAT" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $CTRS -d "$R/$O/pass$i" -o run --output-format csv -- python3 tools/bench_configs.py c4 --p 0.03 --reps 1 --shots 131072 --batch 131072 > "$R/$O/pass$i.log" 2>&1
  echo "pass $i done"
done
python tools/pmc_summary.py $O $O/summary.json > /dev/null
python - <<'PY'
import json
d = json.load(open("gpurun_out/lane_pmc/summary.json"))
for k, v in d["kernels"].items():
    if "lane" in k or "ssf_block" in k:
        print(k[:60], v.get("dispatches"), {c: round(x) for c, x in v["counters_per_dispatch"].items()}, round(v.get("hbm_bytes_per_dispatch", 0)))
PY
