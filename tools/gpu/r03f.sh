#!/bin/bash
# Round 3 checkpoint: full GPU suite, smoke, default bench (f64 headline, f32
# variant, CPU f64/f32 baselines, config-5 HBM line), rocprof kernel stats of
# the bench, and FETCH/WRITE PMC passes of the config-5 slot-group kernel.
set -eo pipefail
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value %.2f M/s %s  ms/step %.2f  variants %s" % (d["value"] / 1e6, d["dtype"], d["ms_per_step"],
      [(v["dtype"], round(v["value"] / 1e6, 2)) for v in d.get("variants", [])]))
print("cpu", d.get("cpu_baseline", {}).get("value"), [v["value"] for v in d.get("cpu_baseline", {}).get("variants", [])])
print("large", json.dumps(d.get("large_code_roofline"))[:600])
PY
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
echo prof done
mkdir -p $R/$O/pmc_c5
i=0
for CTRS in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $CTRS -d "$R/$O/pmc_c5/pass$i" -o run --output-format csv -- python3 tools/bench_configs.py c5 --precision f64 --shots 65536 --batch 65536 --reps 1 --p 0.005 > "$R/$O/pmc_c5/pass$i.log" 2>&1
  echo "pmc pass $i done"
done
python3 tools/pmc_summary.py "$R/$O/pmc_c5" "$R/$O/pmc_c5/summary.json"
python - $O/pmc_c5/summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for name, k in d["kernels"].items():
    if "group" in name:
        print(name[:70], k.get("dispatches"), {kk: k["derived"].get(kk) for kk in ("hbm_read_bytes_per_dispatch", "hbm_write_bytes_per_dispatch", "duration_ms", "hbm_frac")})
PY
