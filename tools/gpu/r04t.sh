#!/bin/bash
# Round 4, session t (final evidence): GPU suite, smoke, default bench, the multi-rank bench path
# rehearsed with 2 ranks on the box's one GPU (gloo bookkeeping group, real
# HIP decode), rocprof kernel trace + stats of the bench.
set -eo pipefail
O=gpurun_out/r04t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("f64 %.2f M/s  f32 %.2f M/s" % (d["value"] / 1e6, d["variants"][0]["value"] / 1e6), "kernel", r["kernel"],
      "lds frac %.3f hbm frac %.4f" % (r["frac"], r["hbm"]["frac"]), "ceilings", r.get("ceilings", {}).get("kernel"))
print("bp", [round(x["bp_kernel_ms_isolated"], 3) for x in d["ler"].values()],
      "ssf", [round(x["ssf_kernel_ms_isolated"], 3) for x in d["ler"].values()])
PY
timeout -k 10 400 python bench.py --gpus 2 --steps 3 --no-cpu-baseline --no-large-code --no-sample-phase > $O/bench_2ranks.json 2> $O/bench_2ranks.err || { tail -30 $O/bench_2ranks.err; exit 1; }
python -c "import json,sys; d=json.load(open('$O/bench_2ranks.json')); print('2 ranks on 1 GPU:', d['n_gpus'], '%.2f M/s' % (d['value']/1e6), d['config']['parallelism'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/prof_bench.json 2> $O/prof.err
python tools/rocprof_phases.py $O/prof/run_kernel_trace.csv $O/prof_bench.json $O/rocprof_phases.json
echo done
