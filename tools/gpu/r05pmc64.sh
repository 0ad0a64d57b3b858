#!/bin/bash
# Round 5: PMC passes over the C4 f64 line (bp_ms_lds64_kernel) and the f32 one.
set -eo pipefail
O=gpurun_out/${1:-r05pmc64}
mkdir -p $O
timeout -k 10 600 bash tools/pmc_cmd.sh $O/f64 tools/gpu/c4_only.py --prec f64 --p 0.01 --shots 131072 > $O/f64.log 2>&1 || { tail -20 $O/f64.log; exit 1; }
tail -2 $O/f64.log
python3 -c "
import json; d=json.load(open('$O/f64/summary.json'))['kernels']
for k,v in d.items():
    if 'lds64' in k: print(k[:60], v['dispatches'], json.dumps(v['derived']))
"
