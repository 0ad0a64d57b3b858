#!/bin/bash
set -eo pipefail
O=gpurun_out/streams3; mkdir -p $O; export TMPDIR=/tmp
for A in "--streams 5" "--streams 5 --heavy-first" "--streams 6" "--streams 7" "--streams 4 --heavy-first" "--streams 3 --heavy-first"; do
  T=$(echo $A | tr -d ' -')
  timeout -k 10 300 python bench.py --no-cpu-baseline $A > $O/b_$T.json 2> $O/b_$T.err
  python -c "import json; d=json.load(open('$O/b_$T.json')); print('$A', round(d['value']/1e6, 2), 'M shots/s')"
done
