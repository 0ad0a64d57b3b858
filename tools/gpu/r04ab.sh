#!/bin/bash
# Round 4, session ab: SSF phase stamps (stamps build) on the final tree, f64.
set -eo pipefail
O=gpurun_out/r04ab
mkdir -p $O
STAMP_PREC=f64 timeout -k 10 300 python tools/dev/stamps.py 0.0316 0.1 > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
grep SSF $O/stamps.log
