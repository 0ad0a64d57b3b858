#!/bin/bash
# Round 4, session j: phase stamps of the compact BP kernel (f64, f32).
set -eo pipefail
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/dev/stamps_cmp.py 0.001 0.0032 0.01 0.1 > $O/stamps_f64.log 2>&1 || { tail -20 $O/stamps_f64.log; exit 1; }
grep "^p=" $O/stamps_f64.log
STAMP_PREC=f32 timeout -k 10 300 python tools/dev/stamps_cmp.py 0.001 0.1 > $O/stamps_f32.log 2>&1 || { tail -20 $O/stamps_f32.log; exit 1; }
grep "^p=" $O/stamps_f32.log
