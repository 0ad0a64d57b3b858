#!/bin/bash
# Round 4, session w: PMC passes (final kernels) of the default bench (tools/pmc.sh, the
# headline's f64 phases + isolated launches) for the roofline's ceilings.
set -eo pipefail
O=gpurun_out/r04w
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 bash tools/pmc.sh $O/pmc --no-cpu-baseline --no-sample-phase --variant none > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
tail -3 $O/pmc.log
