#!/bin/bash
# C5 line alone (2^18 shots at the decoding points), then the PMC of the
# p = 0.001 launch shape.
set -eo pipefail
O=gpurun_out/${1:-r06g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/gpu/lines_only.py --c5 --out $O/c5.json
PMC_HBM=1 PMC_META="c5_p=0.001 c5_shots=262144" bash tools/pmc_cmd.sh $O/pmc_c5_p001 tools/gpu/lines_only.py --c5 --c5-p 0.001 --shots 262144 --c5-warm-full
