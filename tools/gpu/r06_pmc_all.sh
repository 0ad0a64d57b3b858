#!/bin/bash
# The round-6 PMC passes alone: headline kernels (bench, reduced), C5 decoding
# and bandwidth points, C3, C4 f64.  Usage: tools/gpu/r06_pmc_all.sh <tag>
set -eo pipefail
O=gpurun_out/${1:-r06fin}
mkdir -p $O
export TMPDIR=/tmp
bash tools/pmc.sh $O/pmc_bench --no-c4 --no-large-code --no-reference-default --no-c3 --no-cpu-baseline --steps 2
PMC_HBM=1 PMC_META="c5_p=0.005 c5_shots=65536" bash tools/pmc_cmd.sh $O/pmc_c5_p005 tools/gpu/lines_only.py --c5 --c5-p 0.005 --c5-warm-full
PMC_HBM=1 PMC_META="c5_p=0.001 c5_shots=262144" bash tools/pmc_cmd.sh $O/pmc_c5_p001 tools/gpu/lines_only.py --c5 --c5-p 0.001 --shots 262144 --c5-warm-full
PMC_HBM=1 bash tools/pmc_cmd.sh $O/pmc_c3 tools/gpu/lines_only.py --c3
echo "pmc done"
