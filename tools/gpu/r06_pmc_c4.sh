#!/bin/bash
# PMC of the f64 C4 kernel (LDS busy, conflict ratio) on this tree.
set -eo pipefail
TAG=${1:-r06e}
bash tools/pmc_cmd.sh gpurun_out/$TAG/pmc_c4 tools/gpu/c4_only.py --prec f64 --p 0.01 --shots 131072
