#!/bin/bash
set -eo pipefail
CHECK=1 QDEC_LDS_KERNEL=1 timeout -k 5 60 python tools/dev/lds_probe.py 64 20 0 rand
bash tools/gpu_lds.sh
