#!/bin/bash
set -eo pipefail
CHECK=1 QDEC_LDS_KERNEL=1 timeout -k 5 60 python tools/dev/lds_probe.py 1 1 0 rand
CHECK=1 QDEC_LDS_KERNEL=1 timeout -k 5 30 python tools/dev/lds_probe.py 64 20 0 rand
CHECK=1 timeout -k 5 30 python tools/dev/lds_probe.py 1 1 0 c4
bash tools/gpu_lds.sh
