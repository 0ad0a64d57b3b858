#!/bin/bash
# GPU OSD parity (vs the host OSD stage) and the bposd-mode throughput, device vs host OSD.
set -eo pipefail
O=gpurun_out/osd1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_harness.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python -u tools/bench_modes.py > $O/modes.jsonl 2> $O/modes.err
cut -c1-300 $O/modes.jsonl
