set -eo pipefail
O=gpurun_out/osd1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_osd.py tests/test_gpu_harness.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
