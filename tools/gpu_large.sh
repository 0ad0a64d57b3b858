set -eo pipefail
O=gpurun_out/large1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_codes.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python -u tools/bench_configs.py c3 c4 c5 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cat $O/configs.jsonl
