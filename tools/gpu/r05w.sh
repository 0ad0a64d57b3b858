#!/bin/bash
# Round 5, session w: SSF table kernel at 16 (product) / 8 / 4 waves per
# workgroup, interleaved, headline phase + isolated SSF per point; then the SSF
# parity files on the 4- and 8-wave builds.
set -eo pipefail
O=gpurun_out/${1:-r05w}
mkdir -p $O
ARGS="--no-cpu-baseline --no-c4 --no-reference-default --no-large-code --no-sample-phase --variant none"
L=$PWD/exp_ldpc_amd
for r in 1 2; do
  for v in base w8 w4; do
    lib=$L/libqdec_hip.so; [ $v != base ] && lib=$L/libqdec_hip_$v.so
    QDEC_LIB=$lib timeout -k 10 300 python bench.py $ARGS > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
  done
done
for f in $O/*_[12].json; do python -c "
import json; b=json.load(open('$f')); l=b['ler']
print('$f', round(b['value']/1e6,2), round(b['ms_per_step'],2), 'ssf_iso', [round(l[k]['ssf_kernel_ms_isolated'],3) for k in list(l)[-3:]], round(sum(l[k]['ssf_kernel_ms_isolated'] for k in l),3))"; done
for v in w4 w8; do
QDEC_LIB=$L/libqdec_hip_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_compact.py > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
tail -1 $O/pytest_$v.log
done
