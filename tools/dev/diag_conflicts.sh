#!/bin/bash
# Dev: the f64 BP kernel with one LDS access class made conflict-free (wrong
# results; diagnostic builds libqdec_hip_diag{SCATTER,GATHER,SWRITE}.so, from
# tools/dev/patches/r06_diag_conflict_free.patch + python -m exp_ldpc_amd.build
# --tag diagX -DQDEC_DIAG_X) against
# the product build: BP time at p = 0.1 / 0.032 and the PMC conflict share.
set -eo pipefail
O=gpurun_out/${1:-r06l}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in base SCATTER GATHER SWRITE; do
    if [ $v = base ]; then L=$PWD/exp_ldpc_amd/libqdec_hip.so; else L=$PWD/exp_ldpc_amd/libqdec_hip_diag$v.so; fi
    echo "== $v $r"; QDEC_LIB=$L timeout -k 10 120 python -u tools/dev/diag_bp.py 0.1 0.032
  done
done > $O/times.log 2>&1
cat $O/times.log | grep -E "==|bp_ms"
for v in base SCATTER GATHER SWRITE; do
  if [ $v = base ]; then L=$PWD/exp_ldpc_amd/libqdec_hip.so; else L=$PWD/exp_ldpc_amd/libqdec_hip_diag$v.so; fi
  QDEC_LIB=$L bash tools/pmc_cmd.sh $O/pmc_$v tools/dev/diag_bp.py 0.1 > $O/pmc_$v.log 2>&1
  python -c "
import json; d=json.load(open('$O/pmc_$v/summary.json'))
for k,v in d['kernels'].items():
    if 'bp_ms_cmp_kernel<double' in k: print('$v', {a: round(b,4) for a,b in v['derived'].items() if isinstance(b,float)})"
done
