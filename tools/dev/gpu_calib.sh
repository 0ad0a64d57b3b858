#!/bin/bash
# HBM counter calibration of the C2 f64 BP wave kernel:
# FETCH_SIZE / WRITE_SIZE passes of the default library and of the
# QDEC_CALIB_NOBP variant (same staging / output traffic, BP loop compiled out;
# built on the CPU side by: python -c "from exp_ldpc_amd import build;
# build.build(defines=['QDEC_CALIB_NOBP'], tag='calib')").  One sweep point
# (p = 0.1), 2^18 shots per launch, isolated launches only.
set -eo pipefail
O=gpurun_out/${1:-calib}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/$O
export TMPDIR=/tmp
ARGS="--p 0.1 --p 0.001 --steps 2 --warmup 1 --no-cpu-baseline --variant none --no-sample-phase --iso-steps 1 --streams 1"
for V in default calib; do
  if [ $V = calib ]; then export QDEC_LIB=$R/exp_ldpc_amd/libqdec_hip_calib.so; else unset QDEC_LIB; fi
  mkdir -p $R/$O/$V
  i=0
  for CTRS in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d "$R/$O/$V/pass$i" -o run --output-format csv -- python3 bench.py $ARGS > "$R/$O/$V/pass$i.log" 2>&1
    echo "$V pass $i done"
  done
  python3 tools/pmc_summary.py "$R/$O/$V" "$R/$O/$V/summary.json"
done
