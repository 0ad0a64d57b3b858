#!/bin/bash
# CPU sanitizer run (SURVEY §5 "Race detection / sanitizers"): the CPU oracle
# (oracle/qdec_oracle.c) and the host C++ of libqdec_hip.so (ABI, graph layout
# and anneal, host OSD, GF(2) elimination, launchers) built with
# -fsanitize=address,undefined (host code only: -Xarch_host), then the whole
# CPU test suite (pytest -m "not gpu") under clang's ASan runtime.
# Usage: tools/sanitize.sh [log]   (CPU only; no GPU is touched)
set -eo pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r04_sanitizer_cpu.log}
LLVM=/opt/rocm/lib/llvm
RT=$(ls $LLVM/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
make -C oracle SAN=1 CC=$LLVM/bin/clang -s -B
python -m exp_ldpc_amd.build --san --tag san > /dev/null
export QDEC_LIB=$PWD/exp_ldpc_amd/libqdec_hip_san.so
export QDEC_ORACLE_LIB=$PWD/oracle/libqdec_oracle_san.so
# leaks: CPython and torch keep allocations to exit by design; every other
# ASan / UBSan finding aborts the run
export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
{
  echo "# tools/sanitize.sh  $(date -u +%FT%TZ)  runtime=$RT"
  echo "# QDEC_LIB=$QDEC_LIB QDEC_ORACLE_LIB=$QDEC_ORACLE_LIB"
  LD_PRELOAD=$RT python -m pytest tests -m "not gpu" -q -p no:cacheprovider 2>&1
} | tee "$LOG"
