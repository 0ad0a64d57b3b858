#!/bin/bash
# Dev: build a stamped library variant with extra -D flags, e.g.
#   bash tools/dev/build_variant.sh nosplit -DQDEC_SSF_NOSPLIT
# -> exp_ldpc_amd/libqdec_hip_stamps_nosplit.so (load with QDEC_LIB=...).
set -eo pipefail
tag=$1; shift
cd "$(dirname "$0")/../../exp_ldpc_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -pthread -DQDEC_STAMPS "$@" \
  -o ../libqdec_hip_stamps_$tag.so qdec_abi.cpp qdec_osd.cpp qdec_gf2.cpp qdec_bp.hip qdec_bp_block.hip \
  qdec_sample.hip qdec_osd.hip
