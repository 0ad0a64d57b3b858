#!/bin/bash
# Quick bench-path round plus the C4 f64 kernel round, one box.
set -eo pipefail
TAG=${1:-r06d}
bash tools/gpu/r06_quick.sh $TAG
bash tools/gpu/r06_c4.sh ${TAG}c4
