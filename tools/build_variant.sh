#!/bin/bash
# Build libadmm_deconv_<TAG>.so with extra -D flags on the fused-kernel translation unit (experiments;
# tools/run_variants.sh swaps them in on the GPU box).  usage: tools/build_variant.sh TAG -DFOO=1 ...
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/admm-deconv_amd/csrc
O=/tmp/variant_$TAG
mkdir -p $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Xclang -target-feature -Xclang -packed-fp32-ops -mllvm -pragma-unroll-threshold=100000 "$@" \
  -o $O/plane_launch.o $C/plane_launch.hip 2>&1 | grep -v "not a recognized feature" || true
hipcc --offload-arch=gfx950 -fPIC -shared -o $R/admm-deconv_amd/libadmm_deconv_$TAG.so $C/admm_capi.o $O/plane_launch.o $C/metrics_capi.o
echo built $TAG
