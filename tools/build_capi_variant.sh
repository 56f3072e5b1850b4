#!/bin/bash
# Build libadmm_deconv_<TAG>.so with extra flags on the admm_capi.hip translation unit (2-pass and
# runtime-length kernels; experiments, swapped in on the GPU box like tools/build_variant.sh's).
# usage: tools/build_capi_variant.sh TAG -DFOO=1 ...
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/admm-deconv_amd/csrc
O=/tmp/cvariant_$TAG
mkdir -p $O
python3 -c "
import sys; sys.path.insert(0, '$C'); import hazard_pad
hazard_pad.compile_tu('$C/admm_capi.hip', '$O/admm_capi.o',
    ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-Wno-unused-result', '-Wno-unused-value'] + sys.argv[1:])" "$@"
hipcc --offload-arch=gfx950 -fPIC -shared -o $R/admm-deconv_amd/libadmm_deconv_$TAG.so $O/admm_capi.o $C/plane_launch.o $C/admm_smooth.o $C/metrics_capi.o
echo built $TAG
