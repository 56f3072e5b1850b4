#!/bin/bash
# Build libadmm_deconv_<TAG>.so with extra flags on the admm_smooth.hip translation unit (compile-time-plan
# kernels; experiments, swapped in on the GPU box by tools/gen_variants.sh).
# usage: tools/build_smooth_variant.sh TAG -DFOO=1 ...
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/admm-deconv_amd/csrc
O=/tmp/svariant_$TAG
mkdir -p $O
python3 -c "
import sys; sys.path.insert(0, '$C'); import hazard_pad
hazard_pad.compile_tu('$C/admm_smooth.hip', '$O/admm_smooth.o',
    ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC'] + sys.argv[1:])" "$@"
hipcc --offload-arch=gfx950 -fPIC -shared -o $R/admm-deconv_amd/libadmm_deconv_$TAG.so $C/admm_capi.o $C/plane_launch.o $O/admm_smooth.o $C/metrics_capi.o
echo built $TAG
