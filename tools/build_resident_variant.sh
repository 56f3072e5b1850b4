#!/bin/bash
# Build libadmm_deconv_<TAG>.so with extra flags on admm_resident.hip (timing experiments: RS_SKIP_COL,
# RS_SKIP_UPD, RS_SKIP_ROWS; swapped in on the GPU box by tools/run_resident_variants.sh).
# usage: tools/build_resident_variant.sh TAG -DFOO=1 ...
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/admm-deconv_amd/csrc
O=/tmp/rvariant_$TAG
mkdir -p $O
python3 -c "
import sys; sys.path.insert(0, '$C'); import hazard_pad
hazard_pad.compile_tu('$C/admm_resident.hip', '$O/admm_resident.o',
    ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-Xclang', '-target-feature', '-Xclang', '-packed-fp32-ops',
     '-mllvm', '-structurizecfg-skip-uniform-regions=true'] + sys.argv[1:])" "$@"
hipcc --offload-arch=gfx950 -fPIC -shared -o $R/admm-deconv_amd/libadmm_deconv_$TAG.so $C/admm_capi.o $C/plane_launch.o $C/admm_smooth.o $O/admm_resident.o $C/metrics_capi.o
echo built $TAG
