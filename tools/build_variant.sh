#!/bin/bash
# Build libadmm_deconv_<TAG>.so with extra flags on the fused-kernel translation unit (experiments;
# tools/run_variants.sh swaps them in on the GPU box).  The device assembly goes through the same
# hazard-padding pass as the product build (csrc/hazard_pad.py); NOPAD=1 skips it, PK=1 keeps packed FP32.
# usage: [PK=1] [NOPAD=1] tools/build_variant.sh TAG -DFOO=1 ...
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/admm-deconv_amd/csrc
O=/tmp/variant_$TAG
mkdir -p $O
NOPK="-Xclang -target-feature -Xclang -packed-fp32-ops"; [ "${PK:-0}" = 1 ] && NOPK=""
if [ "${NOPAD:-0}" = 1 ]; then
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c $NOPK -mllvm -pragma-unroll-threshold=100000 "$@" \
    -o $O/plane_launch.o $C/plane_launch.hip 2>&1 | grep -v "not a recognized feature" || true
else
  python3 -c "
import sys; sys.path.insert(0, '$C'); import hazard_pad
n = hazard_pad.compile_tu('$C/plane_launch.hip', '$O/plane_launch.o',
    ['--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC'] + '$NOPK'.split() + ['-mllvm', '-pragma-unroll-threshold=100000'] + sys.argv[1:])
print('hazard pads', n)" "$@"
fi
hipcc --offload-arch=gfx950 -fPIC -shared -o $R/admm-deconv_amd/libadmm_deconv_$TAG.so $C/admm_capi.o $O/plane_launch.o $C/admm_smooth.o $C/metrics_capi.o
echo built $TAG
