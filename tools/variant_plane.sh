#!/bin/bash
# On the GPU box: fused-solve time at batch 64 / 256 / 512 (c2 shape) for the in-tree library and
# variant libraries (tools/build_variant.sh); timing only, no census.  usage: bash tools/variant_plane.sh TAG...
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/base_lib.so
for v in base "$@"; do
  if [ $v != base ]; then cp admm-deconv_amd/libadmm_deconv_$v.so $L; fi
  for b in ${BATCHES:-64 256 512}; do
    echo "== $v $b"; timeout -k 10 120 python tools/time_plane.py $b 2>&1 | grep "fused=1" | cut -c1-50 || break
  done
done
cp /tmp/base_lib.so $L
