#!/bin/bash
# On the GPU box: time the c2 fused solve with each variant library (tools/build_variant.sh) swapped in.
# usage: bash tools/run_variants.sh TAG...   (base = the in-tree library)
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/base_lib.so
for v in base "$@"; do
  if [ $v != base ]; then cp admm-deconv_amd/libadmm_deconv_$v.so $L; fi
  echo "== $v"
  ADMM_FUSED=1 timeout -k 10 120 python tools/time_plane.py 512 2>&1 | grep "fused=1" | cut -c1-60 || break
done
cp /tmp/base_lib.so $L
