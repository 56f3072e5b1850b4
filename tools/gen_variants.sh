#!/bin/bash
# On the GPU box: runtime-length path timings for the in-tree library and variant libraries
# (tools/build_capi_variant.sh).  usage: bash tools/gen_variants.sh TAG...   (base = in-tree)
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/base_lib.so
for v in base "$@"; do
  if [ $v != base ]; then cp admm-deconv_amd/libadmm_deconv_$v.so $L; fi
  echo "== $v"
  timeout -k 10 150 python tools/time_generic.py ${GEN_OPTS:-} 480,640,64 96,96,512 250,250,256 2048,2048,8 2>&1 | grep shape | cut -c1-200 || break
done
cp /tmp/base_lib.so $L
