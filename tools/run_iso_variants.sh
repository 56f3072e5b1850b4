#!/bin/bash
# On the GPU box: tools/time_iso.py (192 planes, K = 50) with each variant library swapped in
# (tools/build_variant.sh TAG -D...).  usage: bash tools/run_iso_variants.sh TAG...   (base = in-tree)
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/base_lib.so
for v in base "$@"; do
  if [ $v != base ]; then cp admm-deconv_amd/libadmm_deconv_$v.so $L; fi
  echo "== $v"
  timeout -k 10 120 python tools/time_iso.py 192 50 2>&1 | grep "^iso" || break
done
cp /tmp/base_lib.so $L
