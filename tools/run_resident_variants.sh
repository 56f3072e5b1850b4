#!/bin/bash
# GPU box: time each libadmm_deconv_<TAG>.so variant (timing only) with tools/time_resident.py, then restore.
cd "$(dirname "$0")/.."
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/lib_base.so
for tag in "$@"; do
  cp admm-deconv_amd/libadmm_deconv_$tag.so $L
  echo "== $tag"
  timeout -k 10 120 python -u tools/time_resident.py --time-only ${SHAPES:-250,250,256} || { cp /tmp/lib_base.so $L; exit 1; }
done
cp /tmp/lib_base.so $L
