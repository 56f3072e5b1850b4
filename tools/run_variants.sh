#!/bin/bash
# On the GPU box: for each variant library (tools/build_variant.sh) swapped in: census (bitwise vs the
# 2-pass path, run-to-run), then the fused solve at batch 64 (one partial round: the uncontended
# per-CU critical path) and 512 (c2).  usage: bash tools/run_variants.sh TAG...   (base = in-tree)
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/base_lib.so
for v in base "$@"; do
  if [ $v != base ]; then cp admm-deconv_amd/libadmm_deconv_$v.so $L; fi
  echo "== $v"
  timeout -k 10 200 python tools/census_plane.py 2 2>&1 | tail -1 || break
  for b in 64 512; do
    timeout -k 10 120 python tools/time_plane.py $b 2>&1 | grep "fused=1" | cut -c1-50 || break
  done
done
cp /tmp/base_lib.so $L
