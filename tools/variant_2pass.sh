#!/bin/bash
# On the GPU box: a 2-pass configuration (CONFIG, default c4) for the in-tree library and variant
# libraries (libadmm_deconv_<TAG>.so) under the line-tile option LINE_T (LINE_TS, default "8 4").
# usage: CONFIG=c2 bash tools/variant_2pass.sh TAG...
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/base_lib.so
for v in base "$@"; do
  if [ $v != base ]; then cp admm-deconv_amd/libadmm_deconv_$v.so $L; fi
  for t in ${LINE_TS:-8 4}; do
    echo "== $v LINE_T=$t"
    timeout -k 10 200 python bench.py --opt LINE_T=$t --config ${CONFIG:-c4} --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/v2p.json || break
    python -c "
import json; d=json.load(open('gpurun_out/v2p.json')); print(d['value'], d['ms_per_step'], {k: (round(v['avg_ms'], 3), round(v.get('achieved_GBps', 0))) for k, v in d['kernels'].items()})"
  done
done
cp /tmp/base_lib.so $L
