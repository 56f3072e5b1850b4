#!/bin/bash
# On the GPU box: c4 (512^2 x 3, K=50) under the line-tile option LINE_T.
for t in 8 4 2; do
  echo "== LINE_T=$t"
  timeout -k 10 200 python bench.py --opt LINE_T=$t --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4_t$t.json || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/c4_t$t.json')); print(d['value'], d['ms_per_step'], {k: (v['avg_ms'], round(v.get('achieved_GBps', 0))) for k, v in d['kernels'].items()})"
done
