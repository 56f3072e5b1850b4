#!/bin/bash
# On the GPU box: c5 iso train step (serial branches, per-kernel classes) under the tile knobs.
for cfg in "256 8" "1024 8" "256 4" "256 16" "1024 4"; do
  set -- $cfg
  echo "== COL_THREADS=$1 LINE_T=$2"
  timeout -k 10 200 python bench.py --opt COL_THREADS=$1 --opt LINE_T=$2 --config c5 --iso --serial-branches --steps 2 --warmup 1 > gpurun_out/iso_k.json || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/iso_k.json')); print(d['value'], d['ms_per_step'], {k: round(v['total_ms_per_step'], 2) for k, v in d['kernels'].items()})"
done
