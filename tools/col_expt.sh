#!/bin/bash
# column block size A/B: c4 (N = 512) and c5 (N = 256) with 256 vs 1024 threads per column block
set -o pipefail
mkdir -p gpurun_out
for nt in 256 1024; do
  timeout -k 10 300 python bench.py --opt COL_THREADS=$nt --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/col_c4_$nt.json 2>/dev/null || exit 1
  timeout -k 10 300 python bench.py --opt COL_THREADS=$nt --config c5 --steps 3 --warmup 1 > gpurun_out/col_c5_$nt.json 2>/dev/null || exit 1
done
for f in gpurun_out/col_*.json; do python - "$f" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = d["kernels"]
print(sys.argv[1], d["value"], {n: round(v.get("total_ms_per_solve", v.get("total_ms_per_step", 0)), 2) for n, v in k.items()})
PY
done
