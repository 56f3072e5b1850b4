#!/bin/bash
# line tile height A/B at c4 (M = 512): T = 8 (default), 4, 2
set -o pipefail
mkdir -p gpurun_out
for t in 8 4 2; do
  timeout -k 10 300 python bench.py --opt LINE_T=$t --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lt_c4_$t.json 2>/dev/null || exit 1
done
for f in gpurun_out/lt_*.json; do python - "$f" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = d["kernels"]
print(sys.argv[1], d["value"], {n: round(v.get("total_ms_per_solve", v.get("total_ms_per_step", 0)), 2) for n, v in k.items()})
PY
done
