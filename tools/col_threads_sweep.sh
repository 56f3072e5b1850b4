#!/bin/bash
# column-pass block width sweep (ADMM_OPT_COL_THREADS 256 / 512 / 1024) at c4 (N = 512) and the c2 2-pass path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-colthreads}.jsonl
for rep in 1 2; do
  for cfg in "--config c4 --steps 5 --warmup 2" "--opt FUSED=0 --steps 10"; do
    for ct in 0 256 512 1024; do
      line=$(timeout -k 10 240 python bench.py --no-cpu-baseline $cfg --opt COL_THREADS=$ct) || { echo "rc=$?"; exit 1; }
      echo "{\"col_threads\": $ct, \"cfg\": \"$cfg\", \"rep\": $rep, \"line\": $line}" >> $O
      python -c "import json,sys; d=json.loads(sys.argv[1]); print('$cfg'[:12], $ct, d['value'], round(d['kernels']['column']['avg_ms'],4))" "$line"
    done
  done
done
