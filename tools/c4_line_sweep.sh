#!/bin/bash
# c4 (512^2 x 3, K = 50) line-update block shape sweep (ADMM_EXP_LINE512 = "T,threads"), two rounds, one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
O=gpurun_out/${1:-c4line}.jsonl
for rep in 1 2; do
  for v in default 8,512 16,1024 4,512 8,1024; do
    if [ $v = default ]; then unset ADMM_EXP_LINE512; else export ADMM_EXP_LINE512=$v; fi
    line=$(timeout -k 10 240 python bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 2) || { echo "rc=$? ($v)"; exit 1; }
    echo "{\"variant\": \"$v\", \"rep\": $rep, \"line\": $line}" >> $O
    python -c "import json,sys; d=json.loads(sys.argv[1]); print('$v', d['value'], d['kernels']['line']['avg_ms'])" "$line"
  done
done
