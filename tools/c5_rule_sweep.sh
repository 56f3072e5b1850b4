#!/bin/bash
# c5 training step around the multi-branch plane-count rule: batch 4 / 8 / 16 (60 / 120 / 240 planes in one grid),
# the default rule against the 2-pass kernels forced (MIN_PLANES huge) and the per-plane kernels forced (0).
# usage (GPU box): bash tools/c5_rule_sweep.sh TAG
set -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
O=gpurun_out/${TAG}_c5rule.jsonl
for iso in "--iso" ""; do
  for b in 4 8 16; do
    for mp in -1 0 100000; do
      line=$(timeout -k 10 200 python bench.py --no-cpu-baseline --config c5 $iso --batch $b --steps 10 --warmup 3 --opt MIN_PLANES=$mp) || { echo "rc=$? $iso $b $mp"; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); print(json.dumps({'iso': '$iso'=='--iso', 'batch': $b, 'MIN_PLANES': $mp, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'workload': d['config']['workload']}))" "$line" | tee -a $O
    done
  done
done
