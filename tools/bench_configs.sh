#!/bin/bash
# One bench line per BASELINE configuration the single GPU runs (c1 .. c5, c5 isotropic, the training batch of 2),
# appended to gpurun_out/TAG_configs.jsonl -- the round's record of every config on one box.
# usage (GPU box): bash tools/bench_configs.sh TAG
set -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
O=gpurun_out/${TAG}_configs.jsonl
for a in "--config c1 --steps 50" "--steps 20" "--config c4 --steps 5 --warmup 2" "--config c5 --steps 5 --warmup 2" \
         "--config c5 --iso --steps 5 --warmup 2" "--config c5 --iso --batch 2 --steps 20" "--config c5 --batch 2 --steps 20"; do
  echo "== $a"
  timeout -k 10 300 python bench.py --no-cpu-baseline $a >> $O 2>> gpurun_out/${TAG}_configs.err || { echo "rc=$? ($a)"; exit 1; }
  tail -1 $O | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['unit'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'))"
done
