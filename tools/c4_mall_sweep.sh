#!/bin/bash
# c4 bench at several ADMM_OPT_MALL_STREAMS values (chunk = 224 MiB / (28 B/px x n)).  usage: tools/c4_mall_sweep.sh TAG "1 2 4 6 8"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export PYTHONUNBUFFERED=1
TAG=$1; mkdir -p gpurun_out
for n in $2; do
  timeout -k 10 200 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --opt MALL_STREAMS=$n > gpurun_out/${TAG}_n$n.jsonl 2>/dev/null || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['schedule'])" gpurun_out/${TAG}_n$n.jsonl $n
done
