#!/bin/bash
# c4 / c5-iso benches under GPU_MAX_HW_QUEUES = 4 (HIP's default) and 8, c4 at several MALL stream counts.
# usage: tools/hwq_probe.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export PYTHONUNBUFFERED=1
TAG=$1; mkdir -p gpurun_out
for q in 4 8; do
  for n in 4 6 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --opt MALL_STREAMS=$n > gpurun_out/${TAG}_c4_q${q}_n$n.jsonl 2>/dev/null || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('c4 q', sys.argv[2], 'n', sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/${TAG}_c4_q${q}_n$n.jsonl $q $n
  done
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --config c5 --iso --steps 10 --no-cpu-baseline > gpurun_out/${TAG}_c5iso_q$q.jsonl 2>/dev/null || exit $?
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('c5iso q', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/${TAG}_c5iso_q$q.jsonl $q
done
