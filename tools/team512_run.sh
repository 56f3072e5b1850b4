#!/bin/bash
# round-5 experiment: team512 persistent launch, bitwise check against 2-pass, then c4 timing A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
TAG=${1:-team512}
timeout -k 10 300 python -u tools/team512_check.py > gpurun_out/${TAG}_check.log 2>&1; rc=$?
cat gpurun_out/${TAG}_check.log | tail -3
[ $rc -ne 0 ] && { echo "check rc=$rc"; exit $rc; }
for rep in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export ADMM_EXP_TEAM512=1; else unset ADMM_EXP_TEAM512; fi
    line=$(timeout -k 10 240 python bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 2) || { echo "rc=$? (team=$v)"; exit 1; }
    echo "{\"team512\": $v, \"rep\": $rep, \"line\": $line}" >> gpurun_out/${TAG}.jsonl
    python -c "import json,sys; d=json.loads(sys.argv[1]); print('team=$v', d['value'], {k: round(x['avg_ms'],3) for k,x in d['kernels'].items()})" "$line"
  done
done
