#!/bin/bash
# A/B timing of two library builds on one box: tools/ab/lib_r05_prev.so (previous) vs the in-tree build.
# usage: bash tools/ab_bench.sh TAG "bench args" ["bench args" ...]   (each arg set run prev, new, prev, new)
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG}_ab.jsonl
for a in "$@"; do
  for rep in 1 2; do
    for v in prev new; do
      if [ $v = prev ]; then export ADMM_LIB_PATH=$PWD/tools/ab/lib_r05_prev.so; else unset ADMM_LIB_PATH; fi
      line=$(timeout -k 10 240 python bench.py --no-cpu-baseline $a) || { echo "rc=$? ($v: $a)"; exit 1; }
      echo "{\"build\": \"$v\", \"args\": \"$a\", \"rep\": $rep, \"line\": $line}" >> $O
      python -c "import json,sys; d=json.loads(sys.argv[1]); print('$v', '$a', d['value'], d['ms_per_step'])" "$line"
    done
  done
done
