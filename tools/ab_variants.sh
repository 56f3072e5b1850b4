#!/bin/bash
# A/B/C... timing of library variants on one box: tools/ab/lib_NAME.so for each NAME ("tree" = the in-tree build),
# each bench argument set run twice per variant in turn.
# usage: bash tools/ab_variants.sh TAG "NAME1 NAME2 ..." "bench args" ["bench args" ...]
set -o pipefail
TAG=$1; NAMES=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
O=gpurun_out/${TAG}_abv.jsonl
for a in "$@"; do
  for rep in 1 2; do
    for v in $NAMES; do
      if [ $v = tree ]; then unset ADMM_LIB_PATH; else export ADMM_LIB_PATH=$PWD/tools/ab/lib_$v.so; fi
      line=$(timeout -k 10 240 python bench.py --no-cpu-baseline $a) || { echo "rc=$? ($v: $a)"; exit 1; }
      echo "{\"build\": \"$v\", \"args\": \"$a\", \"rep\": $rep, \"line\": $line}" >> $O
      python -c "import json,sys; d=json.loads(sys.argv[1]); print('$v', '$a', d['value'], d['ms_per_step'])" "$line"
    done
  done
done
