#!/bin/bash
# The MALL-resident schedule on the smooth / runtime-length 2-pass paths: each shape with ADMM_OPT_MALL_STREAMS 1 and 4
# (A/B/A).  usage: tools/mall_generic_ab.sh "480,640,64 480,640,256 2048,2048,8"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export PYTHONUNBUFFERED=1
for n in 1 4 1 4; do
  timeout -k 10 300 python tools/time_generic.py MALL_STREAMS=$n $1 || exit $?
done
