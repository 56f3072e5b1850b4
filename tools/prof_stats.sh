#!/bin/bash
# On the GPU box: rocprofv3 kernel stats of tools/time_generic.py on the given shapes (N,M,B ...), one summary per shape.
# usage: tools/prof_stats.sh TAG N,M,B [N,M,B ...]
set -euo pipefail
TAG=$1; shift
export TMPDIR=/tmp
for SHAPE in "$@"; do
  OUT=gpurun_out/stats_${TAG}_${SHAPE//,/x}
  mkdir -p $OUT
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python tools/time_generic.py $SHAPE > $OUT/log 2>&1
  f=$(find $OUT -name '*kernel_stats.csv' | head -1)
  echo "== $SHAPE"; cut -d, -f1-4 "$f" | sed -E 's/\(.*\)"/"/' | head -12
done
