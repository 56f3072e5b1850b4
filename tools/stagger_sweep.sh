#!/bin/bash
# On the GPU box: fused solve time under the odd-workgroup start delay option (PLANE_STAGGER, 10 ns ticks).
# usage: BATCHES="256 512" bash tools/stagger_sweep.sh 0 1500 3000 ...
for b in ${BATCHES:-512}; do
  for st in "$@"; do
    echo "== batch $b stagger $st"
    timeout -k 10 120 python tools/time_plane.py $b PLANE_STAGGER=$st 2>&1 | grep "fused=1" | cut -c1-50 || exit 1
  done
done
