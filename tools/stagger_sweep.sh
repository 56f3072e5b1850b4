#!/bin/bash
# On the GPU box: fused c2 solve time under the odd-workgroup start delay option (PLANE_STAGGER, 10 ns ticks).
for st in "$@"; do
  echo "== stagger $st"
  timeout -k 10 120 python tools/time_plane.py 512 PLANE_STAGGER=$st 2>&1 | grep "fused=1" | cut -c1-50 || exit 1
done
