#!/bin/bash
# On the GPU box: fused-kernel solve time vs batch (working set in flight vs the 256 MiB Infinity Cache).
for b in 64 128 192 256 512; do
  echo "== B=$b"; timeout -k 10 120 python tools/time_plane.py $b 2>&1 | grep "fused=1" | cut -c1-60 || exit 1
done
