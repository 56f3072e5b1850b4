for st in 0 1000 2000 3000 4000; do
  echo "stagger=$st"; ADMM_PLANE_STAGGER=$st timeout -k 10 100 python tools/time_plane.py 512 2>&1 | grep "fused=1" | cut -c1-50
done
