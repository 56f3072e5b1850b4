for st in 0 2000 4000 6000; do
  echo "stagger=$st"; ADMM_PLANE_STAGGER=$st timeout -k 10 100 python tools/time_plane.py 512 2>&1 | grep "fused=1"
done
