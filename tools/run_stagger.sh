for v in 0 1500 3000 6000; do echo "== stagger $v"; timeout -k 10 120 python tools/time_plane.py PLANE_STAGGER=$v 512 2>&1 | grep "fused=1" | cut -c1-60; done
