cp admm-deconv_amd/libadmm_deconv.so /tmp/base_lib.so
for v in PD3; do
  cp admm-deconv_amd/libadmm_deconv_$v.so admm-deconv_amd/libadmm_deconv.so
  echo "== $v"; timeout -k 10 200 python tools/census_plane.py 3 2>&1 | cat
  timeout -k 10 200 python -m pytest tests/test_gpu_plane.py -q 2>&1 | tail -1
  timeout -k 10 100 python tools/time_plane.py 512 2>&1 | grep "fused=1" | cut -c1-45
done
cp /tmp/base_lib.so admm-deconv_amd/libadmm_deconv.so
