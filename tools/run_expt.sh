cp admm-deconv_amd/libadmm_devtest.so /tmp/base.so
for v in NOSTORE NOLOAD; do
  cp admm-deconv_amd/libadmm_devtest_$v.so admm-deconv_amd/libadmm_devtest.so
  echo "== $v"; timeout -k 10 100 python tools/plane_timing.py 512 2>&1 | grep -v amdgpu.ids | tail -7
done
cp /tmp/base.so admm-deconv_amd/libadmm_devtest.so
