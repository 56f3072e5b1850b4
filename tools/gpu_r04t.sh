# round 4, twentieth GPU call: the isotropic resident A / B phases without look-ahead past a wave's rows
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_dist_iso.py -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04t_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/lib_cur.so
SH="250,250,256 200,200,256 160,160,256 120,120,256 96,96,256"
for round in 1 2; do
  for v in cur prevld; do
    if [ $v = cur ]; then cp /tmp/lib_cur.so $L; else cp admm-deconv_amd/libadmm_deconv_prevld.so $L; fi
    echo "== $v"
    timeout -k 10 200 python -u tools/time_resident.py --iso --time-only $SH || { cp /tmp/lib_cur.so $L; exit 1; }
  done
done > gpurun_out/r04t_ab.log 2>&1
cp /tmp/lib_cur.so $L
echo all-done
