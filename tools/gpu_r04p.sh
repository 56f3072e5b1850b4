# round 4, sixteenth GPU call: the resident solve with 1024-thread workgroups (16 waves, 4 per SIMD) against 512
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/lib_cur.so
SH="250,250,256 240,240,256 200,200,256 192,192,256 160,160,256 128,128,256 120,120,256 96,96,512 64,64,1024 32,32,2048"
timeout -k 10 300 python -u tools/time_resident.py --time-only $SH > gpurun_out/r04p_base.log 2>&1 || exit $?
cp admm-deconv_amd/libadmm_deconv_nt1024.so $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04p_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then cp /tmp/lib_cur.so $L; exit $rc; fi
timeout -k 10 400 python -u tools/time_resident.py $SH > gpurun_out/r04p_nt1024.log 2>&1
rc=$?
cp /tmp/lib_cur.so $L
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/time_resident.py --iso --time-only 250,250,256 200,200,256 160,160,256 120,120,256 96,96,256 > gpurun_out/r04p_isobase.log 2>&1 || exit $?
cp admm-deconv_amd/libadmm_deconv_nt1024.so $L
timeout -k 10 300 python -u tools/time_resident.py --iso --time-only 250,250,256 200,200,256 160,160,256 120,120,256 96,96,256 > gpurun_out/r04p_iso1024.log 2>&1
rc=$?
cp /tmp/lib_cur.so $L
[ $rc -eq 0 ] || exit $rc
echo all-done
