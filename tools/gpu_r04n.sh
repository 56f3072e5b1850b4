# round 4, fourteenth GPU call: the smooth 2-pass update's elementwise phase on pixel pairs -- parity and time
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_smooth.py tests/test_gpu_paths.py tests/test_gpu_parity.py tests/test_gpu_resident.py -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04n_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/time_generic.py 480,640,64 640,480,64 250,250,256 RESIDENT=0 > gpurun_out/r04n_gen.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/time_generic.py 1000,1000,16 2000,2000,4 300,400,128 > gpurun_out/r04n_gen2.log 2>&1 || exit $?
echo all-done
