# round 4, eleventh GPU call: the isotropic resident A / B phases as row walkers -- parity and time
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_paths.py tests/test_gpu_dist_iso.py -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04k_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/time_resident.py --iso 250,250,256 200,200,256 160,160,256 128,128,256 120,120,256 96,96,256 64,64,512 32,32,512 > gpurun_out/r04k_resiso.log 2>&1 || exit $?
echo all-done
