# round 4, closing GPU call: resident tests and timings after the separate isotropic prefetch depth
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_dist_iso.py tests/test_gpu_paths.py -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04x_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/time_resident.py --iso --time-only 250,250,256 200,200,256 160,160,256 120,120,256 96,96,256 > gpurun_out/r04x_resiso.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/time_resident.py --time-only 250,250,256 240,240,256 160,160,256 > gpurun_out/r04x_res.log 2>&1 || exit $?
echo all-done
