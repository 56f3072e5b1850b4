# round 4, thirteenth GPU call: H^T y folded into the resident solve's spectrum, LDS-only barriers -- parity, time
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_paths.py tests/test_gpu_backward.py tests/test_gpu_parity.py -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04m_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SH="250,250,256 240,240,256 200,200,256 192,192,256 160,160,256 128,128,256 120,120,256 96,96,512 64,64,1024 32,32,2048 250,250,128"
timeout -k 10 300 python -u tools/time_resident.py $SH > gpurun_out/r04m_res.log 2>&1 || exit $?
SHAPES="$SH" timeout -k 10 300 bash tools/run_resident_variants.sh fullbar > gpurun_out/r04m_fullbar.log 2>&1 || exit $?
echo all-done
