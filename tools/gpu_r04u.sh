# round 4, twenty-first and -second GPU calls: the setup kernel's PSF spectrum without per-term integer divisions, then with the PSF staged in LDS
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plane.py tests/test_gpu_backward.py tests/test_gpu_smooth.py -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04u_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04u -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04u_bench.jsonl 2> gpurun_out/r04u_bench.err || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r04u_bench_plain.jsonl 2>> gpurun_out/r04u_bench.err || exit $?
echo all-done
