# round 4, sixth GPU call: the whole GPU suite after the isotropic resident default, and the benched configs
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04f_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/r04f_bench.jsonl 2> gpurun_out/r04f_bench.err || exit $?
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline >> gpurun_out/r04f_bench.jsonl 2>> gpurun_out/r04f_bench.err || exit $?
timeout -k 10 300 python bench.py --config c5 --iso --no-cpu-baseline >> gpurun_out/r04f_bench.jsonl 2>> gpurun_out/r04f_bench.err || exit $?
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline >> gpurun_out/r04f_bench.jsonl 2>> gpurun_out/r04f_bench.err || exit $?
echo all-done
