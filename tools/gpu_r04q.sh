# round 4, seventeenth and last GPU calls: the whole GPU suite, smoke() and the default bench line on the current build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04q_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04q_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r04q_bench.jsonl 2> gpurun_out/r04q_bench.err || exit $?
echo all-done
