# round 4, last GPU call: the whole GPU suite, smoke, the default bench line, and the resident shapes (aniso + iso)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04w_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04w_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r04w_bench.jsonl 2> gpurun_out/r04w_bench.err || exit $?
SH="250,250,256 240,240,256 200,200,256 192,192,256 160,160,256 128,128,256 120,120,256 96,96,512 64,64,1024 32,32,2048"
timeout -k 10 400 python -u tools/time_resident.py $SH > gpurun_out/r04w_res.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/time_resident.py --iso --time-only 250,250,256 200,200,256 160,160,256 120,120,256 96,96,256 > gpurun_out/r04w_resiso.log 2>&1 || exit $?
echo all-done
