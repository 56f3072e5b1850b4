# round 4, first GPU call: the whole GPU suite (new prox-live assertions; resident kernel in its register-range
# layout; uniform regions left unstructured), resident vs 2-pass timings of every compiled shape, the c2
# headline profile on this build (rocprof stats + FETCH/WRITE/SQ PMC), and the c5 training configurations
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04a_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/time_resident.py 250,250,256 240,240,256 200,200,256 192,192,256 160,160,256 120,120,256 96,96,512 > gpurun_out/r04a_resident.log 2>&1 || exit $?
bash tools/profile_all.sh r04a_c2 --config c2 || exit $?
for a in "--iso --batch 2" "--iso --batch 2 --merge-iso" "--batch 2" "--iso --batch 64" "--iso --batch 64 --merge-iso" ""; do
  timeout -k 10 240 python bench.py --config c5 $a --no-cpu-baseline >> gpurun_out/r04a_c5.jsonl 2>> gpurun_out/r04a_c5.err || exit $?
done
echo all-done
