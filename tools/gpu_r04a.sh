# round 4, first GPU call: the whole GPU suite (new prox-live assertions), the c2 headline profile on the
# current build (rocprof stats + FETCH/WRITE/SQ PMC), the reference's training configuration (c5 iso batch 2)
# with and without the merged grid, and batch 64 for the merge choice
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/profile_all.sh r04a_c2 --config c2 || exit $?
for a in "--iso --batch 2" "--iso --batch 2 --merge-iso" "--batch 2" "--iso --batch 64" "--iso --batch 64 --merge-iso"; do
  timeout -k 10 240 python bench.py --config c5 $a --no-cpu-baseline >> gpurun_out/r04a_c5.jsonl 2>> gpurun_out/r04a_c5.err || exit $?
done
echo all-done
