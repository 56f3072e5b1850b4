# round 4, second GPU call: the whole GPU suite (decision-table path test, dense-prox demo case), the isotropic
# merge crossover (c5 iso, batch 8 / 16 / 32, one grid vs per-branch streams), resident 250^2 variants and
# the resident kernel's rocprof + PMC traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 800 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for b in 8 16 32; do for m in "--merge-iso" "--no-merge"; do
  timeout -k 10 240 python bench.py --config c5 --iso --batch $b $m --no-cpu-baseline >> gpurun_out/r04b_c5iso.jsonl 2>> gpurun_out/r04b_c5.err || exit $?
done; done
echo "== base" > gpurun_out/r04b_resvar.log
timeout -k 10 120 python -u tools/time_resident.py --time-only 250,250,256 >> gpurun_out/r04b_resvar.log 2>&1 || exit $?
bash tools/run_resident_variants.sh ncc2 pd2 pd4 u16 ncc2pd4 >> gpurun_out/r04b_resvar.log 2>&1 || exit $?
bash tools/prof_resident.sh r04 250,250,256 || exit $?
echo all-done
