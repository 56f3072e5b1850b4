# round 4, fifth GPU call: the whole GPU suite on the plane-count rule build, the isotropic resident solve at a
# full wave of planes, and small batches of the small resident sides (no plane-count rule below side 128)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04e_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/time_resident.py --iso --time-only 250,250,256 200,200,256 160,160,256 120,120,256 64,64,512 > gpurun_out/r04e_resiso.log 2>&1 || exit $?
S="timeout -k 10 240 python -u tools/time_small.py"
$S --iso 250 RESIDENT=2/0 256 > gpurun_out/r04e_small.jsonl 2>> gpurun_out/r04e.err || exit $?
$S --iso 200 RESIDENT=2/0 256 >> gpurun_out/r04e_small.jsonl 2>> gpurun_out/r04e.err || exit $?
$S --iso 160 RESIDENT=2/0 256 >> gpurun_out/r04e_small.jsonl 2>> gpurun_out/r04e.err || exit $?
$S --iso 120 RESIDENT=2/0 256 >> gpurun_out/r04e_small.jsonl 2>> gpurun_out/r04e.err || exit $?
$S --iso 64 RESIDENT=2/0 256 512 >> gpurun_out/r04e_small.jsonl 2>> gpurun_out/r04e.err || exit $?
$S 96 RESIDENT=2/0 1 4 16 64 >> gpurun_out/r04e_small.jsonl 2>> gpurun_out/r04e.err || exit $?
$S 32 RESIDENT=2/0 1 6 64 >> gpurun_out/r04e_small.jsonl 2>> gpurun_out/r04e.err || exit $?
$S 64 RESIDENT=2/0 1 16 128 >> gpurun_out/r04e_small.jsonl 2>> gpurun_out/r04e.err || exit $?
$S --bwd 250 RESIDENT=2/0 64 128 192 256 >> gpurun_out/r04e_small.jsonl 2>> gpurun_out/r04e.err || exit $?
echo all-done
