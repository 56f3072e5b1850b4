# round 4, third GPU call: resident power-of-two squares and the isotropic resident solve (parity + timing vs
# the 2-pass kernels), the lock-step question (250^2 resident at 128..1024 planes), small batches fused vs 2-pass,
# the c5 aniso reverse sweep with its first wave's odd workgroups started late
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_paths.py tests/test_gpu_dist_aniso.py tests/test_gpu_dist_iso.py tests/test_gpu_parity.py -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/time_resident.py --time-only 128,128,256 64,64,1024 32,32,2048 250,250,128 250,250,512 250,250,1024 > gpurun_out/r04c_res.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/time_resident.py --iso --time-only 250,250,64 128,128,192 96,96,256 32,32,512 > gpurun_out/r04c_resiso.log 2>&1 || exit $?
for b in 2 8 32 128; do for o in "" "--opt FUSED=0"; do
  timeout -k 10 120 python bench.py --config c2 --batch $b --no-cpu-baseline --steps 20 $o >> gpurun_out/r04c_small.jsonl 2>> gpurun_out/r04c.err || exit $?
done; done
for a in "--iso --batch 2 --opt FUSED=0" "--batch 2 --opt FUSED=0" "--batch 2"; do
  timeout -k 10 240 python bench.py --config c5 $a --no-cpu-baseline >> gpurun_out/r04c_c5.jsonl 2>> gpurun_out/r04c.err || exit $?
done
for st in 0 1000 2000 3500; do
  timeout -k 10 240 python bench.py --config c5 --no-cpu-baseline --opt PLANE_STAGGER=$st >> gpurun_out/r04c_c5stagger.jsonl 2>> gpurun_out/r04c.err || exit $?
done
echo all-done
