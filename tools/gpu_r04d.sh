# round 4, fourth GPU call: resident power-of-two and isotropic resident solves against the 2-pass kernels
# (parity + time), the 250^2 resident phases (phase-skip builds at 128 / 256 planes), and the small-batch crossovers (fused vs 2-pass, resident vs 2-pass) against plane count
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r04d_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/time_resident.py 128,128,256 64,64,1024 32,32,2048 > gpurun_out/r04d_res.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/time_resident.py --iso 250,250,64 128,128,192 96,96,256 32,32,512 > gpurun_out/r04d_resiso.log 2>&1 || exit $?
S="timeout -k 10 240 python -u tools/time_small.py"
$S 256 FUSED=1/0 8 16 32 48 64 80 96 128 160 192 > gpurun_out/r04d_small.jsonl 2>> gpurun_out/r04d.err || exit $?
$S --iso 256 FUSED=1/0 8 32 64 128 192 >> gpurun_out/r04d_small.jsonl 2>> gpurun_out/r04d.err || exit $?
$S --bwd 256 FUSED=1/0 8 32 64 96 128 192 >> gpurun_out/r04d_small.jsonl 2>> gpurun_out/r04d.err || exit $?
$S 250 RESIDENT=2/0 16 32 64 96 128 192 256 >> gpurun_out/r04d_small.jsonl 2>> gpurun_out/r04d.err || exit $?
$S 128 RESIDENT=2/0 16 64 128 256 512 >> gpurun_out/r04d_small.jsonl 2>> gpurun_out/r04d.err || exit $?
timeout -k 10 120 python -u tools/time_resident.py --time-only 250,250,128 250,250,256 > gpurun_out/r04d_phases.log 2>&1 || exit $?
SHAPES="250,250,128 250,250,256" timeout -k 10 400 bash tools/run_resident_variants.sh nocol noline norows >> gpurun_out/r04d_phases.log 2>&1 || exit $?
# register-column variant (RS_RCOL=1) at the shapes it compiles without spills: parity + time against the base
cp admm-deconv_amd/libadmm_deconv.so /tmp/lib_base.so
cp admm-deconv_amd/libadmm_deconv_rcol.so admm-deconv_amd/libadmm_deconv.so
timeout -k 10 300 python -u tools/time_resident.py 200,200,256 192,192,256 160,160,256 120,120,256 96,96,512 128,128,256 64,64,1024 > gpurun_out/r04d_rcol.log 2>&1
rc=$?
cp /tmp/lib_base.so admm-deconv_amd/libadmm_deconv.so
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/time_resident.py --time-only 200,200,256 192,192,256 160,160,256 120,120,256 96,96,512 > gpurun_out/r04d_rbase.log 2>&1 || exit $?
echo all-done
