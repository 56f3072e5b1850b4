# round 4, third GPU call: small batches, fused (one plane per CU) against the 2-pass path (many blocks per
# plane): c2 shape at 2..128 planes, and the c5 training step at batch 2 (the reference's train_cfg.json)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for b in 2 8 32 64 128; do for o in "" "--opt FUSED=0"; do
  timeout -k 10 120 python bench.py --config c2 --batch $b --no-cpu-baseline --steps 20 $o >> gpurun_out/r04c_small.jsonl 2>> gpurun_out/r04c.err || exit $?
done; done
for a in "--iso --batch 2" "--iso --batch 2 --opt FUSED=0" "--batch 2" "--batch 2 --opt FUSED=0" "--iso --batch 8 --opt FUSED=0" "--batch 8 --opt FUSED=0" "--batch 8"; do
  timeout -k 10 240 python bench.py --config c5 $a --no-cpu-baseline >> gpurun_out/r04c_c5.jsonl 2>> gpurun_out/r04c.err || exit $?
done

timeout -k 10 200 python -u tools/time_resident.py --time-only 250,250,128 250,250,256 250,250,512 250,250,1024 > gpurun_out/r04c_res_batch.log 2>&1 || exit $?
echo res-done
