set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_adjoint_masked.py -k "isofused or fused_iso or iso-256" > gpurun_out/iso_t.log 2>&1 && \
timeout -k 10 120 python -u tools/time_iso.py 192 50 > gpurun_out/iso_time.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_layers.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_device_scalars.py > gpurun_out/iso_t2.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c5 --iso --steps 3 --warmup 1 > gpurun_out/c5iso.json 2> gpurun_out/c5iso.err
