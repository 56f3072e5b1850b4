set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_layers.py > gpurun_out/iso_t.log 2>&1 && \
timeout -k 10 200 python -u bench.py --config c5 --iso --steps 3 --warmup 1 > gpurun_out/c5iso.json 2> gpurun_out/c5iso.err && \
timeout -k 10 200 python -u bench.py --config c5 --iso --no-merge --steps 3 --warmup 1 > gpurun_out/c5iso_nm.json 2> gpurun_out/c5iso_nm.err
