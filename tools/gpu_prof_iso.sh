set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_gpu_dist_iso.py > gpurun_out/dist_iso.log 2>&1 && \
bash tools/run_iso_variants.sh isopd3 isopd4 > gpurun_out/iso_variants.txt 2>&1 && \
bash tools/profile_all.sh r03_c5iso --config c5 --iso
