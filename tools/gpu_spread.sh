set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/wg_spread.py 128 192 256 512 > gpurun_out/wg_spread.txt 2>&1
