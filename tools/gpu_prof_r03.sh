set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/profile_all.sh r03_c2 --config c2 && bash tools/profile_all.sh r03_c5m --config c5
