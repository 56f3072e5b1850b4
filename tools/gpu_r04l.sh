# round 4, twelfth GPU call: rocprof + HBM PMC of the resident 250^2 kernel after the pixel-pair row update
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 700 bash tools/prof_resident.sh r04l 250,250,256 || exit $?
echo all-done
