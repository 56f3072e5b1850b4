# round 4, tenth GPU call: start stagger of the resident 250^2 / 240^2 grids after the pixel-pair row update
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for st in 0 1000 2000 2500 3500 5000; do
  echo "== PLANE_STAGGER=$st"
  timeout -k 10 120 python -u tools/time_resident.py --time-only PLANE_STAGGER=$st 250,250,256 240,240,256 || exit $?
done > gpurun_out/r04j_stagger.log 2>&1
echo all-done
