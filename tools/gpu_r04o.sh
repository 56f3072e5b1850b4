# round 4, fifteenth GPU call: smooth 2-pass kernels -- previous build vs update on pixel pairs vs pairs + column
# multipliers hoisted before the barrier, same box, two rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/lib_cur.so
for round in 1 2; do
  for v in oldsmooth pairs hoist; do
    cp admm-deconv_amd/libadmm_deconv_$v.so $L
    echo "== $v"
    timeout -k 10 200 python -u tools/time_generic.py 480,640,64 250,250,256 1000,1000,16 300,400,128 RESIDENT=0 || { cp /tmp/lib_cur.so $L; exit 1; }
  done
done > gpurun_out/r04o_ab.log 2>&1
cp /tmp/lib_cur.so $L
echo all-done
