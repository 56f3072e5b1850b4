# round 4, fifteenth GPU call: smooth update on pixel pairs against the previous build, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
L=admm-deconv_amd/libadmm_deconv.so
cp $L /tmp/lib_new.so
for round in 1 2; do
  for v in new old; do
    if [ $v = old ]; then cp admm-deconv_amd/libadmm_deconv_oldsmooth.so $L; else cp /tmp/lib_new.so $L; fi
    echo "== $v"
    timeout -k 10 200 python -u tools/time_generic.py 480,640,64 250,250,256 1000,1000,16 300,400,128 RESIDENT=0 || { cp /tmp/lib_new.so $L; exit 1; }
  done
done > gpurun_out/r04o_ab.log 2>&1
cp /tmp/lib_new.so $L
echo all-done
