# round 4, twenty-third GPU call: rows of loads in flight in the resident row update (RS_PD 2 / 3 / 4 / 5), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
L=admm-deconv_amd/libadmm_deconv.so
cp $L admm-deconv_amd/libadmm_deconv_pd4.so
SHAPES="250,250,256 240,240,256 200,200,256 160,160,256" timeout -k 10 700 bash tools/run_resident_variants.sh pd4 pd3 pd5 pd2 pd4 pd3 pd5 > gpurun_out/r04v_pd.log 2>&1 || exit $?
rm -f admm-deconv_amd/libadmm_deconv_pd4.so
echo all-done
