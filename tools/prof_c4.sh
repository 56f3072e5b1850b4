#!/bin/bash
# c4 profiles of the MALL-resident schedule (8-plane chunks on 4 streams, ADMM_OPT_MALL_STREAMS): rocprofv3 kernel
# stats + FETCH_SIZE / WRITE_SIZE / SQ passes, summarised on the box into per-launch HBM bytes (tools/make_traffic.py;
# the raw per-dispatch CSVs of ~10k launches per solve are deleted there).  usage: tools/prof_c4.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-c4}
OUT=gpurun_out/prof_${TAG}; mkdir -p $OUT
B="python bench.py --config c4 --no-cpu-baseline"
CHUNK=$(python -c "import sys; sys.path.insert(0, 'admm-deconv_amd'); from admm_deconv import _lib; print(_lib.forward_schedule(512, 512, False, 15, 768)[0])")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $B --steps 3 --warmup 1 > $OUT/stats.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o p -- $B --steps 1 --warmup 1 > /dev/null 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o p -- $B --steps 1 --warmup 1 > /dev/null 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace --output-format csv -d $OUT/pmc_sq -o p -- $B --steps 1 --warmup 1 > /dev/null 2>&1 || exit $?
python tools/make_traffic.py c4 $CHUNK $OUT/pmc_traffic_c4.json $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_sq || exit $?
find $OUT -name "*counter_collection.csv" -delete; find $OUT -name "*kernel_trace.csv" -delete
echo "done chunk=$CHUNK"
