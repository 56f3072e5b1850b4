#!/bin/bash
# On the GPU box: rocprofv3 kernel stats + HBM PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs, as
# MI355X_MICROARCH.md prescribes) of the CU-resident smooth-size solve.  usage: tools/prof_resident.sh TAG N,M,B
set -euo pipefail
TAG=$1; SHAPE=$2
export TMPDIR=/tmp
OUT=gpurun_out/prof_res_$TAG
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python tools/time_resident.py --time-only $SHAPE > $OUT/stats.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o p -- python tools/time_resident.py --time-only $SHAPE > /dev/null 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o p -- python tools/time_resident.py --time-only $SHAPE > /dev/null 2>&1
echo done $OUT
