#!/bin/bash
# On the GPU box: SQ counters of the runtime-length kernels on one shape (two --pmc passes of <= 8 SQ
# counters each, MI355X_MICROARCH.md limits).  usage: tools/sq_generic.sh TAG N,M,B
set -euo pipefail
TAG=$1; SHAPE=$2
export TMPDIR=/tmp
OUT=gpurun_out/sq_gen_$TAG
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-trace --output-format csv -d $OUT/p1 -o p -- python tools/time_generic.py $SHAPE > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $OUT/p2 -o p -- python tools/time_generic.py $SHAPE > /dev/null 2>&1
python3 tools/pmc_summary.py $OUT/p1 $OUT/p2 --json $OUT/sq.json
