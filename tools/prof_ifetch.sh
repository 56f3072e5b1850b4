#!/bin/bash
# Instruction-fetch view of the fused kernel (c2 bench, one timed step): the counters this gfx950 offers for
# instruction fetch and the wave states, one PMC pass per group (<= 8 SQ counters each), for one or more builds.
# usage (GPU box): bash tools/prof_ifetch.sh TAG "NAME ..." [bench args]   (NAME: tools/ab/lib_NAME.so, or tree)
set -uo pipefail
TAG=$1; NAMES=$2; shift 2
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
WANT="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_IFETCH"
CTR=""
for c in $WANT; do grep -qw "$c" $OUT/avail.txt && CTR="$CTR $c"; done
echo "counters:$CTR" | tee $OUT/counters.txt
[ -n "$CTR" ] || exit 1
for v in $NAMES; do
    if [ $v = tree ]; then unset ADMM_LIB_PATH; else export ADMM_LIB_PATH=$PWD/tools/ab/lib_$v.so; fi
    B="python bench.py --no-cpu-baseline --steps 1 --warmup 1 $*"
    timeout -k 10 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $OUT/$v -o p -- $B > $OUT/$v.log 2>&1 || echo "pass rc=$? ($v)"
done
echo done
