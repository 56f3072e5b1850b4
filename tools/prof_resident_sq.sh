#!/bin/bash
# SQ view of the CU-resident solve (instruction fetch, waits, VALU) at one shape and several plane counts:
# one PMC pass (<= 8 SQ counters) per plane count over tools/time_resident.py --time-only.
# usage (GPU box): bash tools/prof_resident_sq.sh TAG "250,250,128 250,250,256"
set -uo pipefail
TAG=$1; SHAPES=$2
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
CTR="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_IFETCH"
for s in $SHAPES; do
    d=$OUT/${s//,/x}
    timeout -s KILL 90 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d $d -o p -- \
        python3 tools/time_resident.py --time-only $s > $d.log 2>&1 || { echo "pass rc=$? ($s)"; exit 1; }
done
echo done
