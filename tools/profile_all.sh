#!/bin/bash
# Run on the GPU box (via gpurun): bench JSON, rocprofv3 kernel-trace stats, and the two PMC
# passes (FETCH_SIZE, WRITE_SIZE in separate runs, as MI355X_MICROARCH.md prescribes).
# usage: bash tools/profile_all.sh TAG [bench args...]
set -euo pipefail
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python bench.py --no-cpu-baseline $*"
timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $B --steps 10 --warmup 3 > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o p -- $B --steps 1 --warmup 1 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o p -- $B --steps 1 --warmup 1 > /dev/null 2>&1
# SQ pass (<= 8 SQ counters): VALU / LDS / SALU instruction counts for the roofline's compute-side figure
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace --output-format csv -d $OUT/pmc_sq -o p -- $B --steps 1 --warmup 1 > /dev/null 2>&1
echo done $OUT
