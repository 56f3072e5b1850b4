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
echo done $OUT
