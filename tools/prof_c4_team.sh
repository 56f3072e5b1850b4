#!/bin/bash
# PMC passes of the team512 launch alone (the --stats run of it segfaults in the profiler's teardown at exit,
# after writing its CSVs: gpurun_out/prof_r05m_team/stats.log)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp PYTHONUNBUFFERED=1 ADMM_EXP_TEAM512=1
OUT=gpurun_out/prof_${1:-c4}_team; mkdir -p $OUT
B="python bench.py --config c4 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o p -- $B --steps 1 --warmup 1 > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o p -- $B --steps 1 --warmup 1 > $OUT/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace --output-format csv -d $OUT/pmc_sq -o p -- $B --steps 1 --warmup 1 > $OUT/sq.log 2>&1 || exit $?
echo done
