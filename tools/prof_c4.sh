#!/bin/bash
# c4 profiles: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE / SQ passes of the 2-pass path (round 5 also profiled
# the persistent team512 launch, now tools/variants/team512_line512.patch).  usage: tools/prof_c4.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-c4}
for v in 2pass; do
  OUT=gpurun_out/prof_${TAG}_$v; mkdir -p $OUT
  B="python bench.py --config c4 --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- $B --steps 3 --warmup 1 > $OUT/stats.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o p -- $B --steps 1 --warmup 1 > /dev/null 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o p -- $B --steps 1 --warmup 1 > /dev/null 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace --output-format csv -d $OUT/pmc_sq -o p -- $B --steps 1 --warmup 1 > /dev/null 2>&1 || exit $?
  echo "done $v"
done
