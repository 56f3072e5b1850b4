#!/bin/bash
# One parameterised gpurun command file (replaces the per-call tools/gpu_rNNx.sh files).
#
# usage (on the GPU box, through gpurun):
#   bash tools/gpu.sh TAG STEP [STEP ...]
# STEP, each run under its own `timeout -k 10`, in order; the script stops at the first step that fails
# (pytest's rc 1 = "some tests failed" is reported and the script goes on, any other failure ends it):
#   tests[:ARGS]      pytest ARGS (default `tests -m gpu`)          -> gpurun_out/TAG_tests.log
#   smoke             __graft_entry__.smoke()                       -> gpurun_out/TAG_smoke.log
#   bench[:ARGS]      python bench.py ARGS                          -> gpurun_out/TAG_bench.jsonl (appends)
#   hbm               tools/ubench/stream (HBM streaming ceiling)   -> gpurun_out/TAG_hbm.jsonl
#   prof:ARGS         tools/profile_all.sh TAG ARGS (bench + rocprof stats + PMC passes)
#   profres:SHAPE     tools/prof_resident.sh TAG SHAPE
#   py:SCRIPT ARGS    python -u SCRIPT ARGS                         -> gpurun_out/TAG_<script>.log (appends)
# A step may end in @SECONDS to change its time limit (default 300; tests 600).
# Example:  gpurun --timeout 900 -- bash tools/gpu.sh r05a hbm 'bench:--steps 20' 'tests:tests/test_gpu_plane.py -m gpu'
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/$TAG
for step in "$@"; do
    lim=300
    if [[ $step == *@* ]]; then lim=${step##*@}; step=${step%@*}; fi
    kind=${step%%:*}
    arg=""
    [[ $step == *:* ]] && arg=${step#*:}
    echo "[$(date +%T)] $TAG: $kind $arg (limit ${lim}s)"
    case $kind in
        tests)
            [[ $lim == 300 ]] && lim=600
            [[ -z $arg ]] && arg="tests -m gpu"
            timeout -k 10 $lim python -u -m pytest $arg -q -rf --timeout 240 --timeout-method thread \
                -p no:cacheprovider >> ${O}_tests.log 2>&1
            rc=$?
            tail -3 ${O}_tests.log
            if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stop"; exit $rc; fi
            ;;
        smoke)
            timeout -k 10 $lim python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 || exit $?
            cat ${O}_smoke.log
            ;;
        bench)
            timeout -k 10 $lim python bench.py $arg >> ${O}_bench.jsonl 2>> ${O}_bench.err || exit $?
            tail -1 ${O}_bench.jsonl | cut -c1-400
            ;;
        hbm)
            timeout -k 10 $lim tools/ubench/stream ${O}_hbm.jsonl > ${O}_hbm.log 2>&1 || exit $?
            ;;
        prof)
            timeout -k 10 $((lim * 4)) bash tools/profile_all.sh $TAG $arg || exit $?
            ;;
        profres)
            timeout -k 10 $((lim * 2)) bash tools/prof_resident.sh $TAG $arg || exit $?
            ;;
        py)
            script=${arg%% *}
            rest=""
            [[ $arg == *" "* ]] && rest=${arg#* }
            timeout -k 10 $lim python -u $script $rest >> ${O}_$(basename $script .py).log 2>&1 || exit $?
            tail -2 ${O}_$(basename $script .py).log
            ;;
        *)
            echo "unknown step $kind"; exit 2;;
    esac
done
echo "[$(date +%T)] $TAG: all steps done"
