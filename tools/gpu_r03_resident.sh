# gpurun command file (round 3, resident solve): full GPU suite, smoke, default bench, resident shapes, rocprof
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/suite.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
timeout -k 10 200 python -u tools/time_resident.py 250,250,256 240,240,256 200,200,256 192,192,256 160,160,256 120,120,256 96,96,512 > gpurun_out/shapes2.log 2>&1 && \
tools/prof_resident.sh r250 250,250,256
