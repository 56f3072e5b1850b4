#!/bin/bash
# backward/record GPU tests + the c5 bench lines (aniso, iso)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_backward.py tests/test_gpu_layers.py tests/test_gpu_plane.py -q -x > gpurun_out/c5_tests.log 2>&1
rc=$?; tail -25 gpurun_out/c5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && \
timeout -k 10 300 python bench.py --config c5 --iso --steps 3 --warmup 1 > gpurun_out/bench_c5iso.json 2> gpurun_out/bench_c5iso.err
rc=$?
for f in c5 c5iso; do python - gpurun_out/bench_$f.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1], d["value"], d["ms_per_step"], {n: round(v["total_ms_per_step"], 2) for n, v in d["kernels"].items()})
PY
done
exit $rc
