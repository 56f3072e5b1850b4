#!/bin/bash
# One GPU call: the default bench line plus the other single-GPU configs (c4, c5 aniso / iso).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && \
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && \
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && \
timeout -k 10 300 python bench.py --config c5 --iso --steps 3 --warmup 1 > gpurun_out/bench_c5iso.json 2> gpurun_out/bench_c5iso.err
rc=$?
for f in c2 c4 c5 c5iso; do echo "== $f"; cat gpurun_out/bench_$f.json 2>/dev/null | cut -c1-600; done
exit $rc
