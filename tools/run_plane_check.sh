# fused-path check: determinism census, parity tests, timing, phase breakdown (each step time-limited)
timeout -k 10 300 python tools/census_plane.py 4 > gpurun_out/census.log 2>&1 && \
timeout -k 10 300 python -m pytest tests/test_gpu_plane.py tests/test_gpu_devtest.py -q > gpurun_out/plane_test.log 2>&1; \
timeout -k 10 200 python tools/time_plane.py 512 > gpurun_out/time_plane.log 2>&1; \
timeout -k 10 200 python tools/plane_timing.py 512 > gpurun_out/ptime.log 2>&1; \
timeout -k 10 100 python tools/plane_ts.py 512 > gpurun_out/ts.log 2>&1; \
cat gpurun_out/census.log; tail -3 gpurun_out/plane_test.log; cat gpurun_out/time_plane.log gpurun_out/ptime.log gpurun_out/ts.log
