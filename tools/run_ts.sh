timeout -k 10 100 python tools/plane_ts.py 512 > gpurun_out/ts.log 2>&1; cat gpurun_out/ts.log
