"""Streaming-bandwidth probe: device copy y <- x for working sets from L2-size to far beyond the
256 MiB Infinity Cache.  Used to decide whether MALL-resident chunking can beat HBM for the solve."""
import json
import sys

import torch

dev = torch.device("cuda:0")
res = {}
for mib in (8, 16, 32, 64, 96, 128, 192, 256, 512, 1024, 2048):
    n = mib * 1024 * 1024 // 4 // 2   # two buffers of mib/2 each -> working set = mib
    x = torch.rand(n, device=dev)
    y = torch.empty_like(x)
    for _ in range(5):
        y.copy_(x)
    torch.cuda.synchronize()
    reps = max(20, int(20000 / mib))
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        y.copy_(x)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    gbs = 2 * n * 4 / (ms * 1e-3) / 1e9
    res[mib] = round(gbs, 1)
    print(f"working set {mib:5d} MiB: {gbs:8.1f} GB/s  ({ms*1e3:.1f} us)", flush=True)
json.dump(res, open(sys.argv[1] if len(sys.argv) > 1 else "/dev/null", "w"))
