"""What a few foreign resident workgroups cost the fused plane solve (DESIGN.md s6, N = 8 expectation).

An RCCL gather keeps a handful of blocks resident on every rank while it moves data.  The fused kernel
needs a whole CU per workgroup, so each CU such a block sits on delays one plane.  This runs the c2/c3
solve (256 or 512 planes of 256^2, K=25) alone and beside `hog_kernel` (tools/ubench/hog.hip: nblk
workgroups of 256 threads held for `ms` milliseconds) on a second stream, launched just before or just
after the solve, and prints the solve's own event time and the wall time until both are done.

usage (GPU box): python tools/contend.py [planes ...]
"""
import ctypes
import os
import sys
import time

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
import admm_deconv  # noqa: E402
from admm_deconv import synth  # noqa: E402

hog = ctypes.CDLL(os.path.join(REPO, "tools", "ubench", "libhog.so"))
hog.launch_hog.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_ulonglong, ctypes.c_void_p, ctypes.c_void_p]

dev = torch.device("cuda:0")
h = synth.gaussian_psf(15, 2.5)
base = torch.from_numpy(synth.make_batch(64, 256, 256, h)).to(dev)
ht = torch.from_numpy(h).to(dev)
sink = torch.empty(1024, device=dev)
side = torch.cuda.Stream(device=dev)
main = torch.cuda.current_stream(dev)


def run(planes, nblk, ms, order, reps=5):
    y = base.repeat((planes + 63) // 64, 1, 1, 1)[:planes].contiguous()
    out = torch.empty_like(y)
    ws = admm_deconv.Workspace()
    for _ in range(2):
        admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 25, out=out, workspace=ws)
    torch.cuda.synchronize()
    solve_ms, wall_ms = [], []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if nblk and order == "before":
            hog.launch_hog(nblk, 256, int(ms * 1e5), sink.data_ptr(), ctypes.c_void_p(side.cuda_stream))
        e0.record(main)
        admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 25, out=out, workspace=ws)
        e1.record(main)
        if nblk and order == "after":
            hog.launch_hog(nblk, 256, int(ms * 1e5), sink.data_ptr(), ctypes.c_void_p(side.cuda_stream))
        torch.cuda.synchronize()
        wall_ms.append(1e3 * (time.perf_counter() - t0))
        solve_ms.append(e0.elapsed_time(e1))
    solve_ms.sort()
    wall_ms.sort()
    print(f"planes {planes:4d} hog {nblk:3d} blk x {ms:.1f} ms {order:6s}: solve {solve_ms[len(solve_ms) // 2]:.3f} ms  "
          f"wall {wall_ms[len(wall_ms) // 2]:.3f} ms", flush=True)


for planes in [int(a) for a in sys.argv[1:]] or [256, 512]:
    run(planes, 0, 0, "-")
    for nblk in (1, 8, 16, 32):
        run(planes, nblk, 1.2, "before")
    for nblk in (8, 32):
        run(planes, nblk, 1.2, "after")
    run(planes, 0, 0, "-")
