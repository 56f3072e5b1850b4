"""Line-transform microbenchmark: inverse + forward round trips of 256-point real lines held in registers,
lane-pair layout (512 threads per 256 lines, 2 waves/SIMD) vs lane-quad layout (1024 threads, 4 waves/SIMD).
Usage (GPU box): python tools/line_bench.py [planes] [reps]"""
import ctypes
import os
import sys

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
lib = ctypes.CDLL(os.path.join(REPO, "admm-deconv_amd", "libadmm_devtest.so"))
lib.devtest_line_bench.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_float)]
planes = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 25
dev = torch.device("cuda:0")
x = torch.randn(planes * 256, 256, device=dev)
y = torch.empty_like(x)
for quad in (0, 1, 0, 1):
    ms = ctypes.c_float(0)
    assert lib.devtest_line_bench(x.data_ptr(), y.data_ptr(), planes * 256, reps, quad, ctypes.byref(ms)) == 0
    err = (y - x).abs().max().item() / x.abs().max().item()
    print(f"{'quad' if quad else 'pair'}: {planes} planes x {reps} round trips: {ms.value:.3f} ms "
          f"({1e3 * ms.value / reps / (planes / 256):.2f} us per round trip per plane-round), max rel err {err:.1e}",
          flush=True)
