"""Sub-phase breakdown of the fused plane kernel (devtest -DPLANE_TS build, libadmm_devtest_TS.so)."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
from admm_deconv import synth  # noqa: E402

dev = torch.device("cuda:0")
lib = ctypes.CDLL(os.path.join(REPO, "admm-deconv_amd", sys.argv[2] if len(sys.argv) > 2 else "libadmm_devtest_TS.so"))
P = ctypes.c_void_p
lib.devtest_plane_timing.argtypes = [P, P, P, P, P, P, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int, P]
lib.devtest_plane_tables.argtypes = [P, P, P]
lib.devtest_plane_ts_set.argtypes = [P]
M = N = 256
lam, rho, K = 0.0041, 0.021, 25
B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
k = np.arange(M // 2 + 1)[None, :]
kj = np.arange(N)[:, None]
lap = 4 * np.sin(np.pi * kj / N) ** 2 + 4 * np.sin(np.pi * k / M) ** 2
Ct = torch.from_numpy((1.0 / (1.0 + rho * lap) / (M * N)).astype(np.float32).ravel()).to(dev)
Cf = torch.zeros(2 * 32 * 512, device=dev)
C0b = torch.zeros(256, device=dev)
assert lib.devtest_plane_tables(Ct.data_ptr(), Cf.data_ptr(), C0b.data_ptr()) == 0
y = torch.from_numpy(synth.make_batch(8, M, N, None)).to(dev).repeat(B // 8, 1, 1, 1).contiguous()
x = torch.zeros_like(y)
hln = torch.zeros(B * (64 * 512 + 128) * 2, device=dev)   # plane_api.hpp kHtyStrideF2
sln = torch.zeros(B * 64 * 512 * 4, device=dev)
dbg = torch.zeros(B * 8 * 512, dtype=torch.int64, device=dev)
ts = torch.zeros(B * 8 * 64, dtype=torch.int64, device=dev)
assert lib.devtest_plane_ts_set(ts.data_ptr()) == 0
ts.zero_()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
assert lib.devtest_plane_timing(y.data_ptr(), x.data_ptr(), Cf.data_ptr(), C0b.data_ptr(), hln.data_ptr(),
                                sln.data_ptr(), lam / rho, rho, K, B, dbg.data_ptr()) == 0
ev1.record()
torch.cuda.synchronize()
print(f"kernel {ev0.elapsed_time(ev1):.3f} ms (TS build)")
T = ts.view(B, 8, 64).cpu().numpy().astype(np.float64)
names = ["rows->LDS", "barrier", "col read+FFT32", "xchg+radix8", "multiply", "inverse", "barrier"]
for h in (0, 1):
    print(f"-- column half {h} (per call, mean over waves; K={K} calls)")
    for i, nm in enumerate(names):
        d = (T[:, :, h * 8 + i + 1] - T[:, :, h * 8 + i]) / K
        print(f"   {nm:15s} {d.mean():9.0f} cyc   wave0 {d[:, 0].mean():9.0f}   waves1-7 {d[:, 1:].mean():9.0f}")
print(f"-- row_update (per call, {K - 1} calls)")
for i, nm in enumerate(["xb write+barrier", "chunk loop", "barrier"]):
    d = (T[:, :, 17 + i] - T[:, :, 16 + i]) / (K - 1)
    print(f"   {nm:15s} {d.mean():9.0f} cyc")
