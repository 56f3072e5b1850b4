"""Phase breakdown of the fused plane kernel (devtest timing build): shader-clock cycles per phase,
averaged over waves and iterations, for a c2-sized launch (512 planes)."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
from admm_deconv import synth  # noqa: E402

dev = torch.device("cuda:0")
lib = ctypes.CDLL(os.path.join(REPO, "admm-deconv_amd", "libadmm_devtest.so"))
P = ctypes.c_void_p
lib.devtest_plane_timing.argtypes = [P, P, P, P, P, P, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int, P]
lib.devtest_plane_tables.argtypes = [P, P, P]
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
for rep in range(3):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    assert lib.devtest_plane_timing(y.data_ptr(), x.data_ptr(), Cf.data_ptr(), C0b.data_ptr(), hln.data_ptr(),
                                    sln.data_ptr(), lam / rho, rho, K, B, dbg.data_ptr()) == 0
    ev1.record()
    torch.cuda.synchronize()
    print(f"kernel {ev0.elapsed_time(ev1):.3f} ms (timing build)")
t = dbg.view(B, 8, 512).cpu().numpy().astype(np.float64)
phases = {"col_half0": [], "col_half1": [], "line_inv": [], "row_update": [], "line_fwd": []}
for kk in range(2, K):   # steady-state iterations
    prev_fwd = t[:, :, 4 * (kk - 1)]
    phases["col_half0"].append(t[:, :, 256 + kk] - prev_fwd)
    phases["col_half1"].append(t[:, :, 4 * kk - 3] - t[:, :, 256 + kk])
    phases["line_inv"].append(t[:, :, 4 * kk - 2] - t[:, :, 4 * kk - 3])
    phases["row_update"].append(t[:, :, 4 * kk - 1] - t[:, :, 4 * kk - 2])
    phases["line_fwd"].append(t[:, :, 4 * kk] - t[:, :, 4 * kk - 1])
tot = 0
for name, v in phases.items():
    a = np.array(v)
    tot += a.mean()
    print(f"{name:11s} mean {a.mean():9.0f} cyc  p10 {np.percentile(a, 10):9.0f}  p90 {np.percentile(a, 90):9.0f}")
print(f"iteration  {tot:9.0f} cyc")
