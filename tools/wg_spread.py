"""Per-workgroup start / end of the fused 256^2 solve (devtest DBG = 3: the product kernel plus s_memrealtime at start / end, 10 ns ticks):
how much of a single-wave launch (planes <= 256 CUs) is the slowest workgroup's tail, against two waves.
usage: python tools/wg_spread.py [planes ...]   (needs libadmm_devtest.so)"""
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
lib.devtest_plane_wg_times.argtypes = [P, P, P, P, P, P, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int, P]
lib.devtest_plane_tables.argtypes = [P, P, P]
M = N = 256
lam, rho, K = 0.0041, 0.021, 25
k = np.arange(M // 2 + 1)[None, :]
kj = np.arange(N)[:, None]
lap = 4 * np.sin(np.pi * kj / N) ** 2 + 4 * np.sin(np.pi * k / M) ** 2
Ct = torch.from_numpy((1.0 / (1.0 + rho * lap) / (M * N)).astype(np.float32).ravel()).to(dev)
Cf = torch.zeros(2 * 32 * 512, device=dev)
C0b = torch.zeros(256, device=dev)
assert lib.devtest_plane_tables(Ct.data_ptr(), Cf.data_ptr(), C0b.data_ptr()) == 0
for B in [int(a) for a in sys.argv[1:]] or [128, 192, 256, 512]:
    y = torch.from_numpy(synth.make_batch(8, M, N, None)).to(dev).repeat(B // 8, 1, 1, 1).contiguous()
    x = torch.zeros_like(y)
    hln = torch.zeros(B * (64 * 512 + 128) * 2, device=dev)   # plane_api.hpp kHtyStrideF2
    sln = torch.zeros(B * 64 * 512 * 4, device=dev)
    dbg = torch.zeros(B * 8 * 512, dtype=torch.int64, device=dev)
    for rep in range(3):
        assert lib.devtest_plane_wg_times(y.data_ptr(), x.data_ptr(), Cf.data_ptr(), C0b.data_ptr(), hln.data_ptr(),
                                        sln.data_ptr(), lam / rho, rho, K, B, dbg.data_ptr()) == 0
        torch.cuda.synchronize()
    T = dbg.view(B, 8, 512)[:, 0, 508:510].cpu().numpy().astype(np.float64) * 0.01   # us
    t0 = T[:, 0].min()
    st, en = T[:, 0] - t0, T[:, 1] - t0
    dur = en - st
    print(f"planes {B}: span {en.max():.1f} us; workgroup duration mean {dur.mean():.1f} min {dur.min():.1f} "
          f"max {dur.max():.1f} (p90 {np.percentile(dur, 90):.1f}); start spread {st.max():.1f} us; "
          f"end: p10 {np.percentile(en, 10):.1f} p50 {np.percentile(en, 50):.1f} max {en.max():.1f}", flush=True)
    # per XCD (round-robin placement: workgroup i on XCD i % 8)
    xcd = np.array([dur[i::8].mean() for i in range(8)])
    print("   mean duration per XCD (us): " + " ".join(f"{v:.0f}" for v in xcd), flush=True)
