"""PSF variant of debug_plane4: run the fused kernel (debug build) 4x on one plane, report the first
phase whose register state differs between runs."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "admm-deconv_amd"))
from admm_deconv import synth  # noqa: E402

dev = torch.device("cuda:0")
lib = ctypes.CDLL(os.path.join(REPO, "admm-deconv_amd", sys.argv[2] if len(sys.argv) > 2 else "libadmm_devtest.so"))
P = ctypes.c_void_p
lib.devtest_plane_debug_psf.argtypes = [P, P, P, P, P, P, P, P, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                        ctypes.c_int, P]
lib.devtest_plane_tables_psf.argtypes = [P, P, P, P, P, P]
M = N = 256
lam, rho, K = 0.0041, 0.021, int(sys.argv[1]) if len(sys.argv) > 1 else 4
h = synth.gaussian_psf(15, 2.5).astype(np.float64)   # (kw, kh)
kw, kh = h.shape
hh = np.zeros((N, M))
hh[:kw, :kh] = h
Sig = np.fft.rfft2(hh)                                # [kj][k]
k = np.arange(M // 2 + 1)[None, :]
kj = np.arange(N)[:, None]
padd, padr = (kh - 1) // 2, (kw - 1) // 2
Sc = Sig * np.exp(2j * np.pi * (padd * k / M + padr * kj / N))
lap = 4 * np.sin(np.pi * kj / N) ** 2 + 4 * np.sin(np.pi * k / M) ** 2
Ct = torch.from_numpy((1.0 / (np.abs(Sig) ** 2 + rho * lap) / (M * N)).astype(np.float32).ravel()).to(dev)
G = np.conj(Sc) / (M * N)
Gt = torch.from_numpy(np.stack([G.real, G.imag], -1).astype(np.float32).ravel()).to(dev)
Cf = torch.zeros(2 * 32 * 512, device=dev)
C0b = torch.zeros(256, device=dev)
Gf = torch.zeros(2 * 32 * 512 * 2, device=dev)
G0b = torch.zeros(512, device=dev)
assert lib.devtest_plane_tables_psf(Ct.data_ptr(), Gt.data_ptr(), Cf.data_ptr(), C0b.data_ptr(), Gf.data_ptr(),
                                    G0b.data_ptr()) == 0
y = torch.from_numpy(synth.make_batch(1, M, N, synth.gaussian_psf(15, 2.5))).to(dev)
runs = []
for r in range(4):
    x = torch.zeros_like(y)
    hln = torch.zeros(64 * 512 * 2, device=dev)
    sln = torch.full((64 * 512 * 4,), float("nan"), device=dev)
    dbg = torch.zeros(4 * K, 64, 512, 2, device=dev)
    assert lib.devtest_plane_debug_psf(y.data_ptr(), x.data_ptr(), Cf.data_ptr(), C0b.data_ptr(), Gf.data_ptr(),
                                       G0b.data_ptr(), hln.data_ptr(), sln.data_ptr(), lam / rho, rho, K, 1,
                                       dbg.data_ptr()) == 0
    runs.append((dbg.cpu().numpy(), x.cpu().numpy()))
names = {1: "column", 2: "line_inv", 3: "row_update", 0: "line_fwd"}
for r in range(1, 4):
    d0, d1 = runs[0][0], runs[r][0]
    diff = np.abs(d0 - d1).max(axis=(1, 3))
    first = next((sl for sl in range(4 * K - 1) if diff[sl].max() > 0), None)
    if first is None:
        print(f"run {r}: identical (x maxdiff {np.abs(runs[0][1] - runs[r][1]).max():.2e})")
        continue
    dd = np.abs(d0[first] - d1[first]).max(axis=2)
    bad = np.argwhere(dd > 0)
    print(f"run {r}: first differing slot {first} ({names[first % 4]}, k={(first + 3) // 4}), {len(bad)} (n,t), "
          f"max {dd.max():.3e}; threads {sorted(set(bad[:, 1].tolist()))[:24]} regs {sorted(set(bad[:, 0].tolist()))[:24]}")
