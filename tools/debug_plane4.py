"""Run the fused kernel (debug build, devtest) twice on one plane and report the first phase whose
register state differs between the runs (slot = 4k-3 column, 4k-2 line-inverse, 4k-1 row-update, 4k forward)."""
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
lib.devtest_plane_debug.argtypes = [P, P, P, P, P, P, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int, P]
lib.devtest_plane_tables.argtypes = [P, P, P]
M = N = 256
lam, rho, K = 0.0041, 0.021, int(sys.argv[1]) if len(sys.argv) > 1 else 6
k = np.arange(M // 2 + 1)[None, :]
kj = np.arange(N)[:, None]
lap = 4 * np.sin(np.pi * kj / N) ** 2 + 4 * np.sin(np.pi * k / M) ** 2
Ct = torch.from_numpy((1.0 / (1.0 + rho * lap) / (M * N)).astype(np.float32).ravel()).to(dev)
Cf = torch.zeros(2 * 32 * 512, device=dev)
C0b = torch.zeros(256, device=dev)
assert lib.devtest_plane_tables(Ct.data_ptr(), Cf.data_ptr(), C0b.data_ptr()) == 0
y = torch.from_numpy(synth.make_batch(1, M, N, None)).to(dev)
runs = []
for r in range(4):
    x = torch.zeros_like(y)
    hln = torch.zeros(64 * 512 * 2, device=dev)
    sln = torch.zeros(64 * 512 * 4, device=dev)
    dbg = torch.zeros(4 * K, 64, 512, 2, device=dev)
    assert lib.devtest_plane_debug(y.data_ptr(), x.data_ptr(), Cf.data_ptr(), C0b.data_ptr(), hln.data_ptr(),
                                   sln.data_ptr(), lam / rho, rho, K, 1, dbg.data_ptr()) == 0
    runs.append((dbg.cpu().numpy(), x.cpu().numpy()))
names = {1: "column", 2: "line_inv", 3: "row_update", 0: "line_fwd"}
for r in range(1, 4):
    d0, d1 = runs[0][0], runs[r][0]
    diff = np.abs(d0 - d1).max(axis=(1, 3))      # (slot, 512)
    first = None
    for slot in range(4 * K - 1):
        if diff[slot].max() > 0:
            first = slot
            break
    if first is None:
        print(f"run {r}: identical to run 0 (x maxdiff {np.abs(runs[0][1] - runs[r][1]).max():.2e})")
        continue
    dd = np.abs(d0[first] - d1[first]).max(axis=2)   # (64 n, 512 t)
    bad = np.argwhere(dd > 0)
    print(f"run {r}: first differing slot {first} ({names[first % 4]}, k={(first + 3) // 4}), "
          f"{len(bad)} (n,t) entries, max {dd.max():.3e}; first entries (n,t): {bad[:12].tolist()}")
    ts = sorted(set(bad[:, 1].tolist()))
    ns = sorted(set(bad[:, 0].tolist()))
    print(f"   threads {ts[:40]}  registers {ns[:40]}")
