"""Which of h_bar's two cancelling paths carries the GPU's error (VERDICT r05 Next #1; GPU box only).

h_bar = (path through H^T y: corr(Vsum, y), Vsum = sum_k vbar_k) + (path through C = 1/(|Sigma|^2 + rho|D|^2):
-C^2 Q d|Sigma|^2/dh, Q = sum_k Re(conj(G_k) V_k)).  This runs one recorded 2-pass case on the GPU, reads the
sweep's own Vsum, Q and the two paths from the workspace (libadmm_devtest.so offsets), and compares each with
the mask-conditioned fp64 oracle's (leaves on H^T y and on C: their gradients are Vsum and Cbar) and with an fp32
torch evaluation of the same computation.  Prints one JSON line per case.

usage: python tools/hbar_paths.py [case ...]   (cases of tests/test_gpu_adjoint_masked.py with a PSF)
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), os.path.join(REPO, "admm-deconv_amd")]

import admm_deconv  # noqa: E402
import oracle_torch as ot  # noqa: E402
from admm_deconv import synth  # noqa: E402
import test_gpu_adjoint_masked as tm  # noqa: E402


def paths(y, lam, rho, h, K, xbar, masks, dtype):
    """x, Vsum, Cbar, h_bar through H^T y, h_bar through C -- autograd with leaves on H^T y and on C."""
    B, P, N, M = y.shape
    yt = torch.as_tensor(y, dtype=dtype)
    ht = torch.as_tensor(h, dtype=dtype).clone().requires_grad_(True)
    rt = torch.tensor(float(rho), dtype=dtype)
    hty_f = ot._ht(yt, ht)
    C_f = ot._make_C(M, N, rt, ht)
    hty = hty_f.detach().clone().requires_grad_(True)
    C = C_f.detach().clone().requires_grad_(True)
    tau = torch.tensor(float(np.float32(lam) / np.float32(rho)), dtype=dtype)
    x = torch.zeros_like(yt)
    z1 = torch.zeros_like(yt); z2 = torch.zeros_like(yt); u1 = torch.zeros_like(yt); u2 = torch.zeros_like(yt)
    for it in range(K):
        w1, w2 = z1 - u1, z2 - u2
        dtw = (w1 - torch.roll(w1, -1, dims=-2)) + (w2 - torch.roll(w2, -1, dims=-1))
        x = torch.fft.irfft2(C * torch.fft.rfft2(hty + rt * dtw), s=(N, M))
        d1 = x - torch.roll(x, 1, dims=-2)
        d2 = x - torch.roll(x, 1, dims=-1)
        s1, s2 = d1 + u1, d2 + u2
        if it < len(masks):
            m, sg = (torch.as_tensor(a, dtype=dtype) for a in masks[it])
            z1 = m[:, :, 0] * (s1 - sg[:, :, 0] * tau)
            z2 = m[:, :, 1] * (s2 - sg[:, :, 1] * tau)
        else:
            z1 = torch.sign(s1) * torch.clamp(torch.abs(s1) - tau, min=0.0)
            z2 = torch.sign(s2) * torch.clamp(torch.abs(s2) - tau, min=0.0)
        u1, u2 = u1 + d1 - z1, u2 + d2 - z2
    (x * torch.as_tensor(xbar, dtype=dtype)).sum().backward()
    vsum, cbar = hty.grad.detach(), C.grad.detach()
    h_corr = torch.autograd.grad(hty_f, ht, vsum, retain_graph=True)[0]
    h_A = torch.autograd.grad(C_f, ht, cbar)[0]
    return (x.detach().numpy().astype(np.float64), vsum.numpy().astype(np.float64), cbar.numpy().astype(np.float64),
            h_corr.numpy().astype(np.float64), h_A.numpy().astype(np.float64))


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-300))


def run(case, seed=None):
    """seed None: the test's own inputs; otherwise other images (g0) and another xbar, same shapes and PSF."""
    cid, B, P, N, M, spec, lam, rho, K, iso, need_h, opts = case
    assert spec is not None and not iso
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(N + M + K + 31 * B + (0 if seed is None else 1000 * seed))
    h = tm._psf(spec, rng)
    y = synth.make_batch(B, M, N, h, P=P, g0=7 if seed is None else 100 + 3 * seed)
    if seed is not None:
        cid = f"{cid}@seed{seed}"
    xbar = rng.standard_normal(y.shape).astype(np.float32)
    yt, xt, ht = (torch.from_numpy(a).to(dev) for a in (y, xbar, h))
    x, rec = admm_deconv.tvd_fft_record(yt, lam, rho, ht, False, K, need_h=True)
    torch.cuda.synchronize()
    s_traj, _ = tm.read_trajectory(rec, K, False)
    masks = ot.masks_from_trajectory(s_traj, lam, rho, False)
    ws = rec.workspace   # (the replay releases the recording's hold on it)
    yb, hb, lb, rb = admm_deconv.tvd_fft_backward_recorded(rec, x, xt)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(os.path.join(REPO, "admm-deconv_amd", "libadmm_devtest.so"))
    f = lib.devtest_hbar_offsets
    f.argtypes = [ctypes.c_int] * 7 + [ctypes.POINTER(ctypes.c_size_t)]
    off = (ctypes.c_size_t * 4)()
    kw, kh = h.shape
    assert f(M, N, P, B, kh, kw, K, off) == 0
    buf = ws._buf
    ptr, _ = ws.get(0, buf.device)
    base = ptr - buf.data_ptr()
    planes, H = B * P, M // 2 + 1

    def grab(o, n, dt):
        nb = n * np.dtype(dt).itemsize
        return buf[base + o: base + o + nb].cpu().numpy().view(dt).copy()
    vsum_g = grab(off[0], planes * M * N, np.float32).reshape(B, P, N, M).astype(np.float64)
    Q_g = grab(off[1], H * N, np.float64).reshape(N, H)
    hc_g = grab(off[2], kh * kw, np.float64).reshape(kw, kh)
    hA_g = grab(off[3], kh * kw, np.float64).reshape(kw, kh)
    x64, v64, c64, hc64, hA64 = paths(y.astype(np.float64), lam, rho, h.astype(np.float64), K, xbar, masks, torch.float64)
    x32, v32, c32, hc32, hA32 = paths(y, lam, rho, h, K, xbar, masks, torch.float32)
    hb64 = hc64 + hA64
    scale = float(np.linalg.norm(np.abs(hc64) + np.abs(hA64)))
    # Cbar = w_k / (MN) Q (irfft2's normalisation and Hermitian weights): the per-bin factor, and Q's error
    wk = np.full(H, 2.0); wk[0] = 1.0; wk[-1] = 1.0
    Qn = Q_g * wk[None, :] / (M * N)
    # where h_bar's C path lives: |C^2 dS| weight per bin, and the error contributions by band
    k = np.arange(H)[None, :]; kj = np.arange(N)[:, None]
    ring = np.sqrt((np.minimum(kj, N - kj) / N) ** 2 + (k / M) ** 2)
    bands = [0, 0.02, 0.05, 0.1, 0.2, 0.3, 0.75]
    qerr = {}
    for lo, hi in zip(bands[:-1], bands[1:]):
        sel = (ring >= lo) & (ring < hi)
        qerr[f"{lo}-{hi}"] = {"gpu": float(np.linalg.norm((Qn - c64)[sel]) / max(np.linalg.norm(c64[sel]), 1e-300)),
                             "fp32": float(np.linalg.norm((c32 - c64)[sel]) / max(np.linalg.norm(c64[sel]), 1e-300)),
                             "cbar_norm": float(np.linalg.norm(c64[sel]))}
    # the C path from the GPU's own Q through the exact fp64 map (separates Q's error from hbarA_kernel's
    # arithmetic), and each band's share of the C path's error (the Q error of that band alone, mapped)
    hq = torch.from_numpy(h.astype(np.float64)).requires_grad_(True)
    Cq = ot._make_C(M, N, torch.tensor(float(np.float32(rho)), dtype=torch.float64), hq)

    def cmap(cb):
        return torch.autograd.grad(Cq, hq, torch.from_numpy(np.ascontiguousarray(cb)), retain_graph=True)[0].numpy()
    hA_fromQ = cmap(Qn)
    nh = float(np.linalg.norm(hc64 + hA64))
    for lo, hi in zip(bands[:-1], bands[1:]):
        sel = (ring >= lo) & (ring < hi)
        qerr[f"{lo}-{hi}"]["gpu_hA_err_over_hbar"] = float(np.linalg.norm(cmap(np.where(sel, Qn - c64, 0.0)))) / nh
        qerr[f"{lo}-{hi}"]["fp32_hA_err_over_hbar"] = float(np.linalg.norm(cmap(np.where(sel, c32 - c64, 0.0)))) / nh
    # corr(Vsum_gpu, y) in fp64 on the host: separates Vsum's error from the correlation's arithmetic
    yt64 = torch.from_numpy(y.astype(np.float64))
    h_l = torch.from_numpy(h.astype(np.float64)).requires_grad_(True)
    hc_from_vg = torch.autograd.grad(ot._ht(yt64, h_l), h_l, torch.from_numpy(vsum_g))[0].numpy()
    out = {"case": cid,
           "h_bar": {"gpu_rel_value": rel(hb.cpu().numpy(), hb64), "fp32_rel_value": rel(hc32 + hA32, hb64),
                     "gpu_rel_scale": float(np.linalg.norm(hb.cpu().numpy() - hb64)) / scale,
                     "path_scale_over_value": scale / float(np.linalg.norm(hb64))},
           "corr_path": {"gpu_abs_over_hbar": float(np.linalg.norm(hc_g - hc64) / np.linalg.norm(hb64)),
                         "fp32_abs_over_hbar": float(np.linalg.norm(hc32 - hc64) / np.linalg.norm(hb64)),
                         "gpu_rel": rel(hc_g, hc64), "host_corr_of_gpu_vsum_vs_gpu": rel(hc_from_vg, hc_g)},
           "C_path": {"gpu_abs_over_hbar": float(np.linalg.norm(hA_g - hA64) / np.linalg.norm(hb64)),
                      "fp32_abs_over_hbar": float(np.linalg.norm(hA32 - hA64) / np.linalg.norm(hb64)),
                      "gpu_rel": rel(hA_g, hA64), "exact_map_of_gpu_Q_vs_gpu": rel(hA_fromQ, hA_g),
                      "exact_map_of_gpu_Q_err_over_hbar": float(np.linalg.norm(hA_fromQ - hA64)) / nh},
           "vsum": {"gpu_rel": rel(vsum_g, v64), "fp32_rel": rel(v32, v64)},
           "Q": {"gpu_rel": rel(Qn, c64), "fp32_rel": rel(c32, c64), "bands": qerr},
           "x": {"gpu_rel": rel(x.cpu().numpy(), x64), "fp32_rel": rel(x32, x64)}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    args = sys.argv[1:] or ["2pass-256-c2-K25-hbar"]
    seeds = [None]
    for a in args:
        if a.startswith("--seeds="):
            seeds = [int(v) for v in a.split("=", 1)[1].split(",")]
    want = [a for a in args if not a.startswith("--")]
    for c in tm.CASES:
        if c[0] in want:
            for sd in seeds:
                run(c, sd)
