"""Differentiable CPU oracle (PyTorch, fp64) -- TEST INFRASTRUCTURE ONLY.

A torch restatement of /root/reference/src/ops/ops.jl:17-96 (same operators as oracle_np.py's
literal form: np.roll stencils, spatial H^T with the pad2 offsets, rfft/irfft over dims (1,2)),
used as the gradient oracle for the adjoint (the reference gets its gradients
from Zygote unrolling the loop, src/train.jl:51).  torch.autograd differentiates ST/BT exactly as
Zygote's broadcast rules do away from the kinks (sign' = 0, max(., 0)' = step).
Parity status: unpinned against Julia (see oracle_np.py); pinned against oracle_np by tests.

Arrays are C layout (B, P, N, M) like the C ABI; the PSF is (kw, kh).
"""
from __future__ import annotations

import torch


def _ht(y, h):
    """H^T y (ops.jl:72-81): sum_{a,b} h[b,a] y[i+a-padd, j+b-padr]; y (..., N, M), h (kw, kh)."""
    kw, kh = h.shape
    padd, padr = (kh - 1) // 2, (kw - 1) // 2
    out = torch.zeros_like(y)
    for b in range(kw):
        for a in range(kh):
            out = out + h[b, a] * torch.roll(y, shifts=(-(b - padr), -(a - padd)), dims=(-2, -1))
    return out


def _make_C(M, N, rho, h):
    """ops.jl:22-37; differentiable in rho and h.  Shape (N, M//2+1) (rfft over the last dim)."""
    dev, dt = rho.device, rho.dtype
    if h is None:
        s2 = torch.ones((N, M // 2 + 1), dtype=dt, device=dev)
    else:
        kw, kh = h.shape
        hh = torch.zeros((N, M), dtype=dt, device=dev)
        hh = hh.index_put((torch.arange(kw).repeat_interleave(kh), torch.arange(kh).repeat(kw)), h.reshape(-1))
        S = torch.fft.rfft2(hh)
        s2 = S.real ** 2 + S.imag ** 2
    k = torch.arange(M // 2 + 1, dtype=dt, device=dev)[None, :]
    kj = torch.arange(N, dtype=dt, device=dev)[:, None]
    lap = 4 * torch.sin(torch.pi * kj / N) ** 2 + 4 * torch.sin(torch.pi * k / M) ** 2
    return 1.0 / (s2 + rho * lap)


def tvd_fft_torch(y, lam, rho, h=None, isotropic=False, maxit=100, masks=None, record=None, tau=None, terms=None,
                  h_C=None):
    """y: (B,P,N,M) float64 tensor; lam, rho: 0-d tensors; h: (kw,kh) tensor or None.  Returns x.

    masks (optional): the prox's branch decisions held fixed, one entry per iteration k = 1..maxit-1 --
    anisotropic: (m, sgn) of shape (B,P,2,N,M), m = 1[|s_k| > tau] and sgn = sign(s_k); isotropic: m of
    shape (N,M), m = 1[||s_k|| > tau].  The prox then becomes the branch the masks select,
        ST: z = m (s - sgn tau)            BT: z = m (1 - tau/||s||) s,
    which equals the exact prox wherever the masks agree with s_k, and is differentiable there in the
    same way (Zygote / autograd differentiate the selected branch).  Used to condition the gradient
    oracle on the ST / BT masks of an fp32 implementation's own forward (tests/test_gpu_adjoint_masked.py):
    fp32 and fp64 forwards flip different mask bits where |s_k| is within rounding of tau.
    record (optional list): receives (s_k as (B,P,2,N,M), ||s_k|| as (N,M)) for k = 1..maxit-1.
    tau (optional): the threshold as its own variable (default lam / rho, ops.jl:20) -- splits rho's
    gradient into its explicit part and the part through tau (tvd_fft_grads_split).
    terms (optional dict): every use of rho and tau gets its own elementwise copy (lists terms["rho"],
    terms["tau"]; retain_grad), so that after backward() the sum of |grad| over them is the sum of the
    absolute values of the terms rho_bar and tau_bar add up -- the scale fp summation error is measured
    against (the gradients are heavily cancelling sums).
    h_C (optional): the PSF as it enters C = 1/(|Sigma|^2 + rho |Lambda|^2) (ops.jl:22-37), a separate leaf from
    the `h` of H^T y (ops.jl:71-81), so that h_bar splits into its two paths (tvd_fft_grads_split)."""
    B, P, N, M = y.shape
    if tau is None:
        tau = lam / rho                                               # ops.jl:20
    rho0, tau0 = rho, tau

    def _own(v, shape, kind):
        if terms is None:
            return v
        c = v.expand(shape).clone()
        c.retain_grad()
        terms.setdefault(kind, []).append(c)
        return c
    hc = h if h_C is None else h_C
    C = _make_C(M, N, rho, hc)
    hty = y if h is None else _ht(y, h)
    x = torch.zeros_like(y)
    z1 = torch.zeros_like(y); z2 = torch.zeros_like(y)
    u1 = torch.zeros_like(y); u2 = torch.zeros_like(y)
    for it in range(maxit):
        w1, w2 = z1 - u1, z2 - u2
        dtw = (w1 - torch.roll(w1, -1, dims=-2)) + (w2 - torch.roll(w2, -1, dims=-1))
        if terms is not None:
            C = _make_C(M, N, _own(rho0, (N, M // 2 + 1), "rho"), hc)
            rho = _own(rho0, y.shape, "rho")
        x = torch.fft.irfft2(C * torch.fft.rfft2(hty + rho * dtw), s=(N, M))
        d1 = x - torch.roll(x, 1, dims=-2)                             # x[i,j]-x[i,j-1]
        d2 = x - torch.roll(x, 1, dims=-1)                             # x[i,j]-x[i-1,j]
        s1, s2 = d1 + u1, d2 + u2
        if record is not None and it < maxit - 1:
            record.append((torch.stack([s1, s2], dim=2).detach(),
                           torch.sqrt((s1 * s1 + s2 * s2).sum(dim=(0, 1))).detach()))
        fixed = masks is not None and it < len(masks)
        if terms is not None and it < maxit - 1:   # (the last iteration's prox output is dead)
            tau = _own(tau0, (1, 1, N, M) if isotropic else y.shape, "tau")
            tau_b = tau if isotropic else _own(tau0, y.shape, "tau")
        else:
            tau_b = tau
        if isotropic:
            nrm = torch.sqrt((s1 * s1 + s2 * s2).sum(dim=(0, 1), keepdim=True))
            if fixed:
                m = torch.as_tensor(masks[it], dtype=y.dtype)
                f = m * (1 - tau / torch.where(m > 0, nrm, torch.ones_like(nrm)))
            else:
                f = torch.clamp(1 - tau / nrm, min=0.0)
            z1, z2 = f * s1, f * s2
        elif fixed:
            m, sg = (torch.as_tensor(a, dtype=y.dtype) for a in masks[it])
            z1 = m[:, :, 0] * (s1 - sg[:, :, 0] * tau)
            z2 = m[:, :, 1] * (s2 - sg[:, :, 1] * tau_b)
        else:
            z1 = torch.sign(s1) * torch.clamp(torch.abs(s1) - tau, min=0.0)
            z2 = torch.sign(s2) * torch.clamp(torch.abs(s2) - tau_b, min=0.0)
        u1, u2 = u1 + d1 - z1, u2 + d2 - z2
    return x


def tvd_fft_grads(y, lam, rho, h, iso, maxit, xbar, dtype=torch.float64, masks=None):
    """Autograd gradients of <xbar, x(y, lam, rho, h)> in `dtype` (fp64: the gradient oracle; fp32: what an
    fp32 implementation of the reference's own Zygote pass gets, used to size the gradient tolerances):
    returns (x, ybar, hbar, lambar, rhobar).  masks: see tvd_fft_torch (prox branches held fixed)."""
    y = torch.as_tensor(y, dtype=dtype).clone().requires_grad_(True)
    lam_t = torch.tensor(float(lam), dtype=dtype, requires_grad=True)
    rho_t = torch.tensor(float(rho), dtype=dtype, requires_grad=True)
    h_t = None
    if h is not None and h.size:
        h_t = torch.as_tensor(h, dtype=dtype).clone().requires_grad_(True)
    x = tvd_fft_torch(y, lam_t, rho_t, h_t, iso, maxit, masks)
    (x * torch.as_tensor(xbar, dtype=dtype)).sum().backward()
    return (x.detach().numpy(), y.grad.numpy(), None if h_t is None else h_t.grad.numpy(),
            float(lam_t.grad) if lam_t.grad is not None else 0.0, float(rho_t.grad) if rho_t.grad is not None else 0.0)


def masks_from_trajectory(s_traj, lam, rho, iso, nrm_traj=None):
    """Prox branch masks of a recorded fp32 forward (tvd_fft_torch's `masks`): s_traj (K-1, B, P, 2, N, M)
    = s_1..s_{K-1} as the GPU stored them; iso: nrm_traj (K-1, N, M) = the recorded batch norms.  tau is
    formed as the library forms it, lambda / rho in fp32 (ops.jl:20)."""
    import numpy as np
    tau = np.float32(np.float32(lam) / np.float32(rho))
    if iso:
        return [(np.asarray(n) > tau).astype(np.float64) for n in nrm_traj]
    return [((np.abs(s) > tau).astype(np.float64), np.sign(s).astype(np.float64)) for s in s_traj]


def tvd_fft_grads_split(y, lam, rho, h, iso, maxit, xbar, dtype=torch.float64, masks=None, scales=None):
    """Gradients with tau = lam / rho as its own variable: returns (x, ybar, hbar, tau_bar, rho_bar_explicit).
    Then lam_bar = tau_bar / rho and rho_bar = rho_bar_explicit - tau_bar lam / rho^2.
    scales (optional dict): receives "tau" = sum of |terms| of tau_bar and "rho" = of rho_bar_explicit (see
    tvd_fft_torch `terms`): the condition scales of the two cancelling sums; and, with a PSF, "h" = per tap
    |h_bar through H^T y| + |h_bar through C| (the two paths cancel: |h_bar| is ~1/2.7 of that at the c2 and
    128^2 test shapes)."""
    y = torch.as_tensor(y, dtype=dtype).clone().requires_grad_(True)
    lam_v = float(lam)
    rho_t = torch.tensor(float(rho), dtype=dtype, requires_grad=True)
    tau_t = torch.tensor(float(lam) / float(rho), dtype=dtype, requires_grad=True)
    h_t = None
    if h is not None and h.size:
        h_t = torch.as_tensor(h, dtype=dtype).clone().requires_grad_(True)
    terms = {} if scales is not None else None
    h_c = None if (h_t is None or scales is None) else h_t.detach().clone().requires_grad_(True)
    x = tvd_fft_torch(y, torch.tensor(lam_v, dtype=dtype), rho_t, h_t, iso, maxit, masks, tau=tau_t, terms=terms,
                      h_C=h_c)
    (x * torch.as_tensor(xbar, dtype=dtype)).sum().backward()
    hbar = None if h_t is None else h_t.grad.numpy()
    if scales is not None:
        for k in ("tau", "rho"):
            scales[k] = float(sum(t.grad.abs().sum() for t in terms.get(k, []) if t.grad is not None))
        if h_c is not None:
            scales["h"] = h_t.grad.abs().numpy() + h_c.grad.abs().numpy()
            hbar = hbar + h_c.grad.numpy()
    g = lambda t: float(t.grad) if t.grad is not None else 0.0  # noqa: E731
    return (x.detach().numpy(), y.grad.numpy(), hbar, g(tau_t), g(rho_t))
