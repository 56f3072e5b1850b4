"""CPU oracle for the ADMM TV-deconvolution solve (`tvd_fft`) -- TEST INFRASTRUCTURE ONLY.

This module is a numpy restatement of the reference Julia solver
`/root/reference/src/ops/ops.jl:17-96` (`tvd_fft_cpu`; the GPU twin `:99-178` has the
same semantics).  It exists to CHECK the HIP path: only `tests/`, `__graft_entry__.smoke()`
and `bench.py`'s `cpu_baseline` leg may import it.  The product path never routes through it.

Parity status: **parity unpinned**.  The reference is Julia (absent here and on the GPU box),
ships no golden vectors and its only test (`src/tests/admm_deconv_test.jl`) asserts nothing
(SURVEY.md s4, s8c).  The restatement is therefore pinned by two independent forms that must
agree to fp64 rounding (`tvd_fft_literal`: spatial stencils / correlation exactly as the
reference's NNlib convs compute them; `tvd_fft_spectral`: every linear operator applied in the
Fourier domain), by operator identities (D/D^T and H/H^T adjointness), and by the committed
fixtures in `tests/golden/` that were produced from `tvd_fft_literal` (fp64 on fp32 inputs).

Array convention.  Functions here take arrays in the reference's Julia axis order
(M, N, P, B) = (dim1 contiguous, dim2, channel, batch).  A C array `float[B][P][N][M]` (the
C-ABI layout, see include/admm_deconv.h) is the numpy C-order array of shape (B, P, N, M);
`from_c`/`to_c` convert by transposition (no copy).  The PSF `h` is Julia (kh, kw) <-> C
`float[kw][kh]`.
"""
from __future__ import annotations

import numpy as np

__all__ = [
    "from_c", "to_c", "psf_from_c", "ST", "BT", "pixelnorm", "make_C",
    "D_op", "Dt_op", "H_op", "Ht_op", "prox_active_fraction", "tvd_fft_literal", "tvd_fft_spectral", "tvd_fft",
]


# ----------------------------------------------------------------------------------------------
# layout helpers
# ----------------------------------------------------------------------------------------------
def from_c(a):
    """C-order (B,P,N,M) -> Julia-order view (M,N,P,B)."""
    return np.asarray(a).transpose(3, 2, 1, 0)


def to_c(a):
    """Julia-order (M,N,P,B) -> C-order (B,P,N,M) contiguous copy."""
    return np.ascontiguousarray(np.asarray(a).transpose(3, 2, 1, 0))


def psf_from_c(h_c):
    """C `float[kw][kh]` (numpy (kw,kh)) -> Julia (kh,kw)."""
    if h_c is None:
        return None
    h_c = np.asarray(h_c)
    if h_c.size == 0:
        return np.zeros((0, 0))
    return h_c.T


# ----------------------------------------------------------------------------------------------
# prox operators  (ops.jl:6-10)
# ----------------------------------------------------------------------------------------------
def pixelnorm(x):
    """ops.jl:6  sqrt(sum(x.^2, dims=(3,4))) -- over ALL channels of the whole batch."""
    return np.sqrt(np.sum(x * x, axis=(2, 3), keepdims=True))


def ST(x, tau):
    """ops.jl:9 soft-thresholding: sign(x) * max(|x| - tau, 0)."""
    return np.sign(x) * np.maximum(np.abs(x) - tau, 0.0)


def BT(x, tau):
    """ops.jl:10 block-thresholding: max(1 - tau / pixelnorm(x), 0) * x.

    Julia's `max` propagates NaN (tau = 0 and a zero pixel-vector gives 0/0 = NaN, which
    survives the max); numpy's np.maximum propagates NaN too, so the quirk is reproduced."""
    with np.errstate(divide="ignore", invalid="ignore"):
        f = np.maximum(1.0 - tau / pixelnorm(x), 0.0)
    return f * x


# ----------------------------------------------------------------------------------------------
# linear operators, spatial form (ops.jl:52-82)
# Arrays here are (M, N, C, P) as after the permute at ops.jl:19.
# ----------------------------------------------------------------------------------------------
def D_op(x):
    """ops.jl:52-54,62,64: grouped 2x2 conv on pad_circular(x,(1,0,1,0)).
    Output channel 2g-1 = x[i,j]-x[i,j-1] (dim2), 2g = x[i,j]-x[i-1,j] (dim1), periodic."""
    M, N, Bc, P = x.shape
    out = np.empty((M, N, 2 * Bc, P), dtype=x.dtype)
    out[:, :, 0::2, :] = x - np.roll(x, 1, axis=1)
    out[:, :, 1::2, :] = x - np.roll(x, 1, axis=0)
    return out


def Dt_op(z):
    """ops.jl:56-59,63,65: conv on pad_circular(z,(0,1,0,1)) with W^T.
    (z1[i,j]-z1[i,j+1]) + (z2[i,j]-z2[i+1,j]); the exact adjoint of D_op."""
    z1 = z[:, :, 0::2, :]
    z2 = z[:, :, 1::2, :]
    return (z1 - np.roll(z1, -1, axis=1)) + (z2 - np.roll(z2, -1, axis=0))


def _pads(h):
    kh, kw = h.shape
    padu, padd = int(np.ceil((kh - 1) / 2)), (kh - 1) // 2     # ops.jl:73
    padl, padr = int(np.ceil((kw - 1) / 2)), (kw - 1) // 2     # ops.jl:74
    return padu, padd, padl, padr


def Ht_op(x, h):
    """ops.jl:72-81 H^T = conv(pad_circular(x, pad2), reverse(h)):
    out[i,j] = sum_{a,b} h[a,b] * x[i+a-1-padd, j+b-1-padr]  (1-based; periodic)."""
    kh, kw = h.shape
    _, padd, _, padr = _pads(h)
    out = np.zeros_like(x)
    for a in range(kh):
        for b in range(kw):
            w = h[a, b]
            if w == 0.0:
                continue
            out += w * np.roll(x, shift=(-(a - padd), -(b - padr)), axis=(0, 1))
    return out


def H_op(x, h):
    """ops.jl:80 H = conv(pad_circular(x, pad1), h): centred circular convolution.
    out[i,j] = sum_{a,b} h[a,b] * x[i-(a-1)+padd, j-(b-1)+padr]."""
    kh, kw = h.shape
    _, padd, _, padr = _pads(h)
    out = np.zeros_like(x)
    for a in range(kh):
        for b in range(kw):
            w = h[a, b]
            if w == 0.0:
                continue
            out += w * np.roll(x, shift=(a - padd, b - padr), axis=(0, 1))
    return out


def _rfft12(v):
    """FFTW rfft over dims (1,2), halving dim1 (ops.jl:26,35,86)."""
    return np.fft.rfftn(v, axes=(1, 0))


def _irfft12(V, M, N):
    """FFTW irfft(., M, (1,2)) normalised by 1/(MN) (ops.jl:86)."""
    return np.fft.irfftn(V, s=(N, M), axes=(1, 0))


def make_C(M, N, rho, h):
    """ops.jl:22-37  C = 1 / (|Sigma|^2 + rho(|Lx|^2 + |Ly|^2)), shape (M//2+1, N)."""
    if h is None or np.size(h) == 0:
        sig2 = 1.0                                               # ops.jl:23
    else:
        hh = np.zeros((M, N), dtype=np.float64)                  # pad_constant top-left :25
        kh, kw = h.shape
        hh[:kh, :kw] = h
        sig2 = np.abs(_rfft12(hh)) ** 2
    dx = np.zeros((M, N)); dx[0, 0] = 1.0; dx[0, 1] = -1.0       # ops.jl:32
    dy = np.zeros((M, N)); dy[0, 0] = 1.0; dy[1, 0] = -1.0       # ops.jl:34
    lx = np.abs(_rfft12(dx)) ** 2
    ly = np.abs(_rfft12(dy)) ** 2
    return 1.0 / (sig2 + rho * (lx + ly))


def _check(y, lam, rho, maxit):
    y = np.asarray(y)
    if y.ndim != 4:
        raise ValueError("y must be 4-D (M,N,P,B)")
    return np.asarray(y, dtype=np.float64)


def _record_prox(stats, z, maxit, k):
    """stats['prox_active'][k] = fraction of non-zero prox outputs z_k (ST/BT, ops.jl:89).  The K-th
    iteration's z is dead (ops.jl:84-93), so only iterations 1..K-1 are recorded: a case whose fractions are
    all 0 exercises only the linear part of the solve."""
    if stats is not None and k < maxit - 1:
        stats.setdefault("prox_active", []).append(float(np.count_nonzero(z)) / z.size)


def prox_active_fraction(stats):
    """Mean fraction of live prox outputs over the iterations that reach the output (0 when none do)."""
    a = stats.get("prox_active", [])
    return float(np.mean(a)) if a else 0.0


def tvd_fft_literal(y, lam, rho, h=None, isotropic=False, maxit=100, stats=None):
    """Op-for-op restatement of ops.jl:17-96 in fp64 (spatial stencils, spatial H^T).

    y: (M,N,P,B) Julia-order array; lam, rho: scalars; h: (kh,kw) PSF or None/empty.
    stats: optional dict, filled by _record_prox.
    Returns x of shape (M,N,P,B) float64."""
    y = _check(y, lam, rho, maxit)
    M, N, P, B = y.shape
    lam = float(np.asarray(lam, dtype=np.float64).ravel()[0])
    rho = float(np.asarray(rho, dtype=np.float64).ravel()[0])
    yp = y.transpose(0, 1, 3, 2)                                 # ops.jl:19 (M,N,B,P)
    tau = lam / rho                                              # ops.jl:20
    hj = None if h is None or np.size(h) == 0 else np.asarray(h, dtype=np.float64)
    C = make_C(M, N, rho, hj)[:, :, None, None]                  # ops.jl:37
    thresh = BT if isotropic else ST                             # ops.jl:39-43
    x = np.zeros((M, N, B, P))                                   # ops.jl:46-49
    z = np.zeros((M, N, 2 * B, P))
    u = np.zeros((M, N, 2 * B, P))
    # H^T(y) is loop-invariant; the reference re-evaluates it every iteration (ops.jl:86)
    # and gets the identical array each time, so evaluating it once is exact.
    hty = yp.copy() if hj is None else Ht_op(yp, hj)
    for k in range(maxit):                                       # ops.jl:84-92
        x = _irfft12(C * _rfft12(hty + rho * Dt_op(z - u)), M, N)
        Dxk = D_op(x)
        z = thresh(Dxk + u, tau)
        _record_prox(stats, z, maxit, k)
        u = u + Dxk - z
    return x.transpose(0, 1, 3, 2)                               # ops.jl:93


def tvd_fft_spectral(y, lam, rho, h=None, isotropic=False, maxit=100, stats=None):
    """Independent form: D, D^T and H^T applied as Fourier multipliers (cross-check)."""
    y = _check(y, lam, rho, maxit)
    M, N, P, B = y.shape
    lam = float(np.asarray(lam, dtype=np.float64).ravel()[0])
    rho = float(np.asarray(rho, dtype=np.float64).ravel()[0])
    yp = y.transpose(0, 1, 3, 2)
    tau = lam / rho
    k1 = np.arange(M // 2 + 1)[:, None]
    k2 = np.arange(N)[None, :]
    e1 = np.exp(-2j * np.pi * k1 / M)            # shift by one along dim1
    e2 = np.exp(-2j * np.pi * k2 / N)            # shift by one along dim2
    L1 = (1.0 - e2)[:, :, None, None]            # ch1 multiplier (dim2 difference)
    L2 = (1.0 - e1)[:, :, None, None]            # ch2 multiplier (dim1 difference)
    hj = None if h is None or np.size(h) == 0 else np.asarray(h, dtype=np.float64)
    if hj is None:
        Sig = np.ones((M // 2 + 1, N), dtype=np.complex128)
        Sc = Sig
    else:
        kh, kw = hj.shape
        _, padd, _, padr = _pads(hj)
        a = np.arange(kh)[:, None, None, None]
        b = np.arange(kw)[None, :, None, None]
        ph = np.exp(-2j * np.pi * (a * k1[None, None] / M + b * k2[None, None] / N))
        Sig = np.sum(hj[:, :, None, None] * ph, axis=(0, 1))                  # top-left PSF
        phc = np.exp(-2j * np.pi * ((a - padd) * k1[None, None] / M + (b - padr) * k2[None, None] / N))
        Sc = np.sum(hj[:, :, None, None] * phc, axis=(0, 1))                  # centred PSF
    lx = np.abs(1.0 - np.exp(-2j * np.pi * k2 / N)) ** 2
    ly = np.abs(1.0 - np.exp(-2j * np.pi * k1 / M)) ** 2
    C = (1.0 / (np.abs(Sig) ** 2 + rho * (lx + ly)))[:, :, None, None]
    thresh = BT if isotropic else ST
    Y = _rfft12(yp)
    HtY = np.conj(Sc)[:, :, None, None] * Y
    Bsz = B
    z = np.zeros((M, N, 2 * Bsz, P))
    u = np.zeros((M, N, 2 * Bsz, P))
    x = np.zeros((M, N, Bsz, P))
    for k in range(maxit):
        w = z - u
        W1 = _rfft12(w[:, :, 0::2, :])
        W2 = _rfft12(w[:, :, 1::2, :])
        V = HtY + rho * (np.conj(L1) * W1 + np.conj(L2) * W2)
        X = C * V
        x = _irfft12(X, M, N)
        Dx = np.empty((M, N, 2 * Bsz, P))
        Dx[:, :, 0::2, :] = _irfft12(L1 * X, M, N)
        Dx[:, :, 1::2, :] = _irfft12(L2 * X, M, N)
        z = thresh(Dx + u, tau)
        _record_prox(stats, z, maxit, k)
        u = u + Dx - z
    return x.transpose(0, 1, 3, 2)


# default oracle
tvd_fft = tvd_fft_literal


# ----------------------------------------------------------------------------------------------
# layer epilogue (src/layers/deconv_admm.jl:215-225)
# ----------------------------------------------------------------------------------------------
def admm_layer_forward(x, lam, rho, weight, iso, iters, creg=0.0, bias=None, act=None):
    """Restates `(d::Admm)(x)`: clamp lam/rho to [creg, Inf), clamp PSF to [0,1], solve, +bias, act."""
    lam = max(float(lam), float(creg))
    rho = max(float(rho), float(creg))
    w = None if weight is None or np.size(weight) == 0 else np.clip(np.asarray(weight, np.float64), 0.0, 1.0)
    res = tvd_fft_literal(x, lam, rho, w, iso, iters)
    if bias is not None and bias is not False:
        res = res + float(np.asarray(bias).ravel()[0])
    return res if act is None else act(res)
