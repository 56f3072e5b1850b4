"""Numpy model of the HIP kernel decomposition (admm-deconv_amd/csrc/admm_kernels.hip).

Test infrastructure: it restates, in float64 numpy, exactly the algebra the kernels use --
half-length real FFT along dim1 with the (X[0], X[M/2]) slot-0 packing, the column pass with
the mirror form for slot 0, the single-tensor ADMM state s (z = ST(s), u = clip(s)), the
1/(MN) folded into C -- so that the restructuring itself is checked against the oracle
(oracle/oracle_np.py, a restatement of /root/reference/src/ops/ops.jl:17-96) on CPU, before
and independently of the GPU.
"""
import numpy as np


def _pack_forward(v):
    """v: (..., N, M) real lines -> packed half spectrum (..., N, M/2) complex (kernel pack_forward_store)."""
    M = v.shape[-1]
    L = M // 2
    z = v[..., 0::2] + 1j * v[..., 1::2]
    Z = np.fft.fft(z, axis=-1)
    k = np.arange(L)
    Zm = np.conj(Z[..., (L - k) % L])
    E = 0.5 * (Z + Zm)
    O = (Z - Zm) / 2j
    X = E + np.exp(-2j * np.pi * k / M) * O
    X[..., 0] = (Z[..., 0].real + Z[..., 0].imag) + 1j * (Z[..., 0].real - Z[..., 0].imag)
    return X


def _unpack_inverse(X):
    """packed (..., N, L) -> real lines (..., N, 2L), unnormalised inverse (kernel unpack_inverse + IFFT)."""
    L = X.shape[-1]
    M = 2 * L
    k = np.arange(L)
    Xm = np.conj(X[..., (L - k) % L])
    E = X + Xm
    O = (X - Xm) * np.exp(2j * np.pi * k / M)
    Z = E + 1j * O
    a, b = X[..., 0].real, X[..., 0].imag
    Z[..., 0] = (a + b) + 1j * (a - b)
    z = np.fft.ifft(Z, axis=-1) * L          # unnormalised
    out = np.empty(X.shape[:-1] + (M,))
    out[..., 0::2] = z.real
    out[..., 1::2] = z.imag
    return out


def make_Cmat(M, N, rho, h_c):
    """Cmat[k][kj], k = 0..M/2 (setup_kernel), with 1/(MN) folded in.  h_c is C-layout (kw, kh)."""
    L = M // 2
    k = np.arange(L + 1)[:, None]
    kj = np.arange(N)[None, :]
    if h_c is None or np.size(h_c) == 0:
        s2 = 1.0
    else:
        kw, kh = h_c.shape
        S = np.zeros((L + 1, N), complex)
        for b in range(kw):
            for a in range(kh):
                S += h_c[b, a] * np.exp(-2j * np.pi * (a * k / M + b * kj / N))
        s2 = np.abs(S) ** 2
    lap = 4 * np.sin(np.pi * kj / N) ** 2 + 4 * np.sin(np.pi * k / M) ** 2
    return 1.0 / (M * N) / (s2 + rho * lap)


def _column(W, Cm):
    """W: (..., N, L) packed -> FFT_j, xC (slot 0 mirror form), IFFT_j (unnormalised)."""
    N, L = W.shape[-2:]
    Z = np.fft.fft(W, axis=-2)
    out = Z * Cm[:L].T[None] if Z.ndim == 3 else Z * Cm[:L].T
    z0 = Z[..., :, 0]
    kj = np.arange(N)
    zm = np.conj(z0[..., (N - kj) % N])
    c0, cL = Cm[0], Cm[L]
    out[..., :, 0] = 0.5 * (c0 + cL) * z0 + 0.5 * (c0 - cL) * zm
    return np.fft.ifft(out, axis=-2) * N


def ht_c(y, h_c):
    """H^T y on C-layout planes (..., N, M); h_c (kw, kh)."""
    if h_c is None or np.size(h_c) == 0:
        return y.copy()
    kw, kh = h_c.shape
    padd, padr = (kh - 1) // 2, (kw - 1) // 2
    out = np.zeros_like(y)
    for b in range(kw):
        for a in range(kh):
            out += h_c[b, a] * np.roll(y, shift=(-(b - padr), -(a - padd)), axis=(-2, -1))
    return out


def tvd_model(y_c, lam, rho, h_c, maxit):
    """y_c: (planes, N, M) float -> x (planes, N, M), following the kernel sequence."""
    y = np.asarray(y_c, np.float64)
    P_, N, M = y.shape
    tau = lam / rho
    if maxit == 0:
        return np.zeros_like(y)
    Cm = make_Cmat(M, N, rho, h_c)
    hty = ht_c(y, h_c)
    spec0 = _pack_forward(hty)                 # PREP
    s = np.zeros((P_, 2, N, M))
    for it in range(1, maxit + 1):
        spec1 = _column(spec0, Cm)             # COLUMN
        x = _unpack_inverse(spec1)
        if it == maxit:
            return x                           # FINAL
        u = np.clip(s, -tau, tau)              # LINE
        s0 = x - np.roll(x, 1, axis=-2) + u[:, 0]
        s1 = x - np.roll(x, 1, axis=-1) + u[:, 1]
        s = np.stack([s0, s1], axis=1)
        w = np.where(np.abs(s) > tau, s - 2 * tau * np.sign(s), -s)
        v = hty + rho * ((w[:, 0] - np.roll(w[:, 0], -1, axis=-2)) + (w[:, 1] - np.roll(w[:, 1], -1, axis=-1)))
        spec0 = _pack_forward(v)
