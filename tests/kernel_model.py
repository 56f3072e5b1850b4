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


# ---------------------------------------------------------------------------------------------
# Adjoint (reverse sweep) model -- what the backward kernels implement (aniso).
# Forward trajectory: s_k (k = 1..K-1), x_K.  phi(s) = z - u = ST(s) - clip(s), psi(s) = clip(s).
# Step k = K..1:  vbar_k = A^-1 g_k ;  Dvb = D vbar_k
#   rho_bar += -<Dvb, D x_k>            (D x_k = s_k - psi(s_{k-1}), or D(x_K) for k = K)
#   k >= 2: wbar = rho Dvb ; rho_bar += <phi(s_{k-1}), Dvb>
#           sbar_{k-1} = phi'(s_{k-1}) wbar + psi'(s_{k-1}) sbar_k ; tau_bar += dphi/dtau wbar + dpsi/dtau sbar_k
#           g_{k-1} = D^T sbar_{k-1}
#   Vsum += vbar_k ;  Q += Re(conj(G_k) V_k) (spectra of g_k and v_k, for h_bar)
# Final: ybar = H Vsum ; h_bar = dHt/dh . (Vsum, y) - (1/MN) sum_nu C^2 Q d|Sigma|^2/dh ;
#        lam_bar = tau_bar/rho ; rho_bar += -tau_bar lam/rho^2 - (1/MN) sum_nu C^2 Q Lambda  [rho in C]
# ---------------------------------------------------------------------------------------------
def _Dop(x):
    return x - np.roll(x, 1, axis=-2), x - np.roll(x, 1, axis=-1)


def _Dt(a, b):
    return (a - np.roll(a, -1, axis=-2)) + (b - np.roll(b, -1, axis=-1))


def tvd_model_grads(y_c, lam, rho, h_c, K, xbar, iso=False, batch_sum=None):
    """y_c (planes, N, M); returns (x, ybar, hbar, lam_bar, rho_bar) following the kernel reverse sweep.

    iso: the BT prox z = f s, f = max(1 - tau/Nrm, 0), Nrm(pixel) = sqrt(sum over all planes and both
    channels of s^2) (ops.jl:6,10).  Then w = phi(s) = (2f-1) s, u = psi(s) = (1-f) s, and the reverse
    step gains a per-pixel batch reduction R = sum_{planes,channels} s (2 wbar - sbar):
        sbar_{k-1} = (2f-1) wbar + (1-f) sbar_k + [Nrm > tau] (tau/Nrm^3) R s
        tau_bar   += sum_pixels [Nrm > tau] (-R/Nrm).
    batch_sum: for a batch sharded over processes, maps this shard's (N, M) per-pixel partial sum to the
    whole batch's (the admm_batch_reducer contract); tau_bar then uses the shard's own R, so the
    scalar gradients are this shard's contributions."""
    batch_sum = batch_sum or (lambda a: a)
    y = np.asarray(y_c, np.float64)
    Pl, N, M = y.shape
    tau = lam / rho
    hty = ht_c(y, h_c)
    # full-spectrum C (N, M) for A^-1 (normalised irfft2 convention)
    k = np.arange(M)[None, :]
    kj = np.arange(N)[:, None]
    lapf = 4 * np.sin(np.pi * kj / N) ** 2 + 4 * np.sin(np.pi * k / M) ** 2
    if h_c is None or np.size(h_c) == 0:
        S = np.ones((N, M), complex)
    else:
        kw, kh = h_c.shape
        S = sum(h_c[b, a] * np.exp(-2j * np.pi * (a * k / M + b * kj / N)) for b in range(kw) for a in range(kh))
    Cf = 1.0 / (np.abs(S) ** 2 + rho * lapf)
    Ainv = lambda v: np.real(np.fft.ifft2(Cf * np.fft.fft2(v)))   # noqa: E731

    def fmap(sk):
        with np.errstate(divide="ignore"):
            nrm = np.sqrt(batch_sum(np.sum(sk * sk, axis=(0, 1))))
            return np.maximum(1 - tau / nrm, 0.0), nrm

    def phi(sk, f=None):
        if iso:
            return (2 * f - 1) * sk
        return np.where(np.abs(sk) > tau, sk - 2 * tau * np.sign(sk), -sk)

    def psi(sk, f=None):
        if iso:
            return (1 - f) * sk
        return np.clip(sk, -tau, tau)

    # forward with trajectory
    s = [np.zeros((2, Pl, N, M))]
    fs = [np.zeros((N, M))]
    nrms = [np.zeros((N, M))]
    vs = []
    w = np.zeros((2, Pl, N, M))
    u = np.zeros((2, Pl, N, M))
    for it in range(1, K + 1):
        v = hty + rho * _Dt(w[0], w[1])
        vs.append(v)
        x = Ainv(v)
        if it == K:
            break
        d0, d1 = _Dop(x)
        sk = np.stack([d0 + u[0], d1 + u[1]])
        f, nrm = fmap(sk) if iso else (None, None)
        s.append(sk)
        fs.append(f)
        nrms.append(nrm)
        w, u = phi(sk, f), psi(sk, f)
    xK = x
    # reverse sweep
    g = np.asarray(xbar, np.float64).reshape(Pl, N, M)
    sbar = np.zeros((2, Pl, N, M))
    rho_bar = tau_bar = 0.0
    Vsum = np.zeros_like(y)
    Q = np.zeros((N, M))
    for it in range(K, 0, -1):
        vbar = Ainv(g)
        Vsum += vbar
        Q += np.sum(np.real(np.conj(np.fft.fft2(g)) * np.fft.fft2(vs[it - 1])), axis=0)
        dv0, dv1 = _Dop(vbar)
        if it == K:
            dx0, dx1 = _Dop(xK)
        else:
            up = psi(s[it - 1], fs[it - 1])
            dx0, dx1 = s[it][0] - up[0], s[it][1] - up[1]
        rho_bar -= np.sum(dv0 * dx0 + dv1 * dx1)
        if it >= 2:
            sp = s[it - 1]
            dv = np.stack([dv0, dv1])
            wb = rho * dv
            rho_bar += np.sum(phi(sp, fs[it - 1]) * dv)
            if iso:
                f, nrm = fs[it - 1], nrms[it - 1]
                R = np.sum(sp * (2 * wb - sbar), axis=(0, 1))
                act = nrm > tau
                with np.errstate(divide="ignore", invalid="ignore"):
                    tau_bar += np.sum(np.where(act, -R / nrm, 0.0))
                    R = batch_sum(R)
                    coef = np.where(act, tau / nrm ** 3 * R, 0.0)
                sbar_new = (2 * f - 1) * wb + (1 - f) * sbar + coef * sp
            else:
                m = np.abs(sp) > tau
                sbar_new = np.where(m, wb, -wb + sbar)
                tau_bar += np.sum(np.where(m, -2 * np.sign(sp) * wb + np.sign(sp) * sbar, 0.0))
            sbar = sbar_new
            g = _Dt(sbar[0], sbar[1])
    # final assembly
    if h_c is None or np.size(h_c) == 0:
        ybar = Vsum
        hbar = None
    else:
        kw, kh = h_c.shape
        padd, padr = (kh - 1) // 2, (kw - 1) // 2
        ybar = np.zeros_like(y)
        hbar = np.zeros((kw, kh))
        for b in range(kw):
            for a in range(kh):
                ybar += h_c[b, a] * np.roll(Vsum, shift=(b - padr, a - padd), axis=(-2, -1))
                hbar[b, a] += np.sum(Vsum * np.roll(y, shift=(-(b - padr), -(a - padd)), axis=(-2, -1)))
                dS = 2 * np.real(np.conj(S) * np.exp(-2j * np.pi * (a * k / M + b * kj / N)))
                hbar[b, a] -= np.sum(Cf ** 2 * Q * dS) / (M * N)
    rho_bar_spec = -np.sum(Cf ** 2 * Q * lapf) / (M * N)   # equals the spatial -<Dvb, Dx> sum (cross-check)
    lam_bar = tau_bar / rho
    rho_bar -= tau_bar * lam / rho ** 2
    tvd_model_grads.rho_bar_spec_check = rho_bar_spec
    return xK, ybar, hbar, lam_bar, rho_bar
