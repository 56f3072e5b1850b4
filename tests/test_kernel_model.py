"""CPU: the algebra the HIP kernels implement (tests/kernel_model.py: packed half spectra, single-tensor
ADMM state, slot-0 mirror form, spectral H^T y) equals the oracle to fp64 rounding."""
import numpy as np
import pytest

import kernel_model as km
import oracle_np as o


@pytest.mark.parametrize("case", [(2, 1, 16, 32, 5, 4, 6), (1, 2, 64, 64, 9, 9, 10), (1, 1, 8, 4, 0, 0, 3),
                                  (1, 1, 32, 16, 4, 10, 5), (2, 1, 2, 8, 1, 1, 4)])
def test_model_matches_oracle(case):
    B, P, N, M, kh, kw, K = case
    rng = np.random.default_rng(sum(case))
    y = rng.random((B, P, N, M))
    h = rng.random((kw, kh)) if kh else None
    ref = o.to_c(o.tvd_fft_literal(o.from_c(y), 0.05, 0.3, o.psf_from_c(h), False, K)).reshape(B * P, N, M)
    got = km.tvd_model(y.reshape(B * P, N, M), 0.05, 0.3, h, K)
    assert np.abs(got - ref).max() <= 1e-12 * max(1, np.abs(ref).max())


def test_spectral_hty_equals_spatial():
    rng = np.random.default_rng(1)
    y = rng.random((2, 16, 32))
    h = rng.random((5, 6))
    M, N = 32, 16
    kw, kh = h.shape
    padd, padr = (kh - 1) // 2, (kw - 1) // 2
    k = np.arange(M)[None, :]
    kj = np.arange(N)[:, None]
    S = sum(h[b, a] * np.exp(-2j * np.pi * ((a - padd) * k / M + (b - padr) * kj / N))
            for b in range(kw) for a in range(kh))
    spec = np.real(np.fft.ifft2(np.conj(S) * np.fft.fft2(y)))
    assert np.abs(spec - km.ht_c(y, h)).max() < 1e-12
