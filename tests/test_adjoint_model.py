"""CPU: the adjoint restatement the HIP reverse sweep follows (tests/kernel_model.py tvd_model_grads)
against PyTorch fp64 autograd through the unrolled oracle (oracle/oracle_torch.py) -- aniso and iso."""
import numpy as np
import pytest

import oracle_torch
from kernel_model import tvd_model_grads

CASES = [
    # (planes, N, M, psf(kw,kh) or None, lam, rho, K, iso)
    (2, 16, 16, (3, 3), 0.02, 0.1, 5, False),
    (1, 16, 32, None, 0.05, 0.2, 4, False),
    (3, 16, 16, (3, 3), 0.02, 0.1, 5, True),
    (2, 32, 16, None, 0.05, 0.2, 6, True),
    (4, 16, 16, (4, 2), 0.1, 0.3, 3, True),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{'iso' if c[7] else 'aniso'}-{c[0]}x{c[1]}x{c[2]}-K{c[6]}" for c in CASES])
def test_model_grads_match_autograd(case):
    Pl, N, M, psf, lam, rho, K, iso = case
    rng = np.random.default_rng(Pl * 100 + N + K)
    y = rng.random((Pl, N, M))
    h = None
    if psf is not None:
        h = rng.random(psf)
        h /= h.sum()
    xbar = rng.standard_normal((Pl, N, M))
    x0, yb0, hb0, lb0, rb0 = oracle_torch.tvd_fft_grads(y.reshape(Pl, 1, N, M), lam, rho, h, iso, K,
                                                        xbar.reshape(Pl, 1, N, M))
    x1, yb1, hb1, lb1, rb1 = tvd_model_grads(y, lam, rho, h, K, xbar, iso=iso)
    assert np.allclose(x1, x0.reshape(x1.shape), rtol=1e-9, atol=1e-12)
    assert np.allclose(yb1, yb0.reshape(yb1.shape), rtol=1e-7, atol=1e-10)
    assert abs(lb1 - lb0) <= 1e-7 * max(1.0, abs(lb0))
    assert abs(rb1 - rb0) <= 1e-7 * max(1.0, abs(rb0))
    if h is not None:
        assert np.allclose(hb1, hb0, rtol=1e-7, atol=1e-10)
