"""CPU: the oracle (restatement of /root/reference/src/ops/ops.jl:17-96) checked against itself two ways,
against its C twin, against operator identities and against the committed golden fixtures.
Parity vs Julia itself is unpinned (Julia absent; the reference ships no vectors) -- DESIGN.md."""
import glob
import json
import os

import numpy as np
import pytest

import oracle_c
import oracle_np as o
from parity import PROX_MIN_FRACTION

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rand_case(seed, B=2, P=1, N=32, M=16, kh=5, kw=4):
    rng = np.random.default_rng(seed)
    y = rng.random((B, P, N, M)).astype(np.float32)
    h = None
    if kh:
        h = rng.random((kw, kh)).astype(np.float32)
        h /= h.sum()
    return y, h


@pytest.mark.parametrize("iso", [False, True])
@pytest.mark.parametrize("shape", [(2, 1, 32, 16, 5, 4), (1, 2, 16, 32, 10, 10), (3, 1, 8, 8, 0, 0),
                                   (1, 1, 12, 10, 3, 2)])
def test_literal_equals_spectral(shape, iso):
    B, P, N, M, kh, kw = shape
    y, h = rand_case(sum(shape), B, P, N, M, kh, kw)
    a = o.tvd_fft_literal(o.from_c(y), 0.02, 0.1, o.psf_from_c(h), iso, 6)
    b = o.tvd_fft_spectral(o.from_c(y), 0.02, 0.1, o.psf_from_c(h), iso, 6)
    assert np.abs(a - b).max() <= 1e-12 * max(1.0, np.abs(a).max())


@pytest.mark.parametrize("iso", [False, True])
def test_c_oracle_f64_matches_numpy(iso):
    y, h = rand_case(7, B=2, P=2, N=32, M=32, kh=7, kw=7)
    ref = o.to_c(o.tvd_fft_literal(o.from_c(y), 0.0041, 0.021, o.psf_from_c(h), iso, 8))
    got = oracle_c.tvd_fft_c(y, 0.0041, 0.021, h, iso, 8, np.float64, nthreads=2)
    assert np.abs(got - ref).max() <= 1e-11


def test_c_oracle_f32_within_parity():
    y, h = rand_case(8, B=2, P=1, N=64, M=64, kh=9, kw=9)
    ref = o.to_c(o.tvd_fft_literal(o.from_c(y), 0.0041, 0.021, o.psf_from_c(h), False, 10))
    got = oracle_c.tvd_fft_c(y, 0.0041, 0.021, h, False, 10, np.float32, nthreads=2)
    for b in range(2):
        assert np.linalg.norm(got[b] - ref[b]) / np.linalg.norm(ref[b]) < 1e-5


def test_D_adjoint():
    rng = np.random.default_rng(0)
    x = rng.random((16, 8, 3, 2))
    z = rng.random((16, 8, 6, 2))
    assert abs(np.sum(o.D_op(x) * z) - np.sum(x * o.Dt_op(z))) < 1e-10


@pytest.mark.parametrize("k", [(1, 1), (3, 3), (4, 4), (10, 10), (4, 9), (15, 15)])
def test_H_adjoint(k):
    rng = np.random.default_rng(sum(k))
    h = rng.random(k)
    x = rng.random((32, 24, 2, 1))
    w = rng.random((32, 24, 2, 1))
    lhs, rhs = np.sum(o.H_op(x, h) * w), np.sum(x * o.Ht_op(w, h))
    assert abs(lhs - rhs) <= 1e-10 * abs(lhs)


def test_first_iterate_is_wiener_like():
    """z = u = 0 initially, so x_1 = irfft(C .* rfft(H^T y)) (ops.jl:86)."""
    y, h = rand_case(3, B=1, N=16, M=16, kh=3, kw=3)
    yj = o.from_c(y.astype(np.float64)).transpose(0, 1, 3, 2)
    hj = o.psf_from_c(h.astype(np.float64))
    C = o.make_C(16, 16, 0.1, hj)[:, :, None, None]
    x1 = np.fft.irfftn(C * np.fft.rfftn(o.Ht_op(yj, hj), axes=(1, 0)), s=(16, 16), axes=(1, 0))
    got = o.tvd_fft_literal(o.from_c(y), 0.02, 0.1, o.psf_from_c(h), False, 1)
    assert np.abs(got - x1.transpose(0, 1, 3, 2)).max() < 1e-12


def test_maxit_zero_and_empty_psf():
    y, _ = rand_case(4)
    assert np.all(o.tvd_fft_literal(o.from_c(y), 0.1, 1.0, None, False, 0) == 0)
    a = o.tvd_fft_literal(o.from_c(y), 0.1, 1.0, None, False, 3)
    b = o.tvd_fft_literal(o.from_c(y), 0.1, 1.0, np.zeros((0, 0)), False, 3)
    assert np.array_equal(a, b)


def test_iso_nan_quirk():
    """BT with tau = 0 and a zero pixel-vector is 0/0 = NaN in the reference (ops.jl:10, Julia max)."""
    s = np.zeros((2, 2, 2, 1))
    s[0, 0] = 1.0
    z = o.BT(s, 0.0)
    assert np.isnan(z[1, 1]).all() and np.all(z[0, 0] == 1.0)


def test_st_and_pixelnorm():
    x = np.array([-3.0, -0.5, 0.0, 0.5, 3.0]).reshape(5, 1, 1, 1)
    assert np.allclose(o.ST(x, 1.0).ravel(), [-2, 0, 0, 0, 2])
    v = np.ones((1, 1, 4, 2))
    assert np.allclose(o.pixelnorm(v), np.sqrt(8.0))   # over ALL channels and P (dims 3,4)


def test_prox_stats_separate_linear_from_live_cases():
    """oracle_np's prox statistics (tests/parity.py assert_prox_active): K = 1 records nothing (the K-th z is
    dead); the reference demo shape (32 x 32 PSF on 32 x 32 crops, src/ADMM_Deconv.jl:17-23) at tau = 0.05 / 0.3
    never fires (every |Dx| is below tau), at tau = 0.0005 / 0.3 it does; the two forms agree."""
    from admm_deconv import synth
    rng = np.random.default_rng(2 * 1000 + 32 + 32 + 50)
    h = rng.random((32, 32)).astype(np.float32)
    h = (h / h.sum()).astype(np.float32)
    y = synth.make_batch(2, 32, 32, h, P=3, g0=7).astype(np.float64)
    fr = {}
    for lam in (0.05, 0.0005):
        for f in (o.tvd_fft_literal, o.tvd_fft_spectral):
            st = {}
            f(o.from_c(y), np.float32(lam), np.float32(0.3), o.psf_from_c(h), False, 50, stats=st)
            assert len(st["prox_active"]) == 49
            fr[lam, f.__name__] = o.prox_active_fraction(st)
    assert fr[0.05, "tvd_fft_literal"] == 0.0 == fr[0.05, "tvd_fft_spectral"]
    assert fr[0.0005, "tvd_fft_literal"] >= PROX_MIN_FRACTION
    assert abs(fr[0.0005, "tvd_fft_literal"] - fr[0.0005, "tvd_fft_spectral"]) < 1e-3
    st = {}
    o.tvd_fft_literal(o.from_c(y), np.float32(0.0005), np.float32(0.3), o.psf_from_c(h), False, 1, stats=st)
    assert o.prox_active_fraction(st) == 0.0


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "*.npz"))), ids=os.path.basename)
def test_golden_fixture_reproduces(path):
    d = np.load(path)   # allow_pickle=False (default)
    p = json.loads(str(d["params"]))
    h = d["h"] if d["h"].size else None
    st = {}
    x = o.to_c(o.tvd_fft_literal(o.from_c(d["y"].astype(np.float64)), np.float32(p["lam"]), np.float32(p["rho"]),
                                 o.psf_from_c(h), p["iso"], p["K"], stats=st))
    assert np.abs(x - d["x"]).max() <= 1e-6 * max(1.0, np.abs(x).max())
    # every fixture pins the nonlinear solve: its prox fired
    assert o.prox_active_fraction(st) >= PROX_MIN_FRACTION, (path, o.prox_active_fraction(st))
    if p["M"] * p["N"] <= 64 * 128:
        c = oracle_c.tvd_fft_c(d["y"], p["lam"], p["rho"], h, p["iso"], p["K"], np.float64, nthreads=2)
        assert np.abs(c - d["x"]).max() <= 1e-6 * max(1.0, np.abs(c).max())


@pytest.mark.parametrize("iso", [False, True])
def test_mask_conditioned_oracle_equals_oracle_on_its_own_masks(iso):
    """The gradient oracle with the prox branches held at the masks of its OWN fp64 forward is the plain
    oracle (the masked prox is the exact prox there), bitwise in x and to fp64 rounding in every gradient;
    with one mask bit flipped it is not (the conditioning has an effect)."""
    import torch
    import oracle_torch as ot
    from admm_deconv import synth
    rng = np.random.default_rng(4)
    h = synth.gaussian_psf(5, 1.0)
    y = synth.make_batch(2, 24, 20, h, P=1).astype(np.float64)
    xbar = rng.standard_normal(y.shape)
    lam, rho, K = np.float32(0.02), np.float32(0.1), 6
    rec = []
    ot.tvd_fft_torch(torch.from_numpy(y), torch.tensor(float(lam), dtype=torch.float64),
                     torch.tensor(float(rho), dtype=torch.float64), torch.from_numpy(h.astype(np.float64)), iso, K,
                     record=rec)
    assert len(rec) == K - 1
    s_traj = np.stack([r[0].numpy() for r in rec])
    n_traj = np.stack([r[1].numpy() for r in rec])
    masks = ot.masks_from_trajectory(s_traj, lam, rho, iso, n_traj)
    a = ot.tvd_fft_grads(y, lam, rho, h.astype(np.float64), iso, K, xbar)
    b = ot.tvd_fft_grads(y, lam, rho, h.astype(np.float64), iso, K, xbar, masks=masks)
    assert np.allclose(a[0], b[0], rtol=0, atol=1e-13)
    for u, v in zip(a[1:], b[1:]):
        assert np.allclose(u, v, rtol=1e-10, atol=1e-13)
    # flip the mask of one pixel of iteration 2
    m0 = masks[1][0] if not iso else masks[1]
    flip = np.unravel_index(np.argmax(m0), m0.shape)
    if iso:
        masks[1] = masks[1].copy()
        masks[1][flip] = 0.0
    else:
        m, sg = masks[1][0].copy(), masks[1][1]
        m[flip] = 0.0
        masks[1] = (m, sg)
    c = ot.tvd_fft_grads(y, lam, rho, h.astype(np.float64), iso, K, xbar, masks=masks)
    assert not np.allclose(a[1], c[1], rtol=1e-8, atol=1e-12)


@pytest.mark.parametrize("iso", [False, True])
def test_split_gradients_and_term_scales(iso):
    """tau as its own variable reproduces lambda_bar / rho_bar (lam_bar = tau_bar / rho, rho_bar =
    rho_bar_explicit - tau_bar lam / rho^2), and the per-use copies of rho / tau (the term scales) change no
    gradient; each scale bounds its sum from above."""
    import torch
    import oracle_torch as ot
    from admm_deconv import synth
    rng = np.random.default_rng(8)
    h = synth.gaussian_psf(5, 1.0).astype(np.float64)
    y = synth.make_batch(2, 20, 16, h.astype(np.float32), P=1).astype(np.float64)
    xbar = rng.standard_normal(y.shape)
    lam, rho, K = 0.02, 0.1, 5
    _, yb, hb, lb, rb = ot.tvd_fft_grads(y, lam, rho, h, iso, K, xbar)
    sc = {}
    _, yb2, hb2, tb, re = ot.tvd_fft_grads_split(y, lam, rho, h, iso, K, xbar, scales=sc)
    assert np.allclose(yb, yb2, rtol=1e-10, atol=1e-12) and np.allclose(hb, hb2, rtol=1e-10, atol=1e-12)
    assert abs(tb / rho - lb) <= 1e-9 * abs(lb)
    assert abs(re - tb * lam / rho ** 2 - rb) <= 1e-9 * max(abs(rb), 1.0)
    assert sc["tau"] >= abs(tb) * (1 - 1e-12) and sc["rho"] >= abs(re) * (1 - 1e-12)
