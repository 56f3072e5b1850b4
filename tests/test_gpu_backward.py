"""GPU adjoint (admm_tvd_backward_f32) against PyTorch fp64 autograd of the oracle (oracle/oracle_torch.py).

Gradient parity.  The adjoint is exact given the ST masks (1[|s_k| > tau]); fp32 and fp64 forwards
disagree on the mask of the rare elements with |s_k| within ~1e-5 of tau (2 of 262k at 256^2, K=3),
and each such flip perturbs the gradient locally (y_bar: one blob of radius ~40 px) and the heavily
cancelling scalar sums (lambda_bar = tau_bar/rho) by a large absolute amount.  PyTorch's own fp32
autograd shows the same effect.  Criteria (tolerances per case in CASES):
  y_bar: trimmed per-plane relative L2 (worst 1% of pixels removed) <= 1e-4, full <= 5e-3;
  lambda_bar, rho_bar, h_bar: relative error <= the case's scalar tolerance: 1e-3, or 5e-3 where mask flips
  occur (256^2 at K >= 25).
How the mask-flip bound was measured (tools/grad_bounds.py, profiles/r02_grad_bounds.txt): on every case
below, the GPU error next to the error of an fp32 autograd of the same oracle (what an fp32 run of the
reference's own Zygote pass gets).  Where flips occur the fp32 autograd is off by up to 1.2e-2 (lambda_bar),
1.6e-3 (rho_bar), 1.3e-3 (h_bar), 2.6e-3 (y_bar full); the GPU by at most 1.8e-3, 1.1e-3, 1.8e-4, 3.7e-4.
5e-3 sits above the GPU's measured worst case and below the fp32 reference's.  test_backward_vs_autograd also
runs the fp32 autograd itself and allows twice its error where that is larger (the c4 plane at K = 50: fp32
autograd y_bar trimmed 1.8e-3, lambda_bar 1.2e-2, rho_bar 5.5e-2, h_bar 1.8e-2 -- mask flips everywhere)."""
import numpy as np
import pytest
import torch

import admm_deconv
import oracle_torch
from admm_deconv import _lib, synth
from parity import assert_case_prox_active, assert_parity

pytestmark = pytest.mark.gpu

CASES = [
    # (B, P, N, M, psf, lam, rho, K, scalar_tol)
    (2, 1, 32, 32, ("gauss", 5, 1.0), 0.02, 0.1, 6, 1e-3),
    (1, 2, 64, 64, ("rand", 7, 4), 0.0041, 0.021, 10, 1e-3),
    (2, 1, 64, 64, None, 0.05, 0.02, 12, 1e-3),
    (1, 1, 128, 128, ("rand", 10, 10), 0.01, 0.05, 5, 1e-3),
    (1, 1, 16, 32, ("gauss", 3, 0.8), 0.02, 0.1, 1, 1e-3),
    (2, 1, 256, 256, ("gauss", 15, 2.5), 0.0041, 0.021, 25, 5e-3),   # c2 slices: isolated mask flips
    (1, 1, 512, 512, ("gauss", 15, 2.5), 0.0041, 0.021, 50, 1e-3),   # c4 plane at its full K (2-pass adjoint)
]


def psf(spec, rng):
    if spec is None:
        return None
    if spec[0] == "gauss":
        return synth.gaussian_psf(spec[1], spec[2])
    h = rng.random((spec[2], spec[1])).astype(np.float32)
    return (h / h.sum()).astype(np.float32)


def assert_grad(got, ref, what, trim=0.01, tol=1e-4, full_tol=5e-3):
    g = np.asarray(got, np.float64).reshape(-1, got.shape[-2] * got.shape[-1])
    r = np.asarray(ref, np.float64).reshape(g.shape)
    assert np.all(np.isfinite(g)), what
    for i in range(g.shape[0]):
        e = g[i] - r[i]
        keep = np.argsort(np.abs(e))[: int(len(e) * (1 - trim))]
        trimmed = np.linalg.norm(e[keep]) / np.linalg.norm(r[i][keep])
        full = np.linalg.norm(e) / np.linalg.norm(r[i])
        assert trimmed <= tol, f"{what} plane {i}: trimmed rel-L2 {trimmed:.2e}"
        assert full <= full_tol, f"{what} plane {i}: rel-L2 {full:.2e}"


def grad_errs(got, ref, trim=0.01):
    """(worst trimmed, worst full) per-plane relative L2 of got vs ref."""
    g = np.asarray(got, np.float64).reshape(-1, got.shape[-2] * got.shape[-1])
    r = np.asarray(ref, np.float64).reshape(g.shape)
    tr, fu = 0.0, 0.0
    for i in range(g.shape[0]):
        e = g[i] - r[i]
        keep = np.argsort(np.abs(e))[: int(len(e) * (1 - trim))]
        tr = max(tr, np.linalg.norm(e[keep]) / np.linalg.norm(r[i][keep]))
        fu = max(fu, np.linalg.norm(e) / np.linalg.norm(r[i]))
    return tr, fu


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-12)


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[1]}x{c[2]}x{c[3]}-K{c[7]}" for c in CASES])
def test_backward_vs_autograd(dev, case):
    B, P, N, M, spec, lam, rho, K, stol = case
    rng = np.random.default_rng(N + M + K)
    h = psf(spec, rng)
    y = synth.make_batch(B, M, N, h, P=P, g0=11)
    xbar = rng.standard_normal(y.shape).astype(np.float32)
    assert_case_prox_active(y, lam, rho, h, False, K, str(case))
    ht = None if h is None else torch.from_numpy(h).to(dev)
    x, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(torch.from_numpy(y).to(dev), torch.from_numpy(xbar).to(dev),
                                                     lam, rho, ht, False, K)
    torch.cuda.synchronize()
    x0, yb0, hb0, lb0, rb0 = oracle_torch.tvd_fft_grads(y.astype(np.float64), np.float32(lam), np.float32(rho),
                                                        None if h is None else h.astype(np.float64), False, K, xbar)
    # the same gradients from an fp32 autograd of the oracle: where fp32 rounding flips ST masks (large
    # planes, many iterations) it differs from fp64 by far more than the case tolerance, and the GPU
    # (an fp32 implementation too) may then be off by up to twice as much
    _, yb32, hb32, lb32, rb32 = oracle_torch.tvd_fft_grads(y, np.float32(lam), np.float32(rho), h, False, K, xbar,
                                                           dtype=torch.float32)
    t32, f32 = grad_errs(yb32, yb0)
    assert_parity(x.cpu().numpy(), x0, what="x")
    assert_grad(yb.cpu().numpy(), yb0, "y_bar", tol=max(1e-4, 2 * t32), full_tol=max(5e-3, 2 * f32))
    assert rel(float(lb), lb0) < max(stol, 2 * rel(lb32, lb0))
    assert rel(float(rb), rb0) < max(stol, 2 * rel(rb32, rb0))
    if h is not None:
        hb = hb.cpu().numpy()
        e32 = np.linalg.norm(hb32 - hb0) / np.linalg.norm(hb0)
        assert np.linalg.norm(hb - hb0) / np.linalg.norm(hb0) < max(stol, 2 * e32)


ISO_CASES = [
    # (B, P, N, M, psf, lam, rho, K, scalar_tol) -- isotropic (BT) prox: the batch norm couples all planes;
    # 20 planes span two ISO_ADJ_A plane groups (16 planes per group)
    (20, 1, 32, 32, ("gauss", 5, 1.0), 0.02, 0.1, 6, 1e-3),
    (2, 3, 64, 64, ("rand", 7, 4), 0.0041, 0.021, 10, 1e-3),
    (3, 1, 64, 128, None, 0.05, 0.02, 8, 1e-3),
    (1, 1, 16, 32, ("gauss", 3, 0.8), 0.02, 0.1, 1, 1e-3),
    (2, 1, 256, 256, ("gauss", 15, 2.5), 0.0041, 0.021, 25, 1e-2),
]


@pytest.mark.parametrize("case", ISO_CASES, ids=[f"iso-{c[0]}x{c[1]}x{c[2]}x{c[3]}-K{c[7]}" for c in ISO_CASES])
def test_backward_iso_vs_autograd(dev, case):
    B, P, N, M, spec, lam, rho, K, stol = case
    rng = np.random.default_rng(7 * N + M + K)
    h = psf(spec, rng)
    y = synth.make_batch(B, M, N, h, P=P, g0=5)
    xbar = rng.standard_normal(y.shape).astype(np.float32)
    assert_case_prox_active(y, lam, rho, h, True, K, "iso " + str(case))
    ht = None if h is None else torch.from_numpy(h).to(dev)
    x, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(torch.from_numpy(y).to(dev), torch.from_numpy(xbar).to(dev),
                                                     lam, rho, ht, True, K)
    torch.cuda.synchronize()
    x0, yb0, hb0, lb0, rb0 = oracle_torch.tvd_fft_grads(y.astype(np.float64), np.float32(lam), np.float32(rho),
                                                        None if h is None else h.astype(np.float64), True, K, xbar)
    assert_parity(x.cpu().numpy(), x0, what="x")
    assert_grad(yb.cpu().numpy(), yb0, "y_bar")
    assert rel(float(lb), lb0) < stol, (float(lb), lb0)
    assert rel(float(rb), rb0) < stol, (float(rb), rb0)
    if h is not None:
        hb = hb.cpu().numpy()
        assert np.linalg.norm(hb - hb0) / np.linalg.norm(hb0) < stol


def test_autograd_function_and_layer_grads(dev):
    """torch.autograd through tvd_fft and through a layer (the rrule path), against the oracle."""
    from admm_deconv import layers
    rng = np.random.default_rng(3)
    h = synth.gaussian_psf(7, 1.2)
    y = synth.make_batch(2, 64, 64, h)
    L = layers.ADMMDeconv((7, 7), 8, rng=rng, device=dev)
    for t in (L.weight, L.lam, L.rho):
        t.requires_grad_(True)
    yt = torch.from_numpy(y).to(dev).requires_grad_(True)
    out = L(yt)
    loss = (out * out).sum()
    loss.backward()
    w = L.weight.detach().clamp(0, 1).cpu().numpy().reshape(7, 7)
    x0, yb0, hb0, lb0, rb0 = oracle_torch.tvd_fft_grads(y.astype(np.float64), L.lam.item(), L.rho.item(),
                                                        w.astype(np.float64), False, 8,
                                                        2 * out.detach().cpu().numpy().astype(np.float64))
    assert_grad(yt.grad.cpu().numpy(), yb0, "y.grad")
    assert rel(float(L.lam.grad), lb0) < 1e-3 and rel(float(L.rho.grad), rb0) < 1e-3


@pytest.mark.parametrize("iso", [False, True])
def test_backward_deterministic(dev, iso):
    h = synth.gaussian_psf(9, 1.5)
    y = torch.from_numpy(synth.make_batch(3, 64, 64, h)).to(dev)
    xb = torch.randn_like(y)
    ht = torch.from_numpy(h).to(dev)
    a = admm_deconv.tvd_fft_backward(y, xb, 0.01, 0.05, ht, iso, 7)
    b = admm_deconv.tvd_fft_backward(y, xb, 0.01, 0.05, ht, iso, 7)
    torch.cuda.synchronize()
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("with_psf", [False, True])
def test_backward_fused_trajectory(dev, with_psf):
    """256 x 256 anisotropic without h_bar: the fused plane kernel records the trajectory (lane-native
    s slots) and the reverse sweep reads it.  Against the fp64 oracle, and against the 2-pass
    trajectory (library option FUSED = 0)."""
    B, M, N, K, lam, rho = 2, 256, 256, 12, 0.0041, 0.021
    h = synth.gaussian_psf(15, 2.5) if with_psf else None
    y = synth.make_batch(B, M, N, h, g0=3)
    xbar = np.random.default_rng(9).standard_normal(y.shape).astype(np.float32)
    ht = None if h is None else torch.from_numpy(h).to(dev)
    yt, xt = torch.from_numpy(y).to(dev), torch.from_numpy(xbar).to(dev)
    x, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(yt, xt, lam, rho, ht, False, K, need_h=False)
    with _lib.option("FUSED", 0):
        x2, yb2, _, lb2, rb2 = admm_deconv.tvd_fft_backward(yt, xt, lam, rho, ht, False, K, need_h=False)
    torch.cuda.synchronize()
    assert hb is None
    x0, yb0, _, lb0, rb0 = oracle_torch.tvd_fft_grads(y.astype(np.float64), np.float32(lam), np.float32(rho),
                                                      None if h is None else h.astype(np.float64), False, K, xbar)
    assert_parity(x.cpu().numpy(), x0, what="x")
    assert_grad(yb.cpu().numpy(), yb0, "y_bar")
    assert_grad(yb.cpu().numpy(), yb2.cpu().numpy(), "y_bar fused vs 2-pass trajectory")
    assert rel(float(lb), lb0) < 5e-3 and rel(float(rb), rb0) < 5e-3
    assert rel(float(lb), float(lb2)) < 5e-3 and rel(float(rb), float(rb2)) < 5e-3


@pytest.mark.parametrize("case", [(2, 256, 256, None, False, False), (3, 64, 64, ("gauss", 7, 1.2), False, True),
                                  (20, 32, 32, ("gauss", 5, 1.0), True, True), (2, 256, 256, ("gauss", 15, 2.5),
                                                                                False, False)],
                         ids=["256-fused", "64-psf-hbar", "32-iso", "256-psf-fused"])
def test_record_then_backward_equals_combined(dev, case):
    """admm_tvd_forward_record_f32 + admm_tvd_backward_recorded_f32 == admm_tvd_backward_f32, bitwise."""
    B, M, N, spec, iso, need_h = case
    h = psf(spec, None)
    y = torch.from_numpy(synth.make_batch(B, M, N, h)).to(dev)
    xb = torch.randn_like(y)
    ht = None if h is None else torch.from_numpy(h).to(dev)
    K, lam, rho = 9, 0.01, 0.05
    x, rec = admm_deconv.tvd_fft_record(y, lam, rho, ht, iso, K, need_h=need_h)
    yb, hb, lb, rb = admm_deconv.tvd_fft_backward_recorded(rec, x, xb)
    x2, yb2, hb2, lb2, rb2 = admm_deconv.tvd_fft_backward(y, xb, lam, rho, ht, iso, K, need_h=need_h)
    torch.cuda.synchronize()
    assert torch.equal(x, x2) and torch.equal(yb, yb2)
    assert torch.equal(lb, lb2) and torch.equal(rb, rb2)
    if need_h:
        assert torch.equal(hb, hb2)
    with pytest.raises(RuntimeError):
        admm_deconv.tvd_fft_backward_recorded(rec, x, xb)


FUSED_ADJ_CASES = [
    # (B, P, psf, lam, rho, K)
    (2, 1, None, 0.0041, 0.021, 1),
    (1, 2, None, 0.002, 0.02, 2),      # prox live in 1.4 % of z_1
    (3, 1, ("gauss", 15, 2.5), 0.0041, 0.021, 3),
    (2, 1, ("gauss", 9, 1.5), 0.01, 0.05, 12),
    (1, 3, None, 0.0041, 0.021, 50),   # c5 layer shape: RGB, no PSF, K=50
]


@pytest.mark.parametrize("case", FUSED_ADJ_CASES,
                         ids=[f"{c[0]}x{c[1]}-{'psf' if c[2] else 'nopsf'}-K{c[5]}" for c in FUSED_ADJ_CASES])
def test_backward_fused_adjoint(dev, case):
    """256 x 256 anisotropic, no h_bar: the reverse sweep runs in plane256_adj_kernel (one workgroup per
    plane, all K steps).  Against the fp64 oracle, and against the 2-pass reverse sweep over the SAME
    recorded trajectory (option FUSED_ADJ = 0: same ST masks, so only fp32 rounding separates the two)."""
    B, P, spec, lam, rho, K = case
    rng = np.random.default_rng(K + 17 * B)
    h = psf(spec, rng)
    y = synth.make_batch(B, 256, 256, h, P=P, g0=21)
    xbar = rng.standard_normal(y.shape).astype(np.float32)
    assert_case_prox_active(y, lam, rho, h, False, K, "fused adjoint " + str(case))
    ht = None if h is None else torch.from_numpy(h).to(dev)
    yt, xt = torch.from_numpy(y).to(dev), torch.from_numpy(xbar).to(dev)
    x, rec = admm_deconv.tvd_fft_record(yt, lam, rho, ht, False, K, need_h=False)
    yb, _, lb, rb = admm_deconv.tvd_fft_backward_recorded(rec, x, xt)
    with _lib.option("FUSED_ADJ", 0):   # the record and its replay must see the same options
        x_, rec2 = admm_deconv.tvd_fft_record(yt, lam, rho, ht, False, K, need_h=False)
        yb2, _, lb2, rb2 = admm_deconv.tvd_fft_backward_recorded(rec2, x_, xt)
    torch.cuda.synchronize()
    assert torch.equal(x, x_)
    yb_, yb2_ = yb.cpu().numpy(), yb2.cpu().numpy()
    assert_grad(yb_, yb2_, "y_bar fused vs 2-pass adjoint", trim=0.0, tol=1e-5, full_tol=1e-5)
    assert rel(float(lb), float(lb2)) < 1e-4 and rel(float(rb), float(rb2)) < 1e-4, (lb, lb2, rb, rb2)
    x0, yb0, _, lb0, rb0 = oracle_torch.tvd_fft_grads(y.astype(np.float64), np.float32(lam), np.float32(rho),
                                                      None if h is None else h.astype(np.float64), False, K, xbar)
    assert_parity(x.cpu().numpy(), x0, what="x")
    assert_grad(yb_, yb0, "y_bar")
    assert rel(float(lb), lb0) < 5e-3 and rel(float(rb), rb0) < 5e-3


def test_backward_fused_adjoint_deterministic(dev):
    h = synth.gaussian_psf(15, 2.5)
    y = torch.from_numpy(synth.make_batch(4, 256, 256, h)).to(dev)
    xb = torch.randn_like(y)
    ht = torch.from_numpy(h).to(dev)
    a = admm_deconv.tvd_fft_backward(y, xb, 0.0041, 0.021, ht, False, 25, need_h=False)
    b = admm_deconv.tvd_fft_backward(y, xb, 0.0041, 0.021, ht, False, 25, need_h=False)
    torch.cuda.synchronize()
    for u, v in zip(a, b):
        if u is not None:
            assert torch.equal(u, v)


GENERIC_CASES = [
    # (B, P, N, M, psf, lam, rho, K, iso, scalar_tol) -- shapes outside the power-of-two kernels: the
    # runtime-length reverse sweep (admm_generic_bwd.hip), h_bar included
    (2, 1, 40, 48, ("gauss", 5, 1.0), 0.02, 0.1, 6, False, 1e-3),
    (1, 2, 29, 37, ("rand", 7, 4), 0.0041, 0.021, 8, False, 1e-3),
    (2, 1, 50, 30, None, 0.05, 0.02, 10, False, 1e-3),
    (1, 1, 24, 33, ("gauss", 3, 0.8), 0.02, 0.1, 1, False, 1e-3),
    (3, 1, 45, 36, ("gauss", 5, 1.0), 0.02, 0.1, 6, True, 1e-3),
    (2, 2, 24, 33, ("rand", 5, 6), 0.0041, 0.021, 7, True, 1e-3),
    (2, 1, 20, 27, None, 0.05, 0.02, 5, True, 1e-3),
]


@pytest.mark.parametrize("case", GENERIC_CASES,
                         ids=[f"{c[0]}x{c[1]}x{c[2]}x{c[3]}-K{c[7]}{'-iso' if c[8] else ''}" for c in GENERIC_CASES])
def test_backward_generic_shape_vs_autograd(dev, case):
    B, P, N, M, spec, lam, rho, K, iso, stol = case
    rng = np.random.default_rng(3 * N + M + K)
    h = psf(spec, rng)
    y = synth.make_batch(B, M, N, h, P=P, g0=13)
    xbar = rng.standard_normal(y.shape).astype(np.float32)
    assert_case_prox_active(y, lam, rho, h, iso, K, "generic " + str(case))
    ht = None if h is None else torch.from_numpy(h).to(dev)
    x, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(torch.from_numpy(y).to(dev), torch.from_numpy(xbar).to(dev),
                                                     lam, rho, ht, iso, K)
    torch.cuda.synchronize()
    x0, yb0, hb0, lb0, rb0 = oracle_torch.tvd_fft_grads(y.astype(np.float64), np.float32(lam), np.float32(rho),
                                                        None if h is None else h.astype(np.float64), iso, K, xbar)
    assert_parity(x.cpu().numpy(), x0, what="x")
    assert_grad(yb.cpu().numpy(), yb0, "y_bar")
    assert rel(float(lb), lb0) < stol, (float(lb), lb0)
    assert rel(float(rb), rb0) < stol, (float(rb), rb0)
    if h is not None:
        hb = hb.cpu().numpy()
        assert np.linalg.norm(hb - hb0) / np.linalg.norm(hb0) < stol


def test_backward_generic_record_replay(dev):
    """Record + replay on a runtime-length shape equals the combined call, bitwise."""
    h = synth.gaussian_psf(5, 1.0)
    y = torch.from_numpy(synth.make_batch(2, 45, 30, h)).to(dev)
    xb = torch.randn_like(y)
    ht = torch.from_numpy(h).to(dev)
    x, rec = admm_deconv.tvd_fft_record(y, 0.01, 0.05, ht, False, 6, need_h=True)
    yb, hb, lb, rb = admm_deconv.tvd_fft_backward_recorded(rec, x, xb)
    x2, yb2, hb2, lb2, rb2 = admm_deconv.tvd_fft_backward(y, xb, 0.01, 0.05, ht, False, 6, need_h=True)
    torch.cuda.synchronize()
    assert torch.equal(x, x2) and torch.equal(yb, yb2) and torch.equal(hb, hb2)
    assert torch.equal(lb, lb2) and torch.equal(rb, rb2)


NO_YBAR_CASES = [
    # (B, P, M, N, psf, iso, need_h, options): each reverse-sweep variant once
    (2, 3, 256, 256, None, False, False, {}),                          # fused adjoint (c5 aniso layer shape)
    (2, 1, 256, 256, ("gauss", 9, 1.5), False, False, {"FUSED_ADJ": 0}),   # 2-pass adjoint, fused trajectory
    (2, 1, 128, 128, ("gauss", 7, 1.2), False, True, {}),              # 2-pass with h_bar (Vsum still kept)
    (6, 3, 64, 64, None, True, False, {}),                             # iso (c5 use_iso shape class)
    (2, 1, 100, 75, ("gauss", 5, 1.0), False, False, {}),              # runtime-length adjoint
    (4, 1, 96, 96, None, True, False, {}),                             # runtime-length iso adjoint
]


@pytest.mark.parametrize("case", NO_YBAR_CASES,
                         ids=["fused", "2pass", "2pass-hbar", "iso", "generic", "generic-iso"])
def test_backward_without_y_bar_is_bitwise_the_same(dev, case):
    """y_bar = NULL (the input needs no gradient, as a first-layer denoiser's does not): the reverse sweep
    keeps no running sum of vbar (8 B/px less traffic per step), and every other gradient is bitwise the
    one of the full sweep; through autograd, a layer whose input does not require grad gets the same
    parameter gradients as one whose input does."""
    B, P, M, N, spec, iso, need_h, opts = case
    h = psf(spec, None)
    y = torch.from_numpy(synth.make_batch(B, M, N, h, P=P)).to(dev)
    xb = torch.randn_like(y)
    ht = None if h is None else torch.from_numpy(h).to(dev)
    K, lam, rho = 9, 0.01, 0.05
    import contextlib
    with contextlib.ExitStack() as st:
        for k, v in opts.items():
            st.enter_context(_lib.option(k, v))
        full = admm_deconv.tvd_fft_backward(y, xb, lam, rho, ht, iso, K, need_h=need_h)
        part = admm_deconv.tvd_fft_backward(y, xb, lam, rho, ht, iso, K, need_h=need_h, need_y=False)
        x, rec = admm_deconv.tvd_fft_record(y, lam, rho, ht, iso, K, need_h=need_h)
        rep = admm_deconv.tvd_fft_backward_recorded(rec, x, xb, need_y=False)
        # neither y_bar nor rho_bar (ADMMDeconvF2's fixed rho): s_k is not read either
        lo = admm_deconv.tvd_fft_backward(y, xb, lam, rho, ht, iso, K, need_h=need_h, need_y=False, need_rho=False)
        x, rec = admm_deconv.tvd_fft_record(y, lam, rho, ht, iso, K, need_h=need_h)
        rep2 = admm_deconv.tvd_fft_backward_recorded(rec, x, xb, need_y=False, need_rho=False)
    torch.cuda.synchronize()
    assert part[1] is None and rep[0] is None
    assert lo[1] is None and lo[4] is None and rep2[0] is None and rep2[3] is None
    assert torch.equal(full[3], lo[3]) and torch.equal(full[3], rep2[2]), "lambda_bar without rho_bar"
    if need_h:
        assert torch.equal(full[2], lo[2]) and torch.equal(full[2], rep2[1])
    assert torch.equal(full[0], part[0]) and torch.equal(full[0], x)
    for i, what in ((3, "lambda_bar"), (4, "rho_bar")):
        assert torch.equal(full[i], part[i]), what
        assert torch.equal(full[i], rep[i - 1]), what + " (recorded)"
    if need_h:
        assert torch.equal(full[2], part[2]) and torch.equal(full[2], rep[1])


def test_layer_input_without_grad_same_param_grads(dev):
    """autograd: ADMMDeconvF2 (fixed rho) on an input that does not require grad asks the library for
    neither y_bar nor rho_bar; the trainable lambda's gradient equals the one of the same layer on an input
    that does (whose rho is made trainable too, so that the full sweep runs)."""
    from admm_deconv import layers
    y = torch.from_numpy(synth.make_batch(2, 256, 256, None, P=3)).to(dev)
    grads = []
    for need_y in (True, False):
        L = layers.ADMMDeconvF2((), 12, 0.2, layers.relu1, rng=np.random.default_rng(5), device=dev)
        L.lam.requires_grad_(True)
        L.rho.requires_grad_(need_y)
        yi = y.clone().requires_grad_(need_y)
        out = L(yi)
        (out * out).sum().backward()
        grads.append(L.lam.grad.clone())
        assert (yi.grad is not None) == need_y
    torch.cuda.synchronize()
    assert torch.equal(grads[0], grads[1])
