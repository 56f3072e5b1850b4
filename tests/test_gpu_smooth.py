"""GPU parity of the compile-time-plan kernels for smooth non-power-of-two lengths (admm_smooth.hip).

They replace the runtime-length path's per-iteration kernels (column pass when this build compiled N,
line passes when it compiled M) on the same buffers; the oracle is oracle/oracle_np.py (restatement of
/root/reference/src/ops/ops.jl:17-96; parity unpinned against Julia itself).  Tolerance:
tests/parity.py.  Each case also runs with ADMM_OPT_SMOOTH = 0 (runtime plans for everything): two fp32
evaluations of the same algebra (different FFT factorisations), held to the parity bound (1e-5 rel-L2)."""
import numpy as np
import pytest
import torch

import admm_deconv
import oracle_np
import oracle_torch
from admm_deconv import _lib, synth
from parity import assert_parity, oracle_solve

pytestmark = pytest.mark.gpu

CASES = [
    # (B, P, N, M, psf, lam, rho, K, iso) -- N lines of M pixels (Julia M x N)
    (2, 1, 250, 250, ("gauss", 15, 2.5), 0.0041, 0.021, 8, False),   # 250 = 25 x 10 both ways
    (1, 1, 480, 640, ("gauss", 15, 2.5), 0.0041, 0.021, 4, False),   # 640 = 32 x 20, 480 = 24 x 20
    (2, 1, 99, 250, ("gauss", 9, 1.5), 0.01, 0.05, 6, False),        # lines compiled, columns runtime; ragged odd last block
    (1, 2, 250, 99, ("rand", 7, 4), 0.01, 0.05, 6, False),           # columns compiled, lines runtime
    (3, 1, 120, 96, ("rand", 10, 10), 0.02, 0.1, 7, False),          # short lines: row groups in the update
    (1, 1, 64, 2048, ("gauss", 5, 1.0), 0.0041, 0.021, 3, False),    # 2048 = 16 x 16 x 8 (3 passes)
    (1, 1, 3000, 16, None, 0.05, 0.1, 3, False),                     # 3000 = 30 x 10 x 10 columns
    (2, 3, 100, 160, None, 0.05, 0.02, 9, False),                    # empty PSF, RGB
    (3, 1, 250, 250, ("gauss", 9, 1.5), 0.0041, 0.021, 6, True),     # isotropic: compiled column / line inverse
    (1, 1, 250, 250, ("gauss", 15, 2.5), 0.0041, 0.021, 1, False),   # K = 1: no line update
]


@pytest.fixture(autouse=True)
def _two_pass_kernels(dev):
    """This file covers admm_smooth.hip's 2-pass kernels: the CU-resident solve (admm_resident.hip, default at
    the smooth squares <= 256 such as 250 x 250) is switched off here; tests/test_gpu_resident.py covers it."""
    with _lib.option("RESIDENT", 0):
        yield


def _psf(spec, rng):
    if spec is None:
        return None
    if spec[0] == "gauss":
        return synth.gaussian_psf(spec[1], spec[2])
    h = rng.random((spec[2], spec[1])).astype(np.float32)
    return (h / h.sum()).astype(np.float32)


def _solve(dev, y, lam, rho, h, iso, K):
    ht = None if h is None else torch.from_numpy(h).to(dev)
    x = admm_deconv.tvd_fft(torch.from_numpy(y).to(dev), lam, rho, ht, iso, K)
    torch.cuda.synchronize()
    return x.cpu().numpy()


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[1]}x{c[2]}x{c[3]}-K{c[7]}{'-iso' if c[8] else ''}" for c in CASES])
def test_smooth_parity_vs_oracle_and_runtime_plans(dev, case):
    B, P, N, M, spec, lam, rho, K, iso = case
    rng = np.random.default_rng(N + 7 * M + K)
    h = _psf(spec, rng)
    y = synth.make_batch(B, M, N, h, P=P, g0=5)
    got = _solve(dev, y, lam, rho, h, iso, K)
    with _lib.option("SMOOTH", 0):
        rt = _solve(dev, y, lam, rho, h, iso, K)
    ref = oracle_solve(y, lam, rho, h, iso, K, "spectral", linear_only=K == 1, what="smooth " + str(case))
    assert_parity(got, ref, what="smooth " + str(case))
    assert_parity(rt, ref, what="runtime plans " + str(case))
    d = np.linalg.norm((got - rt).ravel()) / np.linalg.norm(rt.ravel())
    assert d < 1e-5, f"compiled vs runtime plans differ by rel-L2 {d:.2e}"


def test_smooth_deterministic_and_batch_invariant(dev):
    h = synth.gaussian_psf(15, 2.5)
    y = torch.from_numpy(synth.make_batch(6, 250, 250, h)).to(dev)
    ht = torch.from_numpy(h).to(dev)
    a = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 7)
    b = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 7)
    part = torch.cat([admm_deconv.tvd_fft(y[i:i + 3].contiguous(), 0.0041, 0.021, ht, False, 7) for i in (0, 3)])
    torch.cuda.synchronize()
    assert torch.equal(a, b), "solve must be bitwise deterministic"
    assert torch.equal(a, part), "planes are independent (ops.jl:168-173): sub-batches give the same planes"


@pytest.mark.parametrize("need_h", [False, True])
def test_smooth_forward_trajectory_feeds_adjoint(dev, need_h):
    """The adjoint's trajectory (s_k written by the compiled line update) against fp64 autograd of the
    oracle; with h_bar the column pass falls back to the runtime kernel that saves the dim-2 spectra."""
    B, N, M, K, lam, rho = 2, 100, 96, 6, 0.02, 0.1
    rng = np.random.default_rng(17)
    h = synth.gaussian_psf(5, 1.0)
    y = synth.make_batch(B, M, N, h, g0=21)
    xbar = rng.standard_normal(y.shape).astype(np.float32)
    ht = torch.from_numpy(h).to(dev)
    x, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(torch.from_numpy(y).to(dev), torch.from_numpy(xbar).to(dev),
                                                     lam, rho, ht, False, K, need_h=need_h)
    torch.cuda.synchronize()
    x0, yb0, hb0, lb0, rb0 = oracle_torch.tvd_fft_grads(y.astype(np.float64), np.float32(lam), np.float32(rho),
                                                        h.astype(np.float64), False, K, xbar)
    assert_parity(x.cpu().numpy(), x0, what="x")
    yb = yb.cpu().numpy()
    assert np.linalg.norm(yb - yb0) / np.linalg.norm(yb0) < 1e-3
    assert abs(float(lb) - lb0) / abs(lb0) < 1e-3 and abs(float(rb) - rb0) / abs(rb0) < 1e-3
    if need_h:
        hb = hb.cpu().numpy()
        assert np.linalg.norm(hb - hb0) / np.linalg.norm(hb0) < 1e-3
