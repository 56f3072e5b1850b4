"""GPU parity of the fused per-plane kernel (plane_kernel.hip: 256 x 256, anisotropic prox).

The fused path is the default for these shapes; the library option FUSED = 0 forces the 2-pass path.  Both are
checked against the fp64 oracle (oracle/oracle_np.py, /root/reference/src/ops/ops.jl:17-96) with the
tolerance of tests/parity.py, and against each other."""

import numpy as np
import pytest
import torch

import admm_deconv
from admm_deconv import _lib, synth
from parity import assert_parity
from test_gpu_parity import make_psf, run_gpu, run_oracle

pytestmark = pytest.mark.gpu

CASES = [
    # (B, P, psf, lam, rho, K)
    (2, 1, ("gauss", 15, 2.5), 0.0041, 0.021, 25),   # c2
    (1, 1, ("gauss", 15, 2.5), 0.0041, 0.021, 1),
    (1, 1, ("gauss", 15, 2.5), 0.0041, 0.021, 2),
    (1, 1, ("gauss", 15, 2.5), 0.0041, 0.021, 3),
    (1, 3, None, 0.02, 0.02, 12),                     # empty PSF denoiser (F2), RGB (prox live in 1.3 %)
    (2, 1, ("rand", 10, 10), 0.01, 0.05, 7),          # even PSF
    (1, 1, ("rand", 4, 9), 0.02, 0.1, 5),             # asymmetric PSF
    (1, 1, ("box",), 0.0041, 0.021, 100),             # reference test PSF, default maxit
    (3, 1, ("gauss", 9, 1.2), 0.1, 0.3, 6),           # large tau: 98 % of s clipped
    (3, 1, ("gauss", 9, 1.2), 0.5, 0.3, 6),           # tau above every |s|: all clipped (linear-only)
]
LINEAR_ONLY = {(3, 1, ("gauss", 9, 1.2), 0.5, 0.3, 6)}


def fused_off():
    return _lib.option("FUSED", 0)


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}x{c[1]}-{c[2][0] if c[2] else 'none'}-K{c[5]}-lam{c[3]}" for c in CASES])
def test_plane_vs_oracle_and_2pass(dev, case):
    B, P, psf, lam, rho, K = case
    rng = np.random.default_rng(B * 31 + P + K)
    h = make_psf(psf, rng)
    y = synth.make_batch(B, 256, 256, h, P=P, g0=11)
    got = run_gpu(dev, y, lam, rho, h, False, K)
    ref = run_oracle(y, lam, rho, h, False, K, linear_only=K == 1 or case in LINEAR_ONLY,
                     what="fused " + str(case))
    assert_parity(got, ref, what="fused " + str(case))
    with fused_off():
        two = run_gpu(dev, y, lam, rho, h, False, K)
    assert_parity(two, ref, what="2-pass " + str(case))
    assert_parity(got, two, what="fused vs 2-pass " + str(case))


def test_plane_deterministic_and_batch_invariant(dev):
    h = synth.gaussian_psf(15, 2.5)
    y = torch.from_numpy(synth.make_batch(6, 256, 256, h)).to(dev)
    ht = torch.from_numpy(h).to(dev)
    a = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 9)
    b = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 9)
    part = torch.cat([admm_deconv.tvd_fft(y[i:i + 2].contiguous(), 0.0041, 0.021, ht, False, 9) for i in (0, 2, 4)])
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert torch.equal(a, part)


@pytest.mark.parametrize("psf", [True, False], ids=["psf", "nopsf"])
def test_plane_census_full_batch(dev, psf):
    """A whole c2 batch (512 planes) twice: every plane equal to the 2-pass path within the parity
    tolerance and bitwise equal across runs.  Guards against the lane-corruption hazard class described
    in DESIGN.md s4 (it showed as a few bad planes per launch, varying run to run)."""
    h = synth.gaussian_psf(15, 2.5) if psf else None
    ht = None if h is None else torch.from_numpy(h).to(dev)
    y = torch.from_numpy(synth.make_batch(64, 256, 256, h)).to(dev).repeat(8, 1, 1, 1).contiguous()
    with fused_off():
        ref = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 6)
    a = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 6)
    b = admm_deconv.tvd_fft(y, 0.0041, 0.021, ht, False, 6)
    torch.cuda.synchronize()
    rel = ((a - ref).flatten(1).norm(dim=1) / ref.flatten(1).norm(dim=1)).cpu()
    assert float(rel.max()) <= 1e-5, f"worst plane rel-L2 {float(rel.max()):.3e}, bad planes {int((rel > 1e-5).sum())}"
    assert torch.equal(a, b)
