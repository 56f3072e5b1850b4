"""GPU: device-resident lambda / rho at the boundary (the reference's `tvd_fft(y, λ::CGPUArray,
ρ::CGPUArray, ...)`, /root/reference/src/ops/ops.jl:99,181), per-stream default workspaces, and the
record/replay contract.

* The *_dev_f32 entry points read lambda / rho in-kernel: results are bitwise those of the host-scalar
  entry points with the same fp32 values, forward and adjoint.
* A layer forward + backward (and the Parallel/chcat caller) issues no host synchronisation: torch's
  sync-debug mode "error" raises on any device-to-host read torch makes.
* Concurrent solves on different streams (layers.Parallel without autograd) do not share scratch.
* A replay whose library options differ from its recording's is rejected (ADMM_E_INVALID)."""
import numpy as np
import pytest
import torch

import admm_deconv
from admm_deconv import _lib, layers, synth

pytestmark = pytest.mark.gpu

LAM, RHO = 0.0041, 0.021


def _inputs(dev, B=2, M=64, N=64, k=7, P=1, g0=5):
    h = synth.gaussian_psf(k, 1.3) if k else None
    y = torch.from_numpy(synth.make_batch(B, M, N, h, P=P, g0=g0)).to(dev)
    return y, (None if h is None else torch.from_numpy(h).to(dev))


@pytest.mark.parametrize("shape", [(2, 64, 64, 7), (2, 256, 256, 15), (2, 48, 40, 5), (1, 256, 256, 0)],
                         ids=["pow2", "fused", "generic", "fused-nopsf"])
@pytest.mark.parametrize("iso", [False, True], ids=["aniso", "iso"])
def test_device_scalars_forward_bitwise(dev, shape, iso):
    B, M, N, k = shape
    y, h = _inputs(dev, B, M, N, k)
    lam_t = torch.tensor([LAM], device=dev)
    rho_t = torch.tensor([RHO], device=dev)
    a = admm_deconv.tvd_fft(y, LAM, RHO, h, iso, 9)
    b = admm_deconv.tvd_fft(y, lam_t, rho_t, h, iso, 9)
    c = admm_deconv.tvd_fft(y, lam_t.double(), RHO, h, iso, 9)   # Float64 λ (deconv_admm.jl F1-F3 init)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(a, c)


@pytest.mark.parametrize("shape", [(2, 64, 64, 7, False), (2, 256, 256, 0, False), (3, 32, 32, 5, True),
                                   (2, 36, 30, 5, False)],
                         ids=["pow2", "fused-adj", "iso", "generic"])
def test_device_scalars_backward_bitwise(dev, shape):
    B, M, N, k, iso = shape
    y, h = _inputs(dev, B, M, N, k)
    xb = torch.randn_like(y)
    lam_t = torch.tensor([LAM], device=dev)
    rho_t = torch.tensor([RHO], device=dev)
    r1 = admm_deconv.tvd_fft_backward(y, xb, LAM, RHO, h, iso, 8)
    r2 = admm_deconv.tvd_fft_backward(y, xb, lam_t, rho_t, h, iso, 8)
    x3, rec = admm_deconv.tvd_fft_record(y, lam_t, rho_t, h, iso, 8)
    yb3, hb3, lb3, rb3 = admm_deconv.tvd_fft_backward_recorded(rec, x3, xb)
    torch.cuda.synchronize()
    for u, v in zip(r1, r2):
        assert (u is None and v is None) or torch.equal(u, v)
    assert torch.equal(r1[0], x3) and torch.equal(r1[1], yb3)
    assert torch.equal(r1[3], lb3) and torch.equal(r1[4], rb3)
    if h is not None:
        assert torch.equal(r1[2], hb3)


def test_layer_step_never_syncs_the_host(dev):
    """ADMMDeconv forward (projection + solve) and backward through the recorded adjoint, and the
    Parallel(chcat) denoiser branch of net_build.jl:113-128, with torch's sync-debug mode raising on
    any device-to-host read."""
    rng = np.random.default_rng(3)
    L1 = layers.ADMMDeconv((5, 5), 6, rng=rng, device=dev)
    br = [layers.ADMMDeconvF2((), 6, r, layers.relu1, rng=rng, device=dev) for r in (0.02, 0.2)]
    for L in [L1] + br:
        for t in L.trainable().values():
            if isinstance(t, torch.Tensor):
                t.requires_grad_(True)
    net = layers.Parallel(layers.chcat, *br)
    y, _ = _inputs(dev, 2, 64, 64, 5)
    y3, _ = _inputs(dev, 1, 64, 64, 0, P=3)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        out = L1(y)
        out.square().sum().backward()
        out2 = net(y3)
        out2.square().sum().backward()
    finally:
        torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    assert L1.lam.grad is not None and L1.rho.grad is not None and L1.weight.grad is not None
    assert all(L.lam.grad is not None for L in br)
    assert torch.isfinite(out).all() and torch.isfinite(out2).all()


def test_parallel_no_grad_streams_match_serial(dev):
    """Without autograd every branch goes through the default workspace of its own stream: concurrent
    branches must not share scratch state (bitwise equal to running them one after the other)."""
    rng = np.random.default_rng(5)
    br = [layers.ADMMDeconvF2((), 12, r, layers.relu1, rng=rng, device=dev) for r in (0.002, 0.02, 0.2, 2.0)]
    x, _ = _inputs(dev, 4, 256, 256, 0, P=3, g0=40)
    with torch.no_grad():
        par = layers.Parallel(layers.chcat, *br, streams=True, merge=False)(x)
        ser = layers.Parallel(layers.chcat, *br, streams=False, merge=False)(x)
        mer = layers.Parallel(layers.chcat, *br)(x)   # one grid for all branches (ops.tvd_fft_multi)
    torch.cuda.synchronize()
    assert torch.equal(par, ser)
    assert torch.equal(mer, ser)


def test_merged_parallel_step_never_syncs_the_host(dev):
    """The one-grid Parallel(chcat) of the c5 denoiser (net_build.jl:113-128), forward + backward, under
    torch's sync-debug mode (raises on any device-to-host read)."""
    rng = np.random.default_rng(4)
    br = [layers.ADMMDeconvF2((), 6, r, layers.relu1, rng=rng, device=dev) for r in (0.02, 0.2, 2.0)]
    for L in br:
        L.lam.requires_grad_(True)
    net = layers.Parallel(layers.chcat, *br)
    y3, _ = _inputs(dev, 2, 256, 256, 0, P=3)
    assert net._mergeable(y3)
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        out = net(y3)
        out.square().sum().backward()
    finally:
        torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    assert all(L.lam.grad is not None for L in br) and torch.isfinite(out).all()


def test_replay_rejects_changed_options(dev):
    y, h = _inputs(dev, 1, 256, 256, 0)
    xb = torch.randn_like(y)
    x, rec = admm_deconv.tvd_fft_record(y, LAM, RHO, None, False, 5)
    with _lib.option("FUSED", 0):
        with pytest.raises(_lib.AdmmError) as e:
            admm_deconv.tvd_fft_backward_recorded(rec, x, xb)
    assert e.value.code == _lib.ADMM_E_INVALID
    torch.cuda.synchronize()


def test_inplace_change_of_y_is_detected(dev):
    """The recorded adjoint reads y again (h_bar correlation): an in-place change between forward and
    backward must raise autograd's version error, not give a wrong gradient."""
    y, h = _inputs(dev, 1, 64, 64, 5)
    h = h.clone().requires_grad_(True)
    x = admm_deconv.tvd_fft(y, LAM, RHO, h, False, 4)
    y.add_(1.0)
    with pytest.raises(RuntimeError):
        x.sum().backward()
