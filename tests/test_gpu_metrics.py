"""GPU: the metrics kernels (csrc/metrics_capi.hip) against the numpy oracle (values) and fp64 torch
autograd of the same formulas (gradients w.r.t. the first argument).
Tolerances: values rel 2e-5 (fp32 window sums vs fp64); gradients rel-L2 2e-3."""
import numpy as np
import pytest
import torch

import metrics_torch as mt
import oracle_metrics as om
import oracle_np as o
from admm_deconv import metrics

pytestmark = pytest.mark.gpu

SHAPES = [(2, 1, 64, 64), (3, 3, 48, 40), (1, 2, 100, 75), (2, 1, 256, 256), (1, 1, 17, 130)]


def _pair(shape, seed):
    rng = np.random.default_rng(seed)
    x = rng.random(shape).astype(np.float32)
    y = np.clip(x + 0.08 * rng.standard_normal(shape), 0, 1).astype(np.float32)
    return x, y


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_ssim_value_and_grad(dev, shape):
    x, y = _pair(shape, 1)
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    yt = torch.from_numpy(y).to(dev)
    s = metrics.ssim(xt, yt)
    s.backward()
    ref, _ = om.ssim(o.from_c(x.astype(np.float64)), o.from_c(y.astype(np.float64)))
    assert abs(float(s) - ref) <= 2e-5 * abs(ref)
    x64 = torch.from_numpy(x.astype(np.float64)).requires_grad_(True)
    mt.ssim_per_image(x64, torch.from_numpy(y.astype(np.float64))).mean().backward()
    assert _rel(xt.grad.cpu().numpy(), x64.grad.numpy()) < 2e-3


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_gmsd_value_and_grad(dev, shape):
    x, y = _pair(shape, 2)
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    yt = torch.from_numpy(y).to(dev)
    g = metrics.gmsd(xt, yt)
    g.backward()
    ref, _ = om.gmsd(o.from_c(x.astype(np.float64)), o.from_c(y.astype(np.float64)))
    assert abs(float(g) - ref) <= 2e-5 * abs(ref)
    x64 = torch.from_numpy(x.astype(np.float64)).requires_grad_(True)
    mt.gmsd_per_image(x64, torch.from_numpy(y.astype(np.float64))).mean().backward()
    assert _rel(xt.grad.cpu().numpy(), x64.grad.numpy()) < 2e-3


def test_per_image_weights_and_reduction(dev):
    """Non-mean reductions: the per-image upstream gradient reaches each image's pixels."""
    x, y = _pair((3, 2, 32, 32), 3)
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    w = torch.tensor([0.5, -2.0, 3.0], dtype=torch.float32, device=dev)
    (metrics.gmsd(xt, torch.from_numpy(y).to(dev), reduction=lambda v: (v * w).sum())).backward()
    x64 = torch.from_numpy(x.astype(np.float64)).requires_grad_(True)
    (mt.gmsd_per_image(x64, torch.from_numpy(y.astype(np.float64))) * w.double().cpu()).sum().backward()
    assert _rel(xt.grad.cpu().numpy(), x64.grad.numpy()) < 2e-3


def test_ssim_variants(dev):
    x, y = _pair((2, 3, 40, 36), 4)
    xt, yt = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    xo, yo = o.from_c(x.astype(np.float64)), o.from_c(y.astype(np.float64))
    # same-size window on the symmetric padding (crop=false)
    assert abs(float(metrics.ssim(xt, yt, crop=False)) - om.ssim(xo, yo, crop=False)[0]) < 2e-5
    # ssim_loss_fast: 5 x 5 box window
    ref = 1.0 - om.ssim(xo, yo, np.full(5, 0.2))[0]
    assert abs(float(metrics.ssim_loss_fast(xt, yt)) - ref) < 2e-5
    # peakval
    assert abs(float(metrics.ssim(xt, yt, peakval=2.0)) - om.ssim(xo, yo, peakval=2.0)[0]) < 2e-5
    # a (k, k, 1, C) kernel as the reference passes it (ssim_kernel output)
    K = torch.from_numpy(np.outer(om.SSIM_KERNEL, om.SSIM_KERNEL)).reshape(11, 11, 1, 1)
    assert abs(float(metrics.ssim(xt, yt, K)) - om.ssim(xo, yo)[0]) < 2e-5


def test_psnr_and_mse(dev):
    x, y = _pair((4, 3, 64, 48), 5)
    xt, yt = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
    xo, yo = o.from_c(x.astype(np.float64)), o.from_c(y.astype(np.float64))
    assert abs(float(metrics.peak_snr(xt, yt)) - om.peak_snr(xo, yo)) < 1e-4
    assert abs(float(metrics.mse(xt, yt)) - np.mean((x.astype(np.float64) - y) ** 2)) < 1e-7


def test_deterministic(dev):
    x, y = _pair((2, 1, 128, 128), 6)
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    yt = torch.from_numpy(y).to(dev)
    grads = []
    for _ in range(2):
        xt.grad = None
        (metrics.gmsd(xt, yt) + metrics.ssim_loss(xt, yt)).backward()
        grads.append(xt.grad.clone())
    assert torch.equal(grads[0], grads[1])


def test_gmsd_on_two_streams_does_not_share_scratch(dev):
    """Two GMSD calls enqueued on two streams at once (the c5 branches' losses could be) each get their own
    scratch: the results equal the same calls made one after the other on the default stream."""
    shapes = [(2, 3, 128, 96), (4, 1, 200, 160)]   # different sizes: the second would grow a shared buffer
    pairs = [tuple(torch.from_numpy(a).to(dev) for a in _pair(s, 10 + i)) for i, s in enumerate(shapes)]
    ref = [metrics.gmsd(x, y, reduction=lambda v: v) for x, y in pairs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in pairs]
    got = [None, None]
    for rep in range(5):
        for i, ((x, y), st) in enumerate(zip(pairs, streams)):
            st.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(st):
                got[i] = metrics.gmsd(x, y, reduction=lambda v: v)
        torch.cuda.synchronize()
        for g, r in zip(got, ref):
            assert torch.equal(g, r)


def test_gmsd_backward_from_the_forward_sums(dev):
    """admm_gmsd_backward_f32 (the autograd backward) forms x_bar from the partial sums the forward left in its
    private workspace: bitwise the one-call gradient (admm_gmsd_f32 with x_bar), also with a second GMSD loss
    evaluated between the forward and the backward."""
    from admm_deconv.metrics import _gmsd_call
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.random((3, 2, 40, 48), dtype=np.float32)).to(dev)
    y = torch.from_numpy(rng.random((3, 2, 40, 48), dtype=np.float32)).to(dev)
    w = torch.tensor([0.5, -1.0, 2.0], device=dev)
    _, ref = _gmsd_call(x, y, 0.0026, 0.0, out_bar=w, want_grad=True)
    xt = x.clone().requires_grad_(True)
    per = metrics.gmsd(xt, y, reduction=lambda v: v)
    other = metrics.gmsd(y.clone().requires_grad_(True), x, reduction=lambda v: v)   # overwrites shared scratch
    (per * w).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(xt.grad, ref)
    assert torch.isfinite(other).all()
