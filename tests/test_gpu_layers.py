"""The layer mirror (src/layers/deconv_admm.jl) on the GPU against the oracle's restated forward."""
import numpy as np
import pytest
import torch

import oracle_np
from admm_deconv import _lib, layers, synth
from parity import assert_parity, assert_parity_fp32ref

pytestmark = pytest.mark.gpu


def oracle_layer(layer, y):
    w = layer.weight.detach().cpu().numpy()
    w = None if w.size == 0 else oracle_np.psf_from_c(w.reshape(w.shape[-2:]))
    bias = None if layer.bias is False else layer.bias.cpu().numpy()
    x = oracle_np.admm_layer_forward(oracle_np.from_c(y.astype(np.float64)), layer.lam.item(), layer.rho.item(), w,
                                     layer.iso, layer.iters, layer.creg, bias, None)
    return oracle_np.to_c(x)


@pytest.mark.parametrize("kind", ["ADMMDeconv", "F1", "F2", "F3", "F2-empty", "F3-iso-bias"])
def test_layer_forward(dev, kind):
    rng = np.random.default_rng(5)
    if kind == "ADMMDeconv":
        L = layers.ADMMDeconv((10, 10), 12, layers.relu, rng=rng, device=dev)
    elif kind == "F1":
        L = layers.ADMMDeconvF1((7, 7), 10, 0.004, rng=rng, device=dev)
    elif kind == "F2":
        L = layers.ADMMDeconvF2((7, 7), 10, 0.04, layers.relu6, rng=rng, device=dev)
    elif kind == "F2-empty":
        L = layers.ADMMDeconvF2((), 50, 0.02, layers.relu1, rng=rng, device=dev)   # net_build.jl:115
    elif kind == "F3":
        L = layers.ADMMDeconvF3((15, 15), 25, 0.0041, 0.021, rng=rng, device=dev)
    else:
        L = layers.ADMMDeconvF3((9, 9), 10, 0.01, 0.05, iso=True, bias=True, rng=rng, device=dev)
        L.bias = L.bias + 0.25
    y = synth.make_batch(3, 64, 64, synth.gaussian_psf(9, 1.2), P=2)
    out = L(torch.from_numpy(y).to(dev))
    torch.cuda.synchronize()
    # the forward wrote the projected parameters back (deconv_admm.jl:216-219)
    assert L.weight.numel() == 0 or (float(L.weight.min()) >= 0.0 and float(L.weight.max()) <= 1.0)
    assert float(L.lam.min()) >= L.creg and float(L.rho.min()) >= L.creg
    ref = oracle_layer(L, y)
    act = {"ADMMDeconv": lambda a: np.maximum(a, 0), "F2": lambda a: np.clip(a, 0, 6),
           "F2-empty": lambda a: np.clip(a, 0, 1)}.get(kind, lambda a: a)
    got = out.cpu().numpy()
    ref = act(ref)
    if kind in ("ADMMDeconv", "F2", "F2-empty"):
        # activations clip; compare with an absolute guard scaled by the pre-activation magnitude
        assert np.abs(got - ref).max() <= 2e-4 * max(1.0, np.abs(ref).max())
    else:
        # F3 solves with a glorot-initialised 15 x 15 PSF (clamped to [0, 1]) whose spectrum has near-zeros: the
        # spectral division amplifies rounding, and every fp32 solve lands about 1e-5 from the fp64 oracle (the C
        # fp32 reference solve 1.2e-5, fp32 torch 0.7e-5 .. 1.0e-5 per plane).  The resident 64^2 path's 1.04e-5
        #  and the 2-pass path's lower figure are two samples of that rounding (different FFT plans
        # and summation orders), not a defect of either.  Bound: max(1e-5, the C fp32 reference's error)
        w = L.weight.detach().cpu().numpy()
        w = None if w.size == 0 else w.reshape(w.shape[-2:]).astype(np.float32)
        lam, rho = np.float32(L.lam.item()), np.float32(L.rho.item())
        sol = oracle_np.to_c(oracle_np.tvd_fft_spectral(oracle_np.from_c(y.astype(np.float64)), lam, rho,
                                                        None if w is None else oracle_np.psf_from_c(w), L.iso, L.iters))
        bias = 0.0 if L.bias is False else float(L.bias.reshape(-1)[0])   # the solve before `.+ bias` (:222)
        assert_parity(got, ref, rel_tol=1.0, maxabs_tol=1.0)                 # shape / finiteness of the layer output
        assert_parity_fp32ref(got - np.float32(bias), sol, y, lam, rho, w, L.iso, L.iters, what=kind)


def test_trainable_sets():
    assert layers.ADMMDeconv.TRAINABLE == ("weight", "bias", "lam", "rho")       # deconv_admm.jl:209
    assert layers.ADMMDeconvF1.TRAINABLE == ("weight", "bias", "rho")            # :55
    assert layers.ADMMDeconvF2.TRAINABLE == ("weight", "bias", "lam")            # :107
    assert layers.ADMMDeconvF3.TRAINABLE == ("weight", "bias")                   # :161


def test_creg_clamp(dev):
    L = layers.ADMMDeconvF3((5, 5), 3, 0.001, 0.002, creg=0.01, device=dev)
    L(torch.from_numpy(synth.make_batch(1, 32, 32, None)).to(dev))
    assert abs(L.lam.item() - 0.01) < 1e-7 and abs(L.rho.item() - 0.01) < 1e-7


def test_parallel_merges_isotropic_branches_only_within_one_wave(dev):
    """Default merge rule (layers.ISO_MERGE_MAX_PLANES = 512): anisotropic branches always share one grid; isotropic
    ones up to 512 planes in all -- the reference's training batch (batch_size 2, RGB, 5 branches: 30 planes,
    src/configs/train_cfg.json:10-14) merges, 36 RGB images (540 planes) do not -- unless merge="always"."""
    from admm_deconv import layers
    rng = np.random.default_rng(1)
    for iso in (False, True):
        branch = [layers.ADMMDeconvF2((), 5, r, layers.relu1, iso=iso, rng=rng, device=dev)
                  for r in (0.002, 0.02, 0.2, 2.0, 4.0)]
        for L in branch:
            L.lam.requires_grad_(True)
        small = torch.zeros(2, 3, 256, 256, device=dev)
        big = torch.zeros(36, 3, 256, 256, device=dev)
        auto = layers.Parallel(layers.chcat, *branch)
        assert auto._mergeable(small)
        assert auto._mergeable(big) == (not iso)
        assert layers.Parallel(layers.chcat, *branch, merge="always")._mergeable(big)


@pytest.mark.parametrize("iso", [False, True], ids=["aniso", "iso"])
@pytest.mark.parametrize("train_rho", [False, True], ids=["lam", "lam+rho"])
def test_parallel_branches_on_streams_match_serial(dev, train_rho, iso):
    """Parallel(chcat, ...) (net_build.jl:121-125): the branches in ONE grid (the default for ADMM branches
    the fused kernel covers), each branch on its own HIP stream, and the branches run one after the other
    give the same forward output and the same parameter gradients, bitwise; the input gradient (a sum over
    the branches, added in a different order) to fp32 rounding.  train_rho: rho trainable too, so the
    recordings keep the full trajectory instead of the ST mask bits (isotropic: no one-grid solve then)."""
    from admm_deconv import layers
    x0 = torch.from_numpy(synth.make_batch(3, 256, 256, None, P=3, sigma=0.1)).to(dev)
    grads = []
    for streams, merge in ((True, False), (False, False), (True, "always")):
        rng = np.random.default_rng(5)
        branch = [layers.ADMMDeconvF2((), 12, r, layers.relu1, iso=iso, rng=rng, device=dev) for r in (0.002, 0.2, 4.0)]
        for L in branch:
            L.lam.requires_grad_(True)
            L.rho.requires_grad_(train_rho)
        net = layers.Parallel(layers.chcat, *branch, streams=streams, merge=merge)
        assert net._mergeable(x0) == (bool(merge) and not (iso and train_rho))
        x = x0.clone().requires_grad_(True)
        out = net(x)
        (out * torch.linspace(0, 1, out.shape[1], device=dev).reshape(1, -1, 1, 1)).sum().backward()
        torch.cuda.synchronize()
        grads.append((out.detach(), x.grad, [L.lam.grad for L in branch], [L.rho.grad for L in branch]))
    (o1, g1, l1, r1) = grads[0]
    assert o1.shape == (3, 9, 256, 256)
    for (o2, g2, l2, r2) in grads[1:]:
        assert torch.equal(o1, o2)
        assert torch.allclose(g1, g2, rtol=1e-6, atol=1e-7 * float(g1.abs().max()))
        assert all(torch.equal(a, b) for a, b in zip(l1, l2))
        if train_rho:
            assert all(torch.equal(a, b) for a, b in zip(r1, r2))


@pytest.mark.parametrize("iso,rule", [(False, False), (True, False),
                                      pytest.param(False, True, marks=pytest.mark.min_planes_rule),
                                      pytest.param(True, True, marks=pytest.mark.min_planes_rule)],
                         ids=["aniso", "iso", "aniso-default-rule", "iso-default-rule"])
def test_c5_denoiser_branch_gradients(dev, iso, rule):
    """BASELINE c5's caller: the get_denoiser branch of src/nets/net_build.jl:113-128 -- Parallel(chcat) of
    5 x ADMMDeconvF2((), 50, rho, relu1, iso=use_iso) -- on a small RGB batch (2 x 3 planes of 256^2),
    branches in one grid; iso = true is the training default (src/configs/train_cfg.json:14),
    where the batch norm couples the 6 planes of a branch.  The gradient of a weighted sum of the output
    w.r.t. every branch's trainable lambda (deconv_admm.jl:107) against fp64 autograd of the oracle: for
    branch i, lambda_bar = <xbar_i, d x_i / d lambda> with xbar_i = w_i * relu1'(x_i).  *-default-rule: the
    library's plane-count rule at its default, under which these 30 planes run the 2-pass kernels over all five
    branches in one grid (the reference's training configuration, train_cfg.json:10-14)."""
    import oracle_torch
    rng = np.random.default_rng(12)
    rhos = (0.002, 0.02, 0.2, 2.0, 4.0)
    br = [layers.ADMMDeconvF2((), 50, r, layers.relu1, iso=iso, rng=rng, device=dev) for r in rhos]
    for L in br:
        L.lam.requires_grad_(True)
    net = layers.Parallel(layers.chcat, *br)
    y = synth.make_batch(2, 256, 256, None, P=3, sigma=0.1, g0=9)
    w = rng.standard_normal((2, 15, 256, 256)).astype(np.float32)
    _lib.profile_reset()
    _lib.profile_enable(True)
    try:
        out = net(torch.from_numpy(y).to(dev))
        (out * torch.from_numpy(w).to(dev)).sum().backward()
        torch.cuda.synchronize()
        columns = _lib.profile_get(_lib.K_COLUMN)[1]
    finally:
        _lib.profile_enable(False)
    # the merged grid: per-plane kernels (no column launches) with MIN_PLANES = 0, the 2-pass ones at the rule
    assert (columns > 0) == rule, columns
    for i, (L, r) in enumerate(zip(br, rhos)):
        lam = float(L.lam.detach().cpu()[0])
        x0 = oracle_torch.tvd_fft_torch(torch.from_numpy(y.astype(np.float64)),
                                        torch.tensor(float(np.float32(lam)), dtype=torch.float64),
                                        torch.tensor(float(np.float32(r)), dtype=torch.float64), None, iso, 50).numpy()
        xbar = w[:, 3 * i:3 * i + 3] * ((x0 > 0) & (x0 < 1))
        _, _, _, lb0, _ = oracle_torch.tvd_fft_grads(y.astype(np.float64), np.float32(lam), np.float32(r), None,
                                                     iso, 50, xbar.astype(np.float32))
        got = float(L.lam.grad.cpu()[0])
        assert abs(got - lb0) <= 5e-3 * abs(lb0), f"branch {i} (rho {r}): lambda_bar {got} vs {lb0}"
        np.testing.assert_allclose(out[:, 3 * i:3 * i + 3].detach().cpu().numpy(), np.clip(x0, 0, 1), atol=2e-4)


def test_reference_demo_layer_forward_and_gradients(dev):
    """The reference's own demo (src/ADMM_Deconv.jl:17-23): ADMMDeconv((32,32), 50, relu6) on a (32,32,3,2)
    batch of crops -- a PSF as large as the image -- forward and the gradients of every trainable (PSF, lambda,
    rho) and of the input, against fp64 autograd of the oracle through the same projection and relu6."""
    import oracle_torch
    rng = np.random.default_rng(17)
    L = layers.ADMMDeconv((32, 32), 50, layers.relu6, rng=rng, device=dev)
    for t in (L.weight, L.lam, L.rho):
        t.requires_grad_(True)
    y = synth.make_batch(2, 32, 32, synth.gaussian_psf(5, 1.0), P=3, g0=40)
    w = rng.standard_normal(y.shape).astype(np.float32)
    yt = torch.from_numpy(y).to(dev).requires_grad_(True)
    out = L(yt)
    (out * torch.from_numpy(w).to(dev)).sum().backward()
    torch.cuda.synchronize()
    h = L.weight.detach().cpu().numpy().reshape(32, 32).astype(np.float64)   # projected to [0, 1] (:219)
    lam, rho = L.lam.item(), L.rho.item()
    x0 = oracle_torch.tvd_fft_torch(torch.from_numpy(y.astype(np.float64)), torch.tensor(lam, dtype=torch.float64),
                                    torch.tensor(rho, dtype=torch.float64), torch.from_numpy(h), False, 50).numpy()
    got = out.detach().cpu().numpy()
    assert np.abs(got - np.clip(x0, 0, 6)).max() <= 2e-4 * max(1.0, np.abs(x0).max())
    xbar = w * ((x0 > 0) & (x0 < 6))
    _, yb0, hb0, lb0, rb0 = oracle_torch.tvd_fft_grads(y.astype(np.float64), np.float32(lam), np.float32(rho), h,
                                                       False, 50, xbar)

    def rel(a, b):
        return float(np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b))
    assert rel(yt.grad.cpu().numpy(), yb0) < 1e-3
    assert rel(L.weight.grad.cpu().numpy().reshape(32, 32), hb0) < 1e-3
    assert abs(float(L.lam.grad) - lb0) <= 1e-3 * abs(lb0)
    assert abs(float(L.rho.grad) - rb0) <= 1e-3 * abs(rb0)


@pytest.mark.parametrize("fn,hi", [(layers.relu1, 1.0), (layers.relu6, 6.0)], ids=["relu1", "relu6"])
def test_clamp_activation_gradient_matches_autograd(dev, fn, hi):
    """relu1 / relu6 backward through admm_clamp_backward_f32: bitwise torch.clamp's autograd, the ties at lo and hi
    (gradient passed) and a length that is not a multiple of 4 included."""
    rng = np.random.default_rng(2)
    x = (rng.standard_normal(4099) * hi).astype(np.float32)
    x[:6] = [0.0, hi, -0.0, np.nextafter(0, -1), np.nextafter(np.float32(hi), np.float32(2 * hi)), hi / 2]
    g = torch.from_numpy(rng.standard_normal(4099).astype(np.float32)).to(dev)
    a = torch.from_numpy(x).to(dev).requires_grad_(True)
    b = torch.from_numpy(x).to(dev).requires_grad_(True)
    ya, yb = fn(a), torch.clamp(b, 0.0, hi)
    assert torch.equal(ya, yb)
    ya.backward(g)
    yb.backward(g)
    assert torch.equal(a.grad, b.grad)
