"""GPU: the one-grid multi-branch solve (admm_tvd_forward_multi_dev_f32 / admm_tvd_backward_multi_recorded_dev_f32)
-- the branches of Parallel(chcat, ADMMDeconvF2((), K, rho_i, relu1) ...) of src/nets/net_build.jl:113-125 in
one launch of the fused kernel -- against the same branches solved one by one through the single-solve
ABI: forward bitwise (chcat layout), lambda_bar / rho_bar bitwise, y_bar (a sum over branches) to fp32
rounding; the mask-bit trajectory (ADMM_REC_MASKS) against the full one; and the isotropic one-grid solve
(ADMM_MULTI_ISO, plane_iso.hip: each branch's batch norm over its own planes) the same way."""
import numpy as np
import pytest
import torch

import admm_deconv
import oracle_torch
from admm_deconv import _lib, synth
from parity import assert_parity

pytestmark = pytest.mark.gpu

RHOS = (0.002, 0.02, 0.2, 2.0, 4.0)   # net_build.jl:113-117


def _branch_scalars(dev, n, seed=3):
    rng = np.random.default_rng(seed)
    lams = [torch.tensor([float(v)], device=dev) for v in np.abs(rng.standard_normal(n)) * 0.01 + 1e-3]
    rhos = [torch.tensor([r], device=dev) for r in RHOS[:n]]
    return lams, rhos


@pytest.mark.parametrize("n,B,P,K", [(1, 2, 1, 5), (2, 1, 3, 9), (5, 2, 3, 12), (3, 3, 1, 1)])
def test_multi_forward_is_the_branches_bitwise(dev, n, B, P, K):
    y = torch.from_numpy(synth.make_batch(B, 256, 256, None, P=P, sigma=0.1, g0=4)).to(dev)
    lams, rhos = _branch_scalars(dev, n)
    x = admm_deconv.tvd_fft_multi(y, lams, rhos, K)
    ref = torch.cat([admm_deconv.tvd_fft(y, l, r, None, False, K) for l, r in zip(lams, rhos)], dim=1)
    torch.cuda.synchronize()
    assert x.shape == (B, n * P, 256, 256)
    assert torch.equal(x, ref)


def test_multi_forward_vs_oracle(dev):
    """One branch plane of a 5-branch call against the fp64 oracle (tests/parity.py tolerance)."""
    y = synth.make_batch(1, 256, 256, None, P=3, sigma=0.1, g0=8)
    lams, rhos = _branch_scalars(dev, 5, seed=9)
    x = admm_deconv.tvd_fft_multi(torch.from_numpy(y).to(dev), lams, rhos, 20).cpu().numpy()
    for i in (0, 3):
        ref = oracle_torch.tvd_fft_torch(torch.from_numpy(y.astype(np.float64)),
                                         torch.tensor(float(lams[i]), dtype=torch.float64),
                                         torch.tensor(float(rhos[i]), dtype=torch.float64), None, False, 20).numpy()
        assert_parity(x[:, 3 * i:3 * i + 3], ref, what=f"branch {i}")


@pytest.mark.parametrize("rule", [False, pytest.param(True, marks=pytest.mark.min_planes_rule)],
                         ids=["per-plane", "default-rule"])
@pytest.mark.parametrize("need_rho", [True, False], ids=["full-trajectory", "mask-bits"])
def test_multi_backward_is_the_branches(dev, need_rho, rule):
    """default-rule: 30 planes are below the fused kernels' plane count, so the merged grid runs the 2-pass
    kernels over every branch's planes and each branch alone the same kernels: everything bitwise (the partial
    rows are laid out per branch as a single solve's)."""
    n, B, P, K = 5, 2, 3, 10
    y = torch.from_numpy(synth.make_batch(B, 256, 256, None, P=P, sigma=0.1, g0=6)).to(dev)
    lams, rhos = _branch_scalars(dev, n, seed=5)
    xb = torch.randn((B, n * P, 256, 256), device=dev)
    _lib.profile_reset()
    _lib.profile_enable(True)
    try:
        x, rec = admm_deconv.tvd_fft_multi(y, lams, rhos, K, record=True, need_rho=need_rho)
        yb, lb, rb = admm_deconv.tvd_fft_multi_backward_recorded(rec, x, xb, need_rho=need_rho)
        columns = _lib.profile_get(_lib.K_COLUMN)[1]
    finally:
        _lib.profile_enable(False)
    assert columns == (2 * K if rule else 0), columns
    yb_sum = torch.zeros_like(y)
    for i in range(n):
        xi, reci = admm_deconv.tvd_fft_record(y, lams[i], rhos[i], None, False, K, need_rho=need_rho)
        ybi, _, lbi, rbi = admm_deconv.tvd_fft_backward_recorded(reci, xi, xb[:, i * P:(i + 1) * P].contiguous(),
                                                                 need_rho=need_rho)
        torch.cuda.synchronize()
        assert torch.equal(xi, x[:, i * P:(i + 1) * P])
        assert torch.equal(lbi.reshape(1), lb[i:i + 1]), (i, float(lbi), float(lb[i]))
        if need_rho:
            assert torch.equal(rbi.reshape(1), rb[i:i + 1])
        yb_sum += ybi
    torch.cuda.synchronize()
    assert rb is None or need_rho
    assert torch.allclose(yb, yb_sum, rtol=1e-6, atol=1e-6 * float(yb_sum.abs().max()))


def test_mask_recording_gives_the_full_recordings_gradients(dev):
    """ADMM_REC_MASKS (single solve, fused 256 x 256): lambda_bar and y_bar bitwise those of the full
    trajectory; rho_bar is refused."""
    y = torch.from_numpy(synth.make_batch(2, 256, 256, synth.gaussian_psf(9, 1.5), P=1, g0=2)).to(dev)
    h = torch.from_numpy(synth.gaussian_psf(9, 1.5)).to(dev)
    xb = torch.randn_like(y)
    x1, r1 = admm_deconv.tvd_fft_record(y, 0.0041, 0.021, h, False, 25, need_h=False)
    yb1, _, lb1, _ = admm_deconv.tvd_fft_backward_recorded(r1, x1, xb)
    x2, r2 = admm_deconv.tvd_fft_record(y, 0.0041, 0.021, h, False, 25, need_h=False, need_rho=False)
    yb2, _, lb2, rb2 = admm_deconv.tvd_fft_backward_recorded(r2, x2, xb, need_rho=False)
    torch.cuda.synchronize()
    assert torch.equal(x1, x2) and torch.equal(yb1, yb2) and torch.equal(lb1, lb2) and rb2 is None
    x3, r3 = admm_deconv.tvd_fft_record(y, 0.0041, 0.021, h, False, 25, need_h=False, need_rho=False)
    with pytest.raises(_lib.AdmmError) as e:
        admm_deconv.tvd_fft_backward_recorded(r3, x3, xb, need_rho=True)
    assert e.value.code == _lib.ADMM_E_INVALID
    # the combined call takes the mask trajectory by itself when rho_bar is not requested
    c = admm_deconv.tvd_fft_backward(y, xb, 0.0041, 0.021, h, False, 25, need_h=False, need_rho=False)
    torch.cuda.synchronize()
    assert torch.equal(c[1], yb1) and torch.equal(c[3], lb1)


def test_multi_validation(dev):
    y = torch.zeros((1, 1, 128, 128), device=dev)
    with pytest.raises(ValueError):
        admm_deconv.tvd_fft_multi(y, [0.01, 0.01], [0.1, 0.2], 5)
    y = torch.zeros((1, 1, 256, 256), device=dev)
    x, rec = admm_deconv.tvd_fft_multi(y, [0.01, 0.02], [0.1, 0.2], 5, record=True, need_rho=False)
    with pytest.raises(ValueError):
        admm_deconv.tvd_fft_multi_backward_recorded(rec, x, torch.zeros_like(x), need_rho=True)
    out = ctypes_null_replay(dev)
    assert out == _lib.ADMM_E_INVALID
    z = admm_deconv.tvd_fft_multi(torch.ones((1, 2, 256, 256), device=dev), [0.01, 0.02], [0.1, 0.2], 0)
    torch.cuda.synchronize()
    assert z.shape == (1, 4, 256, 256) and float(z.abs().max()) == 0.0


def ctypes_null_replay(dev):
    """A multi-branch replay on a workspace that holds no recording fails with ADMM_E_INVALID."""
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    xb = torch.zeros((1, 2, 256, 256), device=dev)
    return _lib.load().admm_tvd_backward_multi_recorded_dev_f32(xb.data_ptr(), None, xb.data_ptr(), None, 256, 256, 1,
                                                                1, 2, 5, xb.data_ptr(), ws.data_ptr(), ws.numel(), None)


def test_multi_deterministic(dev):
    y = torch.from_numpy(synth.make_batch(4, 256, 256, None, P=3, sigma=0.1)).to(dev)
    lams, rhos = _branch_scalars(dev, 5)
    xb = torch.randn((4, 15, 256, 256), device=dev)
    outs = []
    for _ in range(2):
        x, rec = admm_deconv.tvd_fft_multi(y, lams, rhos, 30, record=True, need_rho=False)
        outs.append((x,) + admm_deconv.tvd_fft_multi_backward_recorded(rec, x, xb, need_rho=False)[:2])
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(*outs))


@pytest.mark.parametrize("n,B,P,K", [(5, 2, 3, 12), (2, 1, 1, 1), (3, 3, 1, 2)])
def test_multi_iso_is_the_branches(dev, n, B, P, K):
    """Isotropic: forward bitwise the single fused solves; lambda_bar bitwise the single fused sweeps; y_bar
    their sum to rounding."""
    y = torch.from_numpy(synth.make_batch(B, 256, 256, None, P=P, sigma=0.1, g0=4)).to(dev)
    lams, rhos = _branch_scalars(dev, n, seed=11)
    xp = admm_deconv.tvd_fft_multi(y, lams, rhos, K, isotropic=True)
    xb = torch.randn((B, n * P, 256, 256), device=dev)
    x, rec = admm_deconv.tvd_fft_multi(y, lams, rhos, K, record=True, need_rho=False, isotropic=True)
    yb, lb, rb = admm_deconv.tvd_fft_multi_backward_recorded(rec, x, xb, need_rho=False)
    yb_sum = torch.zeros_like(y)
    for i in range(n):
        xi, reci = admm_deconv.tvd_fft_record(y, lams[i], rhos[i], None, True, K, need_rho=False)
        ybi, _, lbi, _ = admm_deconv.tvd_fft_backward_recorded(reci, xi, xb[:, i * P:(i + 1) * P].contiguous(),
                                                               need_rho=False)
        torch.cuda.synchronize()
        assert torch.equal(xi, x[:, i * P:(i + 1) * P]), i
        assert torch.equal(lbi.reshape(1), lb[i:i + 1]), (i, float(lbi), float(lb[i]))
        yb_sum += ybi
    torch.cuda.synchronize()
    assert rb is None and torch.equal(x, xp)
    assert torch.allclose(yb, yb_sum, rtol=1e-6, atol=1e-6 * float(yb_sum.abs().max()))


@pytest.mark.min_planes_rule
@pytest.mark.parametrize("n,B,P,K", [(5, 2, 3, 12), (2, 1, 1, 1), (3, 3, 1, 2), (4, 5, 3, 6)])
def test_multi_iso_2pass_is_the_branches(dev, n, B, P, K):
    """Below the plane-count rule (ADMM_OPT_MIN_PLANES at its default; 111 planes in all or fewer) the merged
    isotropic grid runs the 2-pass kernels over every branch's planes (admm_launch.hip run_multi_2pass_iso_fwd /
    _bwd, the reference's training configuration: 5 branches x batch 2 x RGB, train_cfg.json:10-14).  Each branch
    alone is below the rule too, so it runs the same kernels: forward bitwise, lambda_bar to the fp64 order of its
    partial rows (the rows are laid out per branch), y_bar the branches' sum to rounding."""
    assert _lib.get_option("MIN_PLANES") == -1 and n * B * P < 112
    y = torch.from_numpy(synth.make_batch(B, 256, 256, None, P=P, sigma=0.1, g0=4)).to(dev)
    lams, rhos = _branch_scalars(dev, n, seed=13)
    _lib.profile_reset()
    _lib.profile_enable(True)
    try:
        xp = admm_deconv.tvd_fft_multi(y, lams, rhos, K, isotropic=True)
        columns = _lib.profile_get(_lib.K_COLUMN)[1]
    finally:
        _lib.profile_enable(False)
    assert columns == K, columns   # one column pass per iteration: the 2-pass kernels, one grid for all branches
    xb = torch.randn((B, n * P, 256, 256), device=dev)
    x, rec = admm_deconv.tvd_fft_multi(y, lams, rhos, K, record=True, need_rho=False, isotropic=True)
    yb, lb, rb = admm_deconv.tvd_fft_multi_backward_recorded(rec, x, xb, need_rho=False)
    yb_sum = torch.zeros_like(y)
    for i in range(n):
        xi, reci = admm_deconv.tvd_fft_record(y, lams[i], rhos[i], None, True, K, need_rho=False)
        ybi, _, lbi, _ = admm_deconv.tvd_fft_backward_recorded(reci, xi, xb[:, i * P:(i + 1) * P].contiguous(),
                                                               need_rho=False)
        torch.cuda.synchronize()
        assert torch.equal(xi, x[:, i * P:(i + 1) * P]), i
        a, b = float(lbi), float(lb[i])
        assert abs(a - b) <= 1e-6 * abs(a) + 1e-30, (i, a, b)
        yb_sum += ybi
    torch.cuda.synchronize()
    assert rb is None and torch.equal(x, xp)
    assert torch.allclose(yb, yb_sum, rtol=1e-6, atol=1e-6 * float(yb_sum.abs().max()))


def test_multi_iso_vs_oracle_and_refusals(dev):
    y = synth.make_batch(2, 256, 256, None, P=3, sigma=0.1, g0=8)
    lams, rhos = _branch_scalars(dev, 3, seed=2)
    x = admm_deconv.tvd_fft_multi(torch.from_numpy(y).to(dev), lams, rhos, 15, isotropic=True).cpu().numpy()
    for i in (0, 2):
        ref = oracle_torch.tvd_fft_torch(torch.from_numpy(y.astype(np.float64)),
                                         torch.tensor(float(lams[i]), dtype=torch.float64),
                                         torch.tensor(float(rhos[i]), dtype=torch.float64), None, True, 15).numpy()
        assert_parity(x[:, 3 * i:3 * i + 3], ref, what=f"iso branch {i}")
    yt = torch.from_numpy(y).to(dev)
    with pytest.raises(ValueError):
        admm_deconv.tvd_fft_multi(yt, lams, rhos, 5, record=True, need_rho=True, isotropic=True)
    # the C-ABI refuses rho_bar from an isotropic recording
    x, rec = admm_deconv.tvd_fft_multi(yt, lams, rhos, 5, record=True, need_rho=False, isotropic=True)
    scal = torch.zeros(6, device=dev)
    ws_ptr, ws_len = rec.workspace.get(0, dev, None)
    rc = _lib.load().admm_tvd_backward_multi_recorded_dev_f32(x.data_ptr(), None, scal.data_ptr(), scal.data_ptr() + 12,
                                                              256, 256, 3, 2, 3, 5, x.data_ptr(), ws_ptr, ws_len, None)
    assert rc == _lib.ADMM_E_INVALID
