"""CPU: the metrics oracle (oracle/oracle_metrics.py) -- identities, and agreement with the
independent fp64 torch restatement used for the gradient checks (tests/metrics_torch.py)."""
import numpy as np
import torch

import metrics_torch as mt
import oracle_metrics as om
import oracle_np as o


def _pair(shape=(2, 3, 24, 20), seed=0):
    rng = np.random.default_rng(seed)
    x = rng.random(shape)
    y = np.clip(x + 0.05 * rng.standard_normal(shape), 0, 1)
    return x, y


def test_identities():
    x, y = _pair()
    assert abs(om.ssim(o.from_c(x), o.from_c(x))[0] - 1.0) < 1e-12
    assert om.gmsd(o.from_c(x), o.from_c(x))[0] < 1e-7
    assert om.ssim(o.from_c(x), o.from_c(y))[0] < 1.0
    assert om.gmsd(o.from_c(x), o.from_c(y))[0] > 0.0
    assert np.isinf(om.peak_snr(o.from_c(x), o.from_c(x)))


def test_oracle_matches_torch_restatement():
    x, y = _pair(seed=1)
    xt, yt = torch.from_numpy(x), torch.from_numpy(y)
    _, s_np = om.ssim(o.from_c(x), o.from_c(y))
    _, g_np = om.gmsd(o.from_c(x), o.from_c(y))
    assert np.allclose(mt.ssim_per_image(xt, yt).numpy(), s_np, rtol=1e-12, atol=1e-12)
    assert np.allclose(mt.gmsd_per_image(xt, yt).numpy(), g_np, rtol=1e-10, atol=1e-12)
    box = np.full(5, 0.2)
    assert np.allclose(mt.ssim_per_image(xt, yt, box).numpy(), om.ssim(o.from_c(x), o.from_c(y), box)[1])


def test_ssim_same_padding_shape():
    x, y = _pair(shape=(1, 1, 16, 16), seed=2)
    full, per = om.ssim(o.from_c(x), o.from_c(y), crop=False)
    assert per.shape == (1,) and 0 < full < 1
