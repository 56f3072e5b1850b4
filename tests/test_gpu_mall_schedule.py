"""GPU: the MALL-resident forward schedule (ADMM_OPT_MALL_STREAMS, admm_paths.hip forward_chunks; VERDICT r05
Next #3).  An anisotropic 2-pass batch whose per-iteration working set (28 B/px) exceeds twice the 256 MiB
Infinity Cache runs in chunks of ~224 MiB / n planes, round-robin on the caller's stream and n - 1 library
streams.  Each chunk is the same per-plane computation as in the whole-batch grid, so the result is bitwise the
one-stream solve; ordering against the caller's stream goes through events (fork / join), checked here by
consuming x on the caller's stream right after the call, and by capturing the call in a HIP graph.
Reference: /root/reference/src/ops/ops.jl:168-173 (the anisotropic planes are independent)."""
import numpy as np
import pytest
import torch

import admm_deconv
from admm_deconv import _lib, synth
from parity import assert_parity, oracle_solve

pytestmark = pytest.mark.gpu

LAM, RHO = 0.0041, 0.021


def _batch(planes, M, h, g0=5):
    base = synth.make_batch(8, M, M, h, g0=g0)
    return np.concatenate([base] * (planes // 8) + [base[: planes % 8]])


def _solve(dev, y, h, K, streams):
    with _lib.option("MALL_STREAMS", streams):
        ws = admm_deconv.Workspace()
        x = admm_deconv.tvd_fft(y, LAM, RHO, h, False, K, workspace=ws)
        s = float(x.double().sum())   # consumed on the caller's stream right away: the join must order it
        torch.cuda.synchronize()
    return x, s


@pytest.mark.parametrize("planes", [81, 100], ids=["81planes-ragged", "100planes"])
def test_mall_schedule_bitwise_one_stream(dev, planes):
    M, K = 512, 6
    assert _lib.get_option("MALL_STREAMS") == 4
    assert _lib.query_paths(M, M, False, 15, planes=planes)[0] == "2pass"
    h = synth.gaussian_psf(15, 2.5)
    y = torch.from_numpy(_batch(planes, M, h)).to(dev)
    ht = torch.from_numpy(h).to(dev)
    b4 = _lib.workspace_bytes(M, M, 1, planes, 15, 15, False)
    with _lib.option("MALL_STREAMS", 1):
        b1 = _lib.workspace_bytes(M, M, 1, planes, 15, 15, False)
    # 8 planes of 512^2 per chunk, 4 chunk workspaces, against the whole batch's one
    assert b4 < b1, (b4, b1)
    x4, s4 = _solve(dev, y, ht, K, 4)
    x1, s1 = _solve(dev, y, ht, K, 1)
    assert torch.equal(x4, x1)
    assert s4 == s1
    # two streams (16-plane chunks) the same
    x2, _ = _solve(dev, y, ht, K, 2)
    assert torch.equal(x2, x1)
    ref = oracle_solve(_batch(planes, M, h)[:2], LAM, RHO, h, False, K, "spectral", what="mall 512^2")
    assert_parity(x4[:2].cpu().numpy(), ref, what="mall schedule 512^2")


def test_mall_schedule_c4_config_full_k(dev):
    """The c4 configuration (512^2, 15x15 Gaussian PSF sigma 2.5, K = 50) over 96 planes -- 12 chunks of 8 on 4
    streams: bitwise the one-stream solve, and planes of the first, a middle and the last chunk against the oracle."""
    M, K, planes = 512, 50, 96
    assert _lib.forward_schedule(M, M, False, 15, planes) == (8, 4)
    h = synth.gaussian_psf(15, 2.5)
    y_np = _batch(planes, M, h, g0=77)
    y = torch.from_numpy(y_np).to(dev)
    ht = torch.from_numpy(h).to(dev)
    x4, _ = _solve(dev, y, ht, K, 4)
    x1, _ = _solve(dev, y, ht, K, 1)
    assert torch.equal(x4, x1)
    pick = [0, 45, 95]   # chunk 0 (stream 0), chunk 5 (stream 1), chunk 11 (stream 3)
    ref = oracle_solve(y_np[pick], LAM, RHO, h, False, K, "spectral", what="mall c4 K=50")
    assert_parity(x4[pick].cpu().numpy(), ref, what="mall schedule c4 K=50")


def test_mall_schedule_smooth_lengths(dev):
    """480 x 640 x 64 runs the smooth-length 2-pass kernels in 6-plane chunks on 4 streams: bitwise the whole batch."""
    N, M, B, K = 480, 640, 64, 4
    assert _lib.query_paths(M, N, False, 15, planes=B)[0] == "smooth"
    assert _lib.forward_schedule(M, N, False, 15, B) == (6, 4)
    h = synth.gaussian_psf(15, 2.5)
    base = synth.make_batch(8, M, N, h, g0=3)
    y = torch.from_numpy(np.concatenate([base] * 8)).to(dev)
    ht = torch.from_numpy(h).to(dev)
    x4, s4 = _solve(dev, y, ht, K, 4)
    x1, s1 = _solve(dev, y, ht, K, 1)
    assert torch.equal(x4, x1) and s4 == s1
    ref = oracle_solve(base[:1], LAM, RHO, h, False, K, "spectral", what="mall 480x640")
    assert_parity(x4[:1].cpu().numpy(), ref, what="mall schedule 480x640")


def test_mall_schedule_under_graph_capture(dev):
    """The fork / join events are graph nodes: a captured call replays to the eager result."""
    M, K, planes = 512, 4, 80
    h = synth.gaussian_psf(15, 2.5)
    y = torch.from_numpy(_batch(planes, M, h, g0=9)).to(dev)
    ht = torch.from_numpy(h).to(dev)
    ref, _ = _solve(dev, y, ht, K, 4)
    ws = admm_deconv.Workspace()
    out = torch.empty_like(y)
    admm_deconv.tvd_fft(y, LAM, RHO, ht, False, K, out=out, workspace=ws)   # sizes the workspace before capture
    torch.cuda.synchronize()
    out.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        admm_deconv.tvd_fft(y, LAM, RHO, ht, False, K, out=out, workspace=ws)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
