"""GPU: the isotropic prox over a batch sharded across 2 processes sharing the one GPU (gloo carries
the M x N maps through admm_batch_reducer; on a multi-GPU node the same call runs over RCCL).
The shards must reassemble the single-process solve of the whole batch (forward and adjoint), up to
the fp32 rounding of the differently ordered batch sums.  64^2 runs the 2-pass kernels; 256^2 the
split-iteration kernels of plane_iso.hip (their batch sums split into shard sum / all-reduce / factor),
with the fused reverse sweep when rho_bar is not requested."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import admm_deconv
from admm_deconv import parallel, synth

pytestmark = pytest.mark.gpu

B, K = 6, 8
LAM, RHO = 0.0041, 0.021


def _inputs(M, nb=B):
    h = synth.gaussian_psf(7, 1.2)
    y = synth.make_batch(nb, M, M, h)
    xbar = np.random.default_rng(11).standard_normal(y.shape).astype(np.float32)
    return h, y, xbar


def _worker(rank, world, port, q, M, need_rho, resident=0, nb=B, min_planes=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from admm_deconv import _lib
    _lib.set_option("RESIDENT", resident if resident else 1)
    # 0: the parent's reference solve runs the per-plane kernels too (conftest); > 0: a threshold the shards
    # straddle (a sharded isotropic call must ignore it)
    _lib.set_option("MIN_PLANES", min_planes)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    h, y, xbar = _inputs(M, nb)
    start, count = parallel.shard_range(nb, world, rank)
    dev = torch.device("cuda", 0)
    ys = torch.from_numpy(y[start:start + count]).to(dev)
    xb = torch.from_numpy(xbar[start:start + count]).to(dev)
    ht = torch.from_numpy(h).to(dev)
    g = dist.group.WORLD
    x = admm_deconv.tvd_fft(ys, LAM, RHO, ht, True, K, group=g)
    x2, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(ys, xb, LAM, RHO, ht, True, K, group=g, need_h=need_rho,
                                                      need_rho=need_rho)
    torch.cuda.synchronize()
    q.put((rank, x.cpu().numpy(), x2.cpu().numpy(), yb.cpu().numpy(), None if hb is None else hb.cpu().numpy(),
           float(lb), None if rb is None else float(rb)))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rel(a, b):
    return float(np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b))


@pytest.mark.parametrize("M,need_rho,resident", [(64, True, 0), (256, True, 0), (256, False, 0), (120, False, 2)],
                         ids=["2pass", "fused-fwd", "fused-fwd+sweep", "resident-iso"])
def test_iso_sharded_two_processes(dev, M, need_rho, resident):
    """resident-iso: 120 x 120 with ADMM_OPT_RESIDENT = 2, the isotropic CU-resident solve (resident_iso_kernel),
    whose norm kernel splits into the shard sum, the reducer and the factor the same way."""
    from admm_deconv import _lib
    _lib.set_option("RESIDENT", resident if resident else 1)
    try:
        _iso_sharded(dev, M, need_rho, resident)
    finally:
        _lib.set_option("RESIDENT", 1)


@pytest.mark.parametrize("rule", [4, 0], ids=["rule4", "norule"])
@pytest.mark.parametrize("need_rho", [False, True], ids=["sweep", "rho"])
def test_iso_uneven_shards_straddling_the_plane_count_rule(dev, need_rho, rule):
    """7 planes at 256^2 on 2 ranks are shards of 4 and 3.  With ADMM_OPT_MIN_PLANES = 4 a shard's
    own plane count would put rank 0 on the fused isotropic kernels and rank 1 on the 2-pass ones, which hand
    the reducer their sum maps in different layouts.  A sharded call ignores the rule, so both take the
    per-plane kernels and the shards reassemble the single-process solve."""
    from admm_deconv import _lib
    assert parallel.shard_range(7, 2, 0)[1] == 4 and parallel.shard_range(7, 2, 1)[1] == 3
    _lib.set_option("MIN_PLANES", 4)
    try:
        assert _lib.query_paths(256, 256, True, 7, planes=4)[0] == "fused_iso"
        assert _lib.query_paths(256, 256, True, 7, planes=3)[0] == "2pass_iso"
    finally:
        _lib.set_option("MIN_PLANES", 0)
    _iso_sharded(dev, 256, need_rho, 0, nb=7, min_planes=rule)


def _check_y_bar(yb, yb0):
    """Sharded vs single-process y_bar.  The shards' batch norms are summed in another order than the single
    process's, so ||s_k|| can differ in its last bit; where ||s_k|| is within that of tau the BT branch
    1[||s_k|| > tau] flips, and the tau / ||s||^3 term moves y_bar of that PIXEL in every plane by far more than
    rounding (test_gpu_adjoint_masked.py holds each sweep to 1e-5 against the oracle conditioned on its own
    branches).  So: at most 0.1 % of the pixels may differ by more than 1e-3 max|y_bar| (such flips), and the
    rest must agree to 1e-4 rel-L2.  A layout mix-up of the reducer's maps would corrupt every pixel."""
    yb, yb0 = np.asarray(yb, np.float64), np.asarray(yb0, np.float64)
    d = np.abs(yb - yb0).reshape(-1, *yb.shape[-2:]).max(axis=0)          # per pixel, over planes and channels
    spots = d > 1e-3 * np.abs(yb0).max()
    per_plane = [f"{_rel(yb[i], yb0[i]):.1e}" for i in range(yb.shape[0])]
    assert spots.mean() <= 1e-3, f"{int(spots.sum())} pixels differ (per-plane rel-L2 {per_plane})"
    keep = ~spots
    rest = _rel(yb[..., keep], yb0[..., keep])
    assert rest < 1e-4, f"y_bar away from {int(spots.sum())} flipped pixels: rel-L2 {rest:.2e} (per plane {per_plane})"


def _iso_sharded(dev, M, need_rho, resident, nb=B, min_planes=0):
    if resident:
        from admm_deconv import _lib
        assert _lib.query_paths(M, M, True, 7)[0] == "resident_iso"
    h, y, xbar = _inputs(M, nb)
    ht = torch.from_numpy(h).to(dev)
    x0 = admm_deconv.tvd_fft(torch.from_numpy(y).to(dev), LAM, RHO, ht, True, K).cpu().numpy()
    _, yb0, hb0, lb0, rb0 = admm_deconv.tvd_fft_backward(torch.from_numpy(y).to(dev),
                                                        torch.from_numpy(xbar).to(dev), LAM, RHO, ht, True, K,
                                                        need_h=need_rho, need_rho=need_rho)
    yb0, lb0 = yb0.cpu().numpy(), float(lb0)
    # the spread of the scalar gradients under a reordered batch sum: the same single-process solve with the
    # batch in other plane orders (mathematically identical: pixelnorm and every gradient sum over the planes)
    spread = {"lam": 0.0, "rho": 0.0, "h": 0.0}
    for order in (np.arange(nb)[::-1], np.r_[np.arange(0, nb, 2), np.arange(1, nb, 2)]):
        _, _, hbp, lbp, rbp = admm_deconv.tvd_fft_backward(
            torch.from_numpy(np.ascontiguousarray(y[order])).to(dev), torch.from_numpy(np.ascontiguousarray(xbar[order])).to(dev),
            LAM, RHO, ht, True, K, need_h=need_rho, need_rho=need_rho)
        spread["lam"] = max(spread["lam"], abs(float(lbp) - lb0))
        if need_rho:
            spread["rho"] = max(spread["rho"], abs(float(rbp) - float(rb0)))
            spread["h"] = max(spread["h"], float(np.linalg.norm(hbp.cpu().numpy() - hb0.cpu().numpy())))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, M, need_rho, resident, nb, min_planes))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    x = np.concatenate([r[1] for r in res])
    assert _rel(x, x0) < 1e-5
    assert _rel(np.concatenate([r[2] for r in res]), x0) < 1e-5
    _check_y_bar(np.concatenate([r[3] for r in res]), yb0)
    # scalar gradients: the shards' contributions add up to the whole batch's within 1e-3, widened by twice the
    # reordered-batch spread (a BT branch flip moves them as it moves y_bar above; the sharded and the
    # single-process sums are two orderings, each within that spread of the others)
    assert abs(sum(r[5] for r in res) - lb0) <= 1e-3 * abs(lb0) + 2 * spread["lam"], (sum(r[5] for r in res), lb0, spread)
    if need_rho:
        hb0n = hb0.cpu().numpy()
        dh = float(np.linalg.norm(sum(r[4] for r in res) - hb0n))
        assert dh <= 1e-3 * float(np.linalg.norm(hb0n)) + 2 * spread["h"], (dh, spread)
        assert abs(sum(r[6] for r in res) - float(rb0)) <= 1e-3 * abs(float(rb0)) + 2 * spread["rho"], spread
    else:
        assert rb0 is None and all(r[6] is None for r in res)
