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


def _inputs(M):
    h = synth.gaussian_psf(7, 1.2)
    y = synth.make_batch(B, M, M, h)
    xbar = np.random.default_rng(11).standard_normal(y.shape).astype(np.float32)
    return h, y, xbar


def _worker(rank, world, port, q, M, need_rho, resident=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from admm_deconv import _lib
    _lib.set_option("RESIDENT", resident if resident else 1)
    _lib.set_option("MIN_PLANES", 0)   # the parent's reference solve runs the per-plane kernels too (conftest)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    h, y, xbar = _inputs(M)
    start, count = parallel.shard_range(B, world, rank)
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


def _iso_sharded(dev, M, need_rho, resident):
    if resident:
        from admm_deconv import _lib
        assert _lib.query_paths(M, M, True, 7)[0] == "resident_iso"
    h, y, xbar = _inputs(M)
    ht = torch.from_numpy(h).to(dev)
    x0 = admm_deconv.tvd_fft(torch.from_numpy(y).to(dev), LAM, RHO, ht, True, K).cpu().numpy()
    _, yb0, hb0, lb0, rb0 = admm_deconv.tvd_fft_backward(torch.from_numpy(y).to(dev),
                                                        torch.from_numpy(xbar).to(dev), LAM, RHO, ht, True, K,
                                                        need_h=need_rho, need_rho=need_rho)
    yb0, lb0 = yb0.cpu().numpy(), float(lb0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, M, need_rho, resident)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    x = np.concatenate([r[1] for r in res])
    assert _rel(x, x0) < 1e-5
    assert _rel(np.concatenate([r[2] for r in res]), x0) < 1e-5
    assert _rel(np.concatenate([r[3] for r in res]), yb0) < 1e-4
    assert abs(sum(r[5] for r in res) - lb0) <= 1e-3 * abs(lb0)
    if need_rho:
        assert _rel(sum(r[4] for r in res), hb0.cpu().numpy()) < 1e-3
        assert abs(sum(r[6] for r in res) - float(rb0)) <= 1e-3 * abs(float(rb0))
    else:
        assert rb0 is None and all(r[6] is None for r in res)
