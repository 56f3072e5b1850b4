"""GPU: the isotropic prox over a batch sharded across 2 processes sharing the one GPU (gloo carries
the M x N maps through admm_batch_reducer; on a multi-GPU node the same call runs over RCCL).
The shards must reassemble the single-process solve of the whole batch (forward and adjoint), up to
the fp32 rounding of the differently ordered batch sums."""
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

B, M, N, K = 6, 64, 64, 8
LAM, RHO = 0.0041, 0.021


def _inputs():
    h = synth.gaussian_psf(7, 1.2)
    y = synth.make_batch(B, M, N, h)
    xbar = np.random.default_rng(11).standard_normal(y.shape).astype(np.float32)
    return h, y, xbar


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    h, y, xbar = _inputs()
    start, count = parallel.shard_range(B, world, rank)
    dev = torch.device("cuda", 0)
    ys = torch.from_numpy(y[start:start + count]).to(dev)
    xb = torch.from_numpy(xbar[start:start + count]).to(dev)
    ht = torch.from_numpy(h).to(dev)
    g = dist.group.WORLD
    x = admm_deconv.tvd_fft(ys, LAM, RHO, ht, True, K, group=g)
    x2, yb, hb, lb, rb = admm_deconv.tvd_fft_backward(ys, xb, LAM, RHO, ht, True, K, group=g)
    torch.cuda.synchronize()
    q.put((rank, x.cpu().numpy(), x2.cpu().numpy(), yb.cpu().numpy(), hb.cpu().numpy(), float(lb), float(rb)))
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


def test_iso_sharded_two_processes(dev):
    h, y, xbar = _inputs()
    ht = torch.from_numpy(h).to(dev)
    x0 = admm_deconv.tvd_fft(torch.from_numpy(y).to(dev), LAM, RHO, ht, True, K).cpu().numpy()
    _, yb0, hb0, lb0, rb0 = admm_deconv.tvd_fft_backward(torch.from_numpy(y).to(dev),
                                                        torch.from_numpy(xbar).to(dev), LAM, RHO, ht, True, K)
    yb0, hb0, lb0, rb0 = yb0.cpu().numpy(), hb0.cpu().numpy(), float(lb0), float(rb0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
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
    assert _rel(sum(r[4] for r in res), hb0) < 1e-3
    assert abs(sum(r[5] for r in res) - lb0) <= 1e-3 * abs(lb0)
    assert abs(sum(r[6] for r in res) - rb0) <= 1e-3 * abs(rb0)
