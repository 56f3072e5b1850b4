"""CPU, world_size 2 over gloo: the isotropic prox over a SHARDED batch.

BT's pixelnorm spans the whole batch (ops.jl:6), so a sharded solve needs the cross-shard sum of an
M x N map every iteration (and of the batch map R every reverse step).  Each rank runs the numpy
kernel-sequence model (tests/kernel_model.py) on its own slice with `batch_sum` routed through the
package's actual admm_batch_reducer callback (admm_deconv.ops._make_reducer) over a workspace
tensor -- the host logic the HIP library calls on a GPU box.  The shards' x / y_bar must reassemble
the unsharded result, and their h_bar / lambda_bar / rho_bar contributions must add up to it."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import kernel_model as km
from admm_deconv import ops, parallel, synth

B, M, N, K = 5, 16, 16, 4
LAM, RHO = 0.02, 0.1
PSF = synth.gaussian_psf(3, 0.8).astype(np.float64)


def _inputs():
    y = synth.make_batch(B, M, N, PSF.astype(np.float32)).astype(np.float64).reshape(B, N, M)
    xbar = np.random.default_rng(5).standard_normal(y.shape)
    return y, xbar


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    y, xbar = _inputs()
    start, count = parallel.shard_range(B, world, rank)
    ws = ops.Workspace()
    ws.get(4096 + 4 * M * N, torch.device("cpu"))
    red, fn = ops._make_reducer(ws, None)
    calls = [0]

    def batch_sum(a):
        # stage the shard's map in the workspace and hand the C callback a pointer into it
        base = ws._buf.data_ptr()
        off = (-base) % 256 + 1024
        view = ws._buf[off: off + 4 * a.size].view(torch.float32)
        view.copy_(torch.from_numpy(a.astype(np.float32).reshape(-1)))
        rc = fn(base + off, a.size, None, None)
        assert rc == 0
        calls[0] += 1
        return view.numpy().astype(np.float64).reshape(a.shape)

    out = km.tvd_model_grads(y[start:start + count], LAM, RHO, PSF, K, xbar[start:start + count], iso=True,
                             batch_sum=batch_sum)
    q.put((rank, start, count, out, calls[0]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_iso_sharded_matches_unsharded():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    y, xbar = _inputs()
    x0, yb0, hb0, lb0, rb0 = km.tvd_model_grads(y, LAM, RHO, PSF, K, xbar, iso=True)
    x = np.concatenate([r[3][0] for r in res])
    yb = np.concatenate([r[3][1] for r in res])
    # the map crosses the reducer as fp32: compare at fp32 resolution
    assert np.allclose(x, x0, rtol=1e-5, atol=1e-6 * np.abs(x0).max())
    assert np.allclose(yb, yb0, rtol=1e-4, atol=1e-5 * np.abs(yb0).max())
    hb = sum(r[3][2] for r in res)
    assert np.linalg.norm(hb - hb0) / np.linalg.norm(hb0) < 1e-4
    lb = sum(r[3][3] for r in res)
    rb = sum(r[3][4] for r in res)
    assert abs(lb - lb0) <= 1e-4 * abs(lb0) and abs(rb - rb0) <= 1e-4 * abs(rb0)
    # forward K-1 norm maps + reverse K-1 R maps per shard
    assert all(r[4] == 2 * (K - 1) for r in res)
