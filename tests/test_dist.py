"""CPU, world_size 2 (and 3) over gloo: batch sharding + gather (admm_deconv.parallel) reassembles exactly
the single-process result -- the one-shot solve_sharded and the chunked, pipelined ShardGather schedule
bench.py runs for BASELINE c3.  The per-rank solve here is the CPU oracle standing in for the GPU solve
(the product path has no CPU path); tests/test_gpu_dist_aniso.py runs the same schedule with the HIP
solve, and on MI355X bench.py runs it with backend "nccl" (RCCL over xGMI)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_np as o
from admm_deconv import parallel, synth

B, M, N, K = 6, 32, 32, 5
PSF = synth.gaussian_psf(5, 1.0)


def _solve(y):
    x = o.to_c(o.tvd_fft_literal(o.from_c(y.numpy().astype(np.float64)), np.float32(0.0041), np.float32(0.021),
                                 o.psf_from_c(PSF), False, K))
    return torch.from_numpy(x.astype(np.float32))


def _solve_into(y, x):
    x.copy_(_solve(y))


def _worker_pipelined(rank, world, port, q, n_local, chunks, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    y = torch.from_numpy(synth.make_batch(n_local, M, N, PSF, g0=rank * n_local))
    calls = []

    def solve(ys, xs):
        calls.append(ys.shape[0])
        _solve_into(ys, xs)

    sg = parallel.ShardGather(y, solve, chunks=chunks)
    for _ in range(steps):
        sg.step()
    sg.wait()
    if rank == 0:
        q.put((sg.gathered().numpy().copy(), calls))
    else:
        assert sg.gathered() is None
    dist.barrier()
    dist.destroy_process_group()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, count = parallel.shard_range(B, world, rank)
    y = torch.from_numpy(synth.make_batch(count, M, N, PSF, g0=start))
    full0 = parallel.solve_sharded(y, _solve, gather="rank0")
    full_all = parallel.solve_sharded(y, _solve, gather="all")
    if rank == 0:
        q.put((full0.numpy(), full_all.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shard_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    g0, gall = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ref = _solve(torch.from_numpy(synth.make_batch(B, M, N, PSF))).numpy()
    assert np.array_equal(g0, ref) and np.array_equal(gall, ref)


@pytest.mark.parametrize("world,n_local,chunks", [(2, 3, 1), (2, 3, 2), (3, 2, 3)])
def test_pipelined_shard_gather(world, n_local, chunks):
    """The c3 schedule: every rank solves its shard in `chunks` slices and each slice is gathered to
    rank 0 as soon as it is solved; two steps back to back reuse the double-buffered outputs."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_pipelined, args=(r, world, port, q, n_local, chunks, 2))
             for r in range(world)]
    for p in procs:
        p.start()
    got, calls = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(calls) == 2 * min(chunks, n_local) and sum(calls) == 2 * n_local   # chunks capped at the shard
    ref = _solve(torch.from_numpy(synth.make_batch(world * n_local, M, N, PSF))).numpy()
    assert np.array_equal(got, ref)


def test_shard_gather_refuses_steps_after_close():
    """a closed ShardGather (single process, CPU) refuses further steps instead of copying into
    released buffers."""
    y = torch.zeros(2, 1, 8, 8)
    sg = parallel.ShardGather(y, lambda ys, xs: xs.copy_(ys + 1))
    sg.step()
    assert torch.equal(sg.local(), torch.ones_like(y))
    sg.close()
    with pytest.raises(RuntimeError):
        sg.step()
