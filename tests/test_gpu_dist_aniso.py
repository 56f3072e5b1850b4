"""GPU: the anisotropic batch shard + gather of BASELINE c3 (/root/reference/src/ops/ops.jl:168-173: every
(image, channel) plane is independent) with the HIP solve on each rank.  Two processes share the one
GPU of the test box and talk over gloo; on an 8-GPU node bench.py runs the same ShardGather schedule
over RCCL.  The gathered batch must be bitwise the single-process solve of the whole batch, for the
fused 256x256 kernel and the 2-pass path, with one and with two slices per shard, and when bench.py
itself runs the schedule (`--gpus 2 --backend gloo`)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import admm_deconv
from admm_deconv import parallel, synth

pytestmark = pytest.mark.gpu

LAM, RHO = 0.0041, 0.021
CASES = {"fused": (256, 256, 15, 2.5, 6), "2pass": (128, 64, 7, 1.2, 6),
         "c3": (256, 256, 15, 2.5, 25)}   # BASELINE c3: 256x256, 15x15 PSF, K = 25


def _shard(case, n_local, rank, distinct):
    """Rank `rank`'s shard: `distinct` synthetic images of global index rank * distinct + i, tiled to n_local
    (bench.py's --distinct tiling: the c3 shard is 256 images, generating all of them on the host would
    take the test's time budget)."""
    M, N, k, sig, _ = CASES[case]
    h = synth.gaussian_psf(k, sig)
    base = synth.make_batch(distinct, M, N, h, g0=rank * distinct)
    reps = (n_local + distinct - 1) // distinct
    return np.ascontiguousarray(np.concatenate([base] * reps)[:n_local]), h


def _worker(rank, world, port, q, case, n_local, chunks, engine, distinct):
    try:
        _work(rank, world, port, q, case, n_local, chunks, engine, distinct)
    except BaseException:   # report instead of leaving the other ranks and the test waiting
        import traceback
        q.put((rank, "error", traceback.format_exc(), None))
        raise


def _work(rank, world, port, q, case, n_local, chunks, engine, distinct):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from admm_deconv import _lib
    _lib.set_option("MIN_PLANES", 0)   # the parent's reference solve runs the per-plane kernels too (conftest)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    K = CASES[case][4]
    y, h = _shard(case, n_local, rank, distinct)
    yt, ht = torch.from_numpy(y).to(dev), torch.from_numpy(h).to(dev)
    ws = [admm_deconv.Workspace() for _ in range(chunks)]
    slot = {}

    def solve(ys, xs):
        i = slot.setdefault(ys.data_ptr(), len(slot) % chunks)
        admm_deconv.tvd_fft(ys, LAM, RHO, ht, False, K, out=xs, workspace=ws[i])

    sg = parallel.ShardGather(yt, solve, chunks=chunks, engine=engine)
    sg.step()
    sg.gathered()         # with ipc, required before the next step (a peer must not run two steps ahead)
    sg.step()
    got = sg.gathered()   # collective: waits for every rank's device work (and, for ipc, a barrier)
    local = sg.local()
    ok_local = bool(torch.equal(local, admm_deconv.tvd_fft(yt, LAM, RHO, ht, False, K)))
    ok_full = None
    if rank == 0:
        # the single-process solve of the whole (global) batch, bitwise
        full = np.concatenate([_shard(case, n_local, r, distinct)[0] for r in range(world)])
        ref = admm_deconv.tvd_fft(torch.from_numpy(full).to(dev), LAM, RHO, ht, False, K)
        ok_full = bool(torch.equal(got.cpu(), ref.cpu()))   # gloo + rccl engine gathers into host memory
    else:
        assert got is None
    q.put((rank, ok_full, ok_local, sg.engine))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(case, chunks, engine, world, n_local, distinct, timeout):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, case, n_local, chunks, engine, distinct))
             for r in range(world)]
    for p in procs:
        p.start()
    res = []
    for _ in range(world):
        r = q.get(timeout=timeout)
        if r[1] == "error":
            for p in procs:
                p.kill()
            raise AssertionError(f"rank {r[0]} failed:\n{r[2]}")
        res.append(r)
    res.sort(key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[3] == engine for r in res), [r[3] for r in res]   # no silent fallback
    assert res[0][1] is True, "gathered batch differs from the single-process solve"
    assert all(r[2] for r in res), "a rank's local shard differs from its own solve"


@pytest.mark.parametrize("case,chunks,engine,world", [
    ("fused", 1, "rccl", 2), ("fused", 2, "rccl", 2), ("2pass", 2, "rccl", 2),
    ("fused", 1, "ipc", 2), ("fused", 2, "ipc", 2), ("2pass", 3, "ipc", 2), ("2pass", 2, "ipc", 4)])
def test_aniso_shard_gather_two_processes(dev, case, chunks, engine, world):
    """engine "rccl" runs dist.gather (here gloo); "ipc" copies every solved slice into rank 0's receive
    buffer opened through a HIP IPC handle (on this box all ranks share the one GPU; 4 ranks = 3 peers
    writing into one shared buffer)."""
    _run(case, chunks, engine, world, n_local=3, distinct=3, timeout=100)


def test_c3_full_size_eight_ranks(dev):
    """BASELINE c3 at its real per-rank size on the one GPU: 8 ranks x 256 images of 256x256 (2048 global),
    15x15 PSF, K = 25, two slices per shard, IPC push gather.  Rank 0's gathered batch is bitwise the
    single-process solve of all 2048 images, and every rank's shard its own solve (size-independent
    properties: the oracle itself would need minutes for 2048 planes at K = 25)."""
    _run("c3", 2, "ipc", 8, n_local=256, distinct=16, timeout=110)


def test_bench_two_ranks_gloo(dev):
    """bench.py --gpus 2 spawns its two ranks and runs the c3 schedule (here over gloo, both ranks on
    this box's one GPU, with a small batch); rank 0 prints one JSON line with n_gpus 2."""
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--batch", "8", "--steps", "2", "--warmup", "1", "--distinct", "4", "--chunks", "2"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=repo)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 16
    assert "IPC push gather" in d["config"]["parallelism"] and d["value"] > 0
    # the per-rank diagnostics of a multi-GPU record: what each rank saw and where its time went
    assert [r["rank"] for r in d["ranks"]] == [0, 1]
    for r in d["ranks"]:
        assert r["world_seen"] == 2 and r["backend"] == "gloo" and r["gather_engine"] == "ipc"
        assert r["ms_per_step"] > 0 and r["solve_only_ms_per_step"] > 0 and r["gather_tail_ms"] >= 0
        assert r["device"] == 0 and r["visible_devices"] >= 1
    assert d["solve_only"]["value"] > 0 and d["solve_only"]["ms_per_step"] > 0
    # --gather-engine both (default): the same steps gathered by RCCL (here gloo), timed per rank
    for r in d["ranks"]:
        assert r["other_engine"]["engine"] == "rccl" and r["other_engine"]["ms_per_step"] > 0
    assert d["solve_only"]["other_engine"]["engine"] == "rccl" and d["solve_only"]["other_engine"]["value"] > 0


def _ipc_worker(rank, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        from admm_deconv import _lib
        dist.init_process_group("gloo", rank=rank, world_size=2)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        # rank 0: a buffer inside a larger allocation (offset != 0, as a caching allocator hands out)
        big = torch.zeros(3 << 20, dtype=torch.float32, device=dev)
        view = big[(1 << 20) + 64: (2 << 20) + 64]
        obj = [None]
        if rank == 0:
            view.copy_(torch.arange(1 << 20, dtype=torch.float32, device=dev))
            torch.cuda.synchronize()
            obj = [_lib.ipc_get_handle(view.data_ptr())]
            assert obj[0][1] >= ((1 << 20) + 64) * 4     # the view's offset in its allocation
        dist.broadcast_object_list(obj, src=0)
        ok = True
        if rank == 1:
            handle, off = obj[0]
            base = _lib.ipc_open(handle, dev.index)
            local = torch.empty(1 << 20, dtype=torch.float32, device=dev)
            st = torch.cuda.Stream(device=dev)
            _lib.copy_async(local.data_ptr(), base + off, local.numel() * 4, st.cuda_stream)   # peer -> local
            st.synchronize()
            ok = bool(torch.equal(local, torch.arange(1 << 20, dtype=torch.float32, device=dev)))
            local.fill_(-1.0)
            _lib.copy_async(base + off, local.data_ptr(), 4096 * 4, st.cuda_stream)           # local -> peer
            st.synchronize()
            _lib.ipc_close(base, dev.index)
        dist.barrier()
        if rank == 0:
            torch.cuda.synchronize()
            ok = bool((view[:4096] == -1.0).all()) and bool(view[4096] == 4096.0) and bool((big[:1 << 20] == 0).all())
        q.put((rank, ok))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def test_ipc_handle_open_close_through_the_library(dev):
    """admm_ipc_get_handle / admm_ipc_open / admm_ipc_close (include/admm_deconv.h): rank 0 shares a buffer that
    sits at an offset inside a larger allocation; rank 1 maps it on its own device, reads it and writes into it
    with admm_copy_async, and unmaps it.  Both directions land where the offset says."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ipc_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] is True for r in res), res


def _ahead_worker(rank, port, q, stream_only):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=2)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        y = torch.ones(2, 1, 64, 64, device=dev)
        sg = parallel.ShardGather(y, lambda ys, xs: xs.copy_(ys), engine="ipc", stream_only=stream_only)
        assert sg.engine == "ipc"
        sg.step()
        try:
            sg.step()
            raised = False
        except RuntimeError:
            raised = True
        sg.gathered()
        q.put((rank, raised))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


@pytest.mark.parametrize("stream_only", [False, True])
def test_ipc_step_requires_gathered_unless_stream_only(dev, stream_only):
    """with the ipc engine a peer two steps ahead of rank dst would overwrite the receive buffer dst
    is reading, so step() raises unless gathered() followed the previous step -- except for stream_only
    callers (the benchmark), which never read the buffers between steps."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ahead_worker, args=(r, port, q, stream_only)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] is (not stream_only) for r in res), res


def _close_worker(rank, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=2)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        y = torch.full((4, 1, 512, 512), float(rank + 1), device=dev)
        sg = parallel.ShardGather(y, lambda ys, xs: xs.copy_(ys), engine="ipc", stream_only=True)
        assert sg.engine == "ipc"
        sg.step()
        sg.close()   # rank 1: its peer copy may still be in flight -- close() drains the comm stream first
        dist.barrier()
        ok = True
        if rank == 0:
            torch.cuda.synchronize(dev)
            got = sg.recv[0]
            ok = bool((got[:4] == 1.0).all()) and bool((got[4:] == 2.0).all())
        try:
            sg.step()
            raised = False
        except RuntimeError:
            raised = True
        q.put((rank, ok and raised and sg.remote is None))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException:
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def test_ipc_close_after_stream_only_step(dev):
    """close() right after a stream_only step (nothing waited for the peer copy) drains the copy
    stream before unmapping -- rank 0's buffer holds both shards -- and a later step() raises instead of copying
    to an unmapped address."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_close_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] is True for r in res), res


def test_copy_async_is_a_stream_ordered_device_copy(dev):
    """admm_copy_async (the IPC gather's peer copy, include/admm_deconv.h): a hipMemcpyAsync on the given stream,
    ordered after earlier work on that stream and before later work; NULL pointers are rejected; 0 bytes is a
    no-op."""
    from admm_deconv import _lib
    src = torch.arange(1 << 20, dtype=torch.float32, device=dev)
    dst = torch.zeros_like(src)
    st = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(st):
        src.mul_(2.0)                                         # earlier work on st
        _lib.copy_async(dst.data_ptr(), src.data_ptr(), src.numel() * 4, st.cuda_stream)
        dst.add_(1.0)                                         # later work on st
    st.synchronize()
    assert torch.equal(dst, torch.arange(1 << 20, dtype=torch.float32, device=dev) * 2 + 1)
    _lib.copy_async(dst.data_ptr(), src.data_ptr(), 0, st.cuda_stream)
    with pytest.raises(_lib.AdmmError):
        _lib.copy_async(0, src.data_ptr(), 4, st.cuda_stream)
