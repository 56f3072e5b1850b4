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

LAM, RHO, K = 0.0041, 0.021, 6
CASES = {"fused": (256, 256, 15, 2.5), "2pass": (128, 64, 7, 1.2)}


def _batch(case, n, g0=0):
    M, N, k, sig = CASES[case]
    h = synth.gaussian_psf(k, sig)
    return synth.make_batch(n, M, N, h, g0=g0), h


def _worker(rank, world, port, q, case, n_local, chunks, engine):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    y, h = _batch(case, n_local, g0=rank * n_local)
    yt, ht = torch.from_numpy(y).to(dev), torch.from_numpy(h).to(dev)
    ws = admm_deconv.Workspace()

    def solve(ys, xs):
        admm_deconv.tvd_fft(ys, LAM, RHO, ht, False, K, out=xs, workspace=ws)

    sg = parallel.ShardGather(yt, solve, chunks=chunks, engine=engine)
    sg.step()
    sg.step()
    sg.wait()
    torch.cuda.synchronize()
    dist.barrier()   # ipc: rank 0's buffer is complete once every rank's copies have finished
    q.put((rank, None if rank else sg.gathered().cpu().numpy().copy(), sg.local().cpu().numpy(), sg.engine))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("case,chunks,engine,world", [
    ("fused", 1, "rccl", 2), ("fused", 2, "rccl", 2), ("2pass", 2, "rccl", 2),
    ("fused", 1, "ipc", 2), ("fused", 2, "ipc", 2), ("2pass", 3, "ipc", 2), ("2pass", 2, "ipc", 4)])
def test_aniso_shard_gather_two_processes(dev, case, chunks, engine, world):
    """engine "rccl" runs dist.gather (here gloo); "ipc" copies every solved slice into rank 0's receive
    buffer opened through a HIP IPC handle (on this box all ranks share the one GPU; 4 ranks = 3 peers
    writing into one shared buffer)."""
    n_local = 3
    y, h = _batch(case, world * n_local)
    ref = admm_deconv.tvd_fft(torch.from_numpy(y).to(dev), LAM, RHO, torch.from_numpy(h).to(dev), False, K)
    ref = ref.cpu().numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, case, n_local, chunks, engine))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(r[3] == engine for r in res), [r[3] for r in res]   # no silent fallback
    assert np.array_equal(res[0][1], ref)
    for r in range(world):
        assert np.array_equal(res[r][2], ref[r * n_local:(r + 1) * n_local])


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
