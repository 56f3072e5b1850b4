"""Batch sharding across ranks (one process per GPU) and the output gather over RCCL.

The anisotropic solve is independent per (image, channel) plane (ops.jl:168-173), so a batch of B
images is split into contiguous per-rank ranges by GLOBAL image index (synthetic inputs are seeded
by global index, so a sharded run is bit-identical to the unsharded one) and solved with no
communication.  The only exchange is optional: gathering every rank's outputs to rank 0 (or to all
ranks) after the solve -- `torch.distributed` with backend "nccl" is RCCL over xGMI on MI355X;
with "gloo" the same code runs on CPU tensors for the multi-process tests.

The isotropic prox couples the whole batch (pixelnorm over dims 3,4, ops.jl:6), so its shards need a
per-iteration all-reduce of an M x N map.  That exchange lives inside the solve: pass `group=` to
`tvd_fft` / the layers (ops._make_reducer hands the library an admm_batch_reducer that all-reduces the
map over the group); this module only shards batches and gathers outputs.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib

__all__ = ["shard_range", "solve_sharded", "ShardGather"]


def shard_range(total, world, rank):
    """Contiguous [start, start+count) of `total` items owned by `rank` (first ranks take the remainder)."""
    base, rem = divmod(int(total), int(world))
    count = base + (1 if rank < rem else 0)
    start = rank * base + min(rank, rem)
    return start, count


def solve_sharded(y_local, solve, *, gather="none", total=None, group=None):
    """Run `solve(y_local)` on this rank's shard; optionally gather all shards.

    gather: "none" -> return the local result; "rank0" -> rank 0 returns the full batch (others None);
            "all"  -> every rank returns the full batch.
    Shards must have equal size for the collective path (the bench uses equal shards)."""
    x_local = solve(y_local)
    if gather == "none" or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return x_local
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if gather == "all":
        parts = [torch.empty_like(x_local) for _ in range(world)]
        dist.all_gather(parts, x_local.contiguous(), group=group)
        return torch.cat(parts)
    if gather == "rank0":
        parts = [torch.empty_like(x_local) for _ in range(world)] if rank == 0 else None
        dist.gather(x_local.contiguous(), parts, dst=0, group=group)
        return torch.cat(parts) if rank == 0 else None
    raise ValueError(f"unknown gather mode {gather!r}")


class ShardGather:
    """Batch-sharded solve with the output gather to rank `dst` overlapped with compute (BASELINE c3:
    2048 images of 256x256 sharded over the GPUs of a node, "RCCL gather").

    Every `step()` solves this rank's shard y_local (in `chunks` slices, `solve(y_slice, out_slice)`)
    into one of two output buffers and gathers each slice to rank `dst` as soon as it is solved.  On a
    ROCm device with backend "nccl" (RCCL over xGMI) the gathers run on their own stream: slice c's
    gather waits only for slice c's solve, and the next step's solve (into the other buffer) does not
    wait for this step's gathers -- it waits only for the gathers that read the buffer it is about to
    overwrite (two steps back).  So the xGMI transfer of one batch overlaps the solve of the next.
    With "gloo" (CPU collectives: the multi-process tests) the same schedule runs synchronously,
    CUDA slices going through host copies.

    `gathered()` returns rank dst's (world * B_local, ...) result of the last step (None elsewhere).  It is
    a collective (every rank calls it): it makes the device work of every rank complete and, for "ipc",
    runs a barrier, so the peer writes into rank dst's buffer have landed.  The receive side is double
    buffered by step parity: the returned tensor stays valid until two more steps have been issued -- on
    EVERY rank.  step() itself does not synchronise the ranks, so with engine "ipc" a peer that runs two
    steps ahead of rank dst would overwrite the buffer rank dst is still reading.  So with "ipc" step() raises
    unless gathered() was called (collectively) after the previous step; a caller that only streams steps and
    never reads the buffers in between (the benchmark) passes stream_only=True.

    engine="ipc" moves the outputs without any collective kernel: rank dst shares its receive buffer
    once through a HIP IPC handle (admm_ipc_get_handle), every other rank maps it on its own device
    (admm_ipc_open) and copies each solved slice into its part of it with an async device copy on the
    second stream.  The HIP runtime hands peer copies of >= ROC_P2P_SDMA_SIZE
    to the SDMA engines, so no CU is held while the bytes cross xGMI.  An RCCL gather keeps kernel blocks
    resident for the whole transfer, and the fused solve needs every CU: one such block costs it
    ~0.8 ms per 1.2 ms (tools/contend.py).  With ipc a receive buffer is complete once
    every rank has finished its copies (what `gathered()` waits for).  If any rank cannot open the
    handles, every rank falls back to engine "rccl" (`self.engine` says which ran)."""

    def __init__(self, y_local, solve, *, chunks=1, group=None, dst=0, engine="rccl", stream_only=False):
        self.y = y_local
        self.stream_only = bool(stream_only)
        self.consumed = -1    # last step whose gathered() was called
        self.solve = solve
        self.group = group
        self.dst = dst
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        n = y_local.shape[0]
        chunks = max(1, min(int(chunks), n))
        self.bounds = [shard_range(n, chunks, c) for c in range(chunks)]
        self.out = [torch.empty_like(y_local) for _ in range(2)]
        self.cuda = y_local.is_cuda
        self.gloo = self.world > 1 and dist.get_backend(group) == "gloo"
        self.engine = "rccl"
        if engine == "ipc" and self.cuda and self.world > 1:
            self.engine = "ipc" if self._ipc_setup(y_local) else "rccl"
        self.async_comm = self.cuda and self.world > 1 and (not self.gloo or self.engine == "ipc")
        if self.engine == "ipc":
            pass   # self.recv (rank dst) / self.remote (others): two buffers each, set by _ipc_setup
        elif self.world > 1 and self.rank == dst:
            full = (self.world * n,) + tuple(y_local.shape[1:])
            dev = "cpu" if self.gloo else y_local.device
            self.recv = [torch.empty(full, dtype=y_local.dtype, device=dev) for _ in range(2)]
        else:
            self.recv = None
        if self.async_comm:
            self.comm = getattr(self, "comm", None) or torch.cuda.Stream(device=y_local.device)
            self.freed = [None, None]      # event: the gathers reading out[b] have completed
        self.i = 0

    def _ipc_setup(self, y_local):
        """Rank dst allocates the receive buffers and shares their IPC handles; the others map them through the
        library (admm_ipc_open on their OWN device: no context, stream or queue on rank dst's GPU).  Returns
        whether every rank succeeded (a collective: all ranks agree)."""
        n = y_local.shape[0]
        full = (self.world * n,) + tuple(y_local.shape[1:])
        nbytes = y_local.element_size() * self.world * y_local.numel()
        self.row_bytes = y_local.element_size() * (y_local.numel() // max(n, 1))
        ok = 1
        self.recv, self.remote, self._mapped = None, None, []
        obj = [None]
        try:
            if self.rank == self.dst:
                self.recv = [torch.empty(full, dtype=y_local.dtype, device=y_local.device) for _ in range(2)]
                obj = [[(*_lib.ipc_get_handle(r.data_ptr()), nbytes) for r in self.recv]]
        except Exception:   # noqa: BLE001 -- any failure selects the RCCL path on every rank
            ok = 0
        dist.broadcast_object_list(obj, src=self.dst, group=self.group)
        try:
            if self.rank != self.dst:
                if obj[0] is None:
                    raise RuntimeError("no handle")
                self.remote = []
                for handle, off, size in obj[0]:
                    if size != nbytes:
                        raise RuntimeError("receive buffer size mismatch")
                    base = _lib.ipc_open(handle, y_local.device.index)
                    self._mapped.append(base)
                    self.remote.append(base + off)
                # one real copy through the path the steps use (peer access, engine choice): any error
                # here selects RCCL instead of failing mid-run; the slice is overwritten by the first step
                self.comm = torch.cuda.Stream(device=y_local.device)
                for r in self.remote:
                    self._push(r, y_local, 0, 1)
                torch.cuda.synchronize(y_local.device)
        except Exception:   # noqa: BLE001
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device="cpu" if self.gloo else y_local.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        if int(flag.item()) == 1:
            return True
        self.close()
        self.closed = False   # only the peer mappings are gone: the RCCL path takes over
        self.recv, self.remote = None, None
        return False

    def close(self):
        """Unmap the peer receive buffers this rank opened (engine "ipc"); the object is unusable afterwards.
        The copies into the peer's mapping run asynchronously on the comm stream (stream_only steps never wait
        for them), so the stream is drained before the mapping goes away; later steps raise."""
        mapped = getattr(self, "_mapped", [])
        if mapped and getattr(self, "comm", None) is not None:
            try:
                self.comm.synchronize()
            except Exception:   # noqa: BLE001 -- a failed device: unmapping below is all that is left
                pass
        for base in mapped:
            try:
                _lib.ipc_close(base, self.y.device.index)
            except Exception:   # noqa: BLE001 -- best effort at teardown
                pass
        self._mapped = []
        self.remote = None
        self.closed = True

    def __del__(self):
        if getattr(self, "_mapped", None):
            self.close()

    def _out(self, b):
        """Output buffer b of this rank.  With ipc, rank dst solves straight into its own part of the
        receive buffer (nothing reads it during the steps), so it copies nothing."""
        if self.engine == "ipc" and self.rank == self.dst:
            n = self.y.shape[0]
            return self.recv[b][self.rank * n: (self.rank + 1) * n]
        return self.out[b]

    def _parts(self, c, b):
        """rank dst's receive views (buffer b) for chunk c of every rank (rank r's chunk lands at r * n + start)."""
        if self.recv is None:
            return None
        n = self.y.shape[0]
        s, k = self.bounds[c]
        return [self.recv[b][r * n + s: r * n + s + k] for r in range(self.world)]

    def _push(self, remote, out, s, k):
        """Copy this rank's solved slice [s, s + k) into its part of rank dst's IPC-mapped receive buffer (base
        address `remote`), on the comm stream.  An explicit hipMemcpyAsync through the library (admm_copy_async),
        not Tensor.copy_: a cross-device copy_ also synchronises with the current stream of the PEER device, which
        would make this process create and use a queue on rank dst's GPU.  The runtime gives device-to-device
        copies between GPUs of >= ROC_P2P_SDMA_SIZE (1 MiB default; a c3 slice is 64 MiB / chunks) to an SDMA
        engine."""
        n = self.y.shape[0]
        src = out[s:s + k]
        assert src.is_contiguous()
        src.record_stream(self.comm)
        _lib.copy_async(remote + (self.rank * n + s) * self.row_bytes, src.data_ptr(), k * self.row_bytes,
                        self.comm.cuda_stream)

    def step(self):
        if getattr(self, "closed", False):
            raise RuntimeError("ShardGather: step() after close()")
        if (self.engine == "ipc" and self.world > 1 and not self.stream_only and self.i >= 1
                and self.consumed != self.i - 1):
            raise RuntimeError("ShardGather(engine='ipc'): call gathered() (on every rank) after each step before the "
                               "next one -- a peer running ahead would overwrite the receive buffer rank dst is "
                               "reading; pass stream_only=True if nothing reads the gathered batches between steps")
        b = self.i & 1
        out = self._out(b)
        if self.async_comm and self.freed[b] is not None:
            torch.cuda.current_stream(self.y.device).wait_event(self.freed[b])
        for c, (s, k) in enumerate(self.bounds):
            self.solve(self.y[s:s + k], out[s:s + k])
            if self.world == 1 or (self.engine == "ipc" and self.rank == self.dst):
                continue
            if self.async_comm:
                done = torch.cuda.Event()
                done.record(torch.cuda.current_stream(self.y.device))
                with torch.cuda.stream(self.comm):
                    self.comm.wait_event(done)
                    if self.engine == "ipc":
                        self._push(self.remote[b], out, s, k)
                    else:
                        dist.gather(out[s:s + k], self._parts(c, b), dst=self.dst, group=self.group)
            else:
                src = out[s:s + k].cpu() if (self.gloo and self.cuda) else out[s:s + k]
                dist.gather(src, self._parts(c, b), dst=self.dst, group=self.group)
        if self.async_comm:
            ev = torch.cuda.Event()
            ev.record(self.comm)
            self.freed[b] = ev
        self.i += 1

    def wait(self):
        """Make the caller's stream wait for every gather issued so far."""
        if self.async_comm:
            torch.cuda.current_stream(self.y.device).wait_stream(self.comm)

    def local(self):
        """This rank's solved shard from the last step."""
        return self._out((self.i - 1) & 1)

    def gathered(self):
        """Rank dst's gathered batch of the last step (None on other ranks).  Collective: call on every rank."""
        if self.world == 1:
            return self.local()
        self.wait()
        if self.cuda:
            torch.cuda.synchronize(self.y.device)
        if self.engine == "ipc":
            dist.barrier(group=self.group)   # every peer's copies into rank dst's buffer have completed
        self.consumed = self.i - 1
        return None if self.recv is None else self.recv[(self.i - 1) & 1]
