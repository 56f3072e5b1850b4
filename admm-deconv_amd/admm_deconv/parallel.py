"""Batch sharding across ranks (one process per GPU) and the output gather over RCCL.

The anisotropic solve is independent per (image, channel) plane (ops.jl:168-173), so a batch of B
images is split into contiguous per-rank ranges by GLOBAL image index (synthetic inputs are seeded
by global index, so a sharded run is bit-identical to the unsharded one) and solved with no
communication.  The only exchange is optional: gathering every rank's outputs to rank 0 (or to all
ranks) after the solve -- `torch.distributed` with backend "nccl" is RCCL over xGMI on MI355X;
with "gloo" the same code runs on CPU tensors for the multi-process tests.

The isotropic prox couples the whole batch (pixelnorm over dims 3,4, ops.jl:6), so it does NOT
shard this way; see DESIGN.md (it needs a per-iteration all-reduce of an M x N map).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

__all__ = ["shard_range", "solve_sharded"]


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
