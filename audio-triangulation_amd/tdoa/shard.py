"""Frame sharding across GPUs (one process per GPU, torch.distributed).

Frames are independent: a global batch splits into contiguous
slices of ceil(B / world) frames, each rank localizes its slice on its own
GPU, and only the small per-frame results (lags, gate, cell, xy: <= 24 B per
frame) are gathered.  There is no data-path collective; RCCL carries only the
result gather and timing reductions.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def shard_range(B: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) slice of B frames owned by `rank`."""
    per = -(-B // world) if world > 0 else B
    lo = min(B, rank * per)
    return lo, min(B, lo + per)


def max_over_ranks(x: float, device=None) -> float:
    """Max of a scalar over all ranks (the bench's whole-job time)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_results(local: dict, B: int) -> dict | None:
    """Concatenate every rank's per-frame numpy results in rank order on rank 0."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return local
    world = dist.get_world_size()
    parts = [None] * world
    dist.all_gather_object(parts, local)
    if dist.get_rank() != 0:
        return None
    out = {k: np.concatenate([p[k] for p in parts], axis=0) for k in local}
    for k, v in out.items():
        assert v.shape[0] == B, f"gathered {k} has {v.shape[0]} != {B} frames"
    return out


def localize_sharded(frames: np.ndarray, compute, keys=("lags", "gate", "cell", "xy")) -> dict | None:
    """Run `compute(shard_frames) -> dict of per-frame arrays` on this rank's
    slice of `frames` and gather on rank 0 (None elsewhere)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    lo, hi = shard_range(frames.shape[0], rank, world)
    res = compute(frames[lo:hi])
    local = {k: np.asarray(res[k]) for k in keys}
    return gather_results(local, frames.shape[0])
