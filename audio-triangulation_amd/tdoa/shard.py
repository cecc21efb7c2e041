"""Frame sharding across GPUs (one process per GPU, torch.distributed).

Frames are independent: each rank owns its own frames -- a
fixed per-rank batch (weak scaling, configs 2, 3, 5) or a contiguous slice of
ceil(B / world) frames of one global batch (strong scaling, config 4's 1e6
frames over 8 GPUs) -- and localizes them on its own GPU.  There is no
data-path collective: RCCL carries only the timing barrier, the max-over-
ranks of the elapsed time and (results / counts) reductions.

bench.py's rank logic lives here so that the world-2 gloo test
(tests/test_distributed.py) runs the same functions the driver's N-GPU runs
execute: `init_distributed`, `frame_seed`, `rank_frames`, `timed`,
`max_over_ranks`, `sum_over_ranks`, `ranks_seen`.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist


@dataclass(frozen=True)
class RankInfo:
    rank: int
    world: int
    local_rank: int


def rank_info() -> RankInfo:
    """RANK / WORLD_SIZE / LOCAL_RANK of a torch.distributed.run launch (1 process otherwise)."""
    return RankInfo(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def _active() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def init_distributed(backend: str = "nccl") -> RankInfo:
    """Join the process group when launched with WORLD_SIZE > 1.  backend
    "nccl" (RCCL on ROCm) binds the group to this rank's GPU; "gloo" is the
    CPU rehearsal.  The rendezvous address defaults to 127.0.0.1."""
    ri = rank_info()
    if ri.world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", ri.local_rank))
        else:
            dist.init_process_group(backend)
    return ri


def finalize() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def ranks_seen() -> int:
    """World size of the live process group (1 when not distributed)."""
    return dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1


def frame_seed(base: int, rank: int, r: int = 0) -> int:
    """Seed of rank `rank`'s r-th synthetic batch: every rank and every
    rotating batch gets distinct frames."""
    return int(base) + 7919 * int(rank) + 104729 * int(r)


def shard_range(B: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [lo, hi) slice of B frames owned by `rank`."""
    per = -(-B // world) if world > 0 else B
    lo = min(B, rank * per)
    return lo, min(B, lo + per)


def rank_frames(batch: int, rank: int, world: int, scaling: str) -> int:
    """Frames this rank processes per step: `batch` per rank ("weak") or its
    shard_range slice of a global `batch` ("strong")."""
    if scaling == "weak":
        return int(batch)
    lo, hi = shard_range(int(batch), rank, world)
    return hi - lo


def barrier() -> None:
    if _active():
        dist.barrier()


def _coll_device(device):
    """Where a reduction's tensor lives: the rank's GPU under RCCL, the host
    under gloo (a CPU process group, also when the ranks hold GPUs)."""
    return None if dist.get_backend() == "gloo" else device


def max_over_ranks(x: float, device=None) -> float:
    """Max of a scalar over all ranks (the bench's whole-job time)."""
    if not _active():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(xs, device=None) -> list[float]:
    """Element-wise sum of a few scalars over all ranks (frame / trigger counts)."""
    xs = [float(x) for x in xs]
    if not _active():
        return xs
    t = torch.tensor(xs, dtype=torch.float64, device=_coll_device(device))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def timed(step, steps: int, warmup: int, sync=lambda: None, device=None,
          on_start=None, on_end=None, barrier_fn=None) -> dict:
    """The bench contract's timed region: `warmup` untimed calls of step(k),
    then EXACTLY `steps` calls bracketed by sync + barrier + sync on both
    sides; the job time is the max over ranks.  on_start runs before the opening
    sync, on_end right after the last step (e.g. HIP event records on the launch
    stream: the events bracket the K launches, the clock the K steps).

    The start is barrier-aligned (every rank leaves the opening barrier
    together); each rank's clock stops right after its OWN closing sync, before
    the closing barrier, so the barrier's RCCL round trip is not part of any
    rank's time.  max over ranks then still is the slowest rank's end: the
    whole-job time for frames that are independent (sample_compute.h:105-139).
    `barrier_fn` replaces the process-group barrier (tests inject a slow one)."""
    bar = barrier_fn or barrier
    for k in range(warmup):
        step(k)
    sync()
    bar()
    if on_start:  # an event record: enqueued before the clock starts
        on_start()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    if on_end:
        on_end()
    sync()
    wall = time.perf_counter() - t0  # this rank's own end
    bar()
    sync()
    return {"wall_s": wall, "wall_max_s": max_over_ranks(wall, device)}


def gather_results(local: dict, B: int) -> dict | None:
    """Concatenate every rank's per-frame numpy results in rank order on rank 0."""
    if not _active():
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
