"""World-size-2 gloo rehearsal of the multi-GPU path on CPU: each rank
localizes its contiguous frame shard (here with the oracle, as no GPU is
present) and rank 0 gathers; the gathered results must equal the
single-process run frame for frame.  Also checks the max-over-ranks timing
reduction bench.py uses."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, PKG, ROOT  # noqa: F401


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    for p in (PKG, os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        from tdoa import shard
        g = np.load(os.path.join(GOLDEN, "pipeline_cfg2.npz"))
        win = np.load(os.path.join(GOLDEN, "window_q15.npz"))["n1024"]
        frames, lut = g["frames"][:45], g["lut"]  # 45: ragged split 23 + 22
        res = shard.localize_sharded(frames, lambda f: O.localize_batch(f, 46, win, lut))
        t = shard.max_over_ranks(float(rank + 1))
        if rank == 0:
            full = O.localize_batch(frames, 46, win, lut)
            ok = all((res[k] == full[k]).all() for k in ("lags", "gate", "cell", "xy"))
            q.put((ok, t, shard.shard_range(45, 0, world), shard.shard_range(45, 1, world)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gloo_shards_match_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, t, r0, r1 = q.get(timeout=5)
    assert ok
    assert t == 2.0
    assert r0 == (0, 23) and r1 == (23, 45)


def test_shard_range_covers_everything_once():
    from tdoa.shard import shard_range
    for B in (0, 1, 7, 4096, 1_000_000):
        for world in (1, 2, 3, 8):
            cover = np.zeros(B, np.int32)
            for r in range(world):
                lo, hi = shard_range(B, r, world)
                cover[lo:hi] += 1
            assert (cover == 1).all()
