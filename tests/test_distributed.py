"""World-size-2 gloo rehearsal of the multi-GPU path on CPU.

bench.py's rank logic lives in tdoa/shard.py; the workers below run those
same functions -- init_distributed (from RANK / WORLD_SIZE / LOCAL_RANK),
frame_seed, rank_frames with bench.CONFIGS' scaling, the timed bracket
(barrier + max over ranks), sum_over_ranks and ranks_seen -- with the
oracle as the injected compute (no GPU here).  The gathered per-frame
results must equal the single-process run frame for frame."""
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
    for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    import oracle as O
    from tdoa import shard
    ri = shard.init_distributed("gloo")
    try:
        g = np.load(os.path.join(GOLDEN, "pipeline_cfg2.npz"))
        win = np.load(os.path.join(GOLDEN, "window_q15.npz"))["n1024"]
        frames, lut = g["frames"][:45], g["lut"]  # 45: ragged split 23 + 22
        res = shard.localize_sharded(frames, lambda f: O.localize_batch(f, 46, win, lut))
        # the bench's timed bracket with an injected CPU step: every rank's own
        # shard, the wall time max-reduced, the frame count sum-reduced
        lo, hi = shard.shard_range(45, ri.rank, ri.world)
        done = []
        t = shard.timed(lambda k: done.append(O.localize_batch(frames[lo:hi], 46, win, lut)),
                        steps=3, warmup=1)
        # the closing barrier is outside every rank's clock: a barrier that
        # sleeps 50 ms on its second (closing) call must not show in wall_max_s
        calls = []

        def slow_barrier():
            calls.append(1)
            if len(calls) == 2:
                import time
                time.sleep(0.05)
            shard.barrier()

        ts = shard.timed(lambda k: None, steps=3, warmup=0, barrier_fn=slow_barrier)
        total = shard.sum_over_ranks([(hi - lo) * 3])[0]
        mx = shard.max_over_ranks(float(rank + 1))
        cfg4 = bench.CONFIGS[4]
        per4 = shard.rank_frames(cfg4["batch"], ri.rank, ri.world, cfg4["scaling"])
        per2 = shard.rank_frames(bench.CONFIGS[2]["batch"], ri.rank, ri.world,
                                 bench.CONFIGS[2]["scaling"])
        seeds = [shard.frame_seed(0x5EED0002, ri.rank, r) for r in range(3)]
        out = {"rank": rank, "ranks_seen": shard.ranks_seen(), "wall": t["wall_s"],
               "wall_max": t["wall_max_s"], "steps_done": len(done), "total": total, "max": mx,
               "per4": per4, "per2": per2, "seeds": seeds, "slow_wall_max": ts["wall_max_s"],
               "slow_calls": len(calls)}
        if rank == 0:
            full = O.localize_batch(frames, 46, win, lut)
            out["ok"] = all((res[k] == full[k]).all() for k in ("lags", "gate", "cell", "xy"))
        q.put(out)
        dist.barrier()
    finally:
        shard.finalize() if dist.is_initialized() else None


@pytest.mark.timeout(300)
def test_two_rank_gloo_bench_rank_logic():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    rs = sorted([q.get(timeout=5) for _ in range(2)], key=lambda r: r["rank"])
    assert rs[0]["ok"]
    assert all(r["ranks_seen"] == 2 for r in rs)
    assert all(r["steps_done"] == 3 + 1 for r in rs)           # warmup 1 + exactly 3 timed
    assert all(r["total"] == 45 * 3 for r in rs)               # every frame counted once
    wall_max = max(r["wall"] for r in rs)
    assert all(abs(r["wall_max"] - wall_max) < 1e-12 for r in rs)
    assert all(r["max"] == 2.0 for r in rs)
    assert rs[0]["per4"] + rs[1]["per4"] == 1_000_000           # config 4: one global batch
    assert rs[0]["per2"] == rs[1]["per2"] == 4096               # config 2: per-GPU batch
    assert len(set(rs[0]["seeds"] + rs[1]["seeds"])) == 6       # distinct frames per rank/batch
    # the closing barrier (slept 50 ms) is not inside the timed window
    assert all(r["slow_calls"] == 2 for r in rs)
    assert all(r["slow_wall_max"] < 0.04 for r in rs), [r["slow_wall_max"] for r in rs]


def test_shard_range_covers_everything_once():
    from tdoa.shard import shard_range
    for B in (0, 1, 7, 4096, 1_000_000):
        for world in (1, 2, 3, 8):
            cover = np.zeros(B, np.int32)
            for r in range(world):
                lo, hi = shard_range(B, r, world)
                cover[lo:hi] += 1
            assert (cover == 1).all()


def test_single_process_defaults():
    from tdoa import shard
    os.environ.pop("WORLD_SIZE", None)
    ri = shard.init_distributed("gloo")
    assert (ri.rank, ri.world) == (0, 1) and shard.ranks_seen() == 1
    assert shard.max_over_ranks(3.5) == 3.5 and shard.sum_over_ranks([2, 3]) == [2.0, 3.0]
    assert shard.rank_frames(10, 0, 1, "strong") == 10


def _bench(*argv, env_extra=None, timeout=240):
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(300)
def test_bench_self_launches_two_ranks():
    """`python bench.py --gpus 2` (no torchrun around it) starts its two rank
    processes itself, before touching a GPU; here over gloo with the stand-in
    CPU step of --cpu-rehearsal.  One JSON line: both ranks joined, and the
    rank-0 cpu_baseline is attached at N > 1 too."""
    import json
    r = _bench("--gpus", "2", "--cpu-rehearsal", "--steps", "3", "--warmup", "1",
               "--cpu-seconds", "0.5")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["ranks_seen"] == 2 and d["rehearsal"] is True and d["steps"] == 3
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"


def test_bench_refuses_a_world_that_is_not_gpus():
    """A launch whose WORLD_SIZE differs from --gpus exits non-zero instead of
    timing the wrong number of GPUs."""
    r = _bench("--gpus", "2", "--cpu-rehearsal", env_extra={"WORLD_SIZE": "1"}, timeout=120)
    assert r.returncode == 3 and "--gpus 2" in r.stderr
