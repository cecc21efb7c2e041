"""bench.py's N-rank path on a real GPU box: `--gpus 2` self-launches two rank
processes (torch.distributed.run), here over gloo with both ranks on cuda:0
(`--dist-backend gloo --rank-device 0`), so the per-rank GPU data generation,
the prepared launches, the timed bracket, the max / sum reductions and the
rank-0 JSON line run on hardware with ranks_seen 2.  This exercises the code;
it is not a 2-GPU measurement (the driver's SCALE runs are)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("config", [2, 5])
def test_bench_two_ranks_on_one_gpu(config):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    argv = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
            "--rank-device", "0", "--config", str(config), "--steps", "5", "--warmup", "2",
            "--cpu-seconds", "0.5", "--no-parity"]
    if config == 2:
        argv += ["--rotate-mib", "16", "--preflight-s", "0"]
    else:
        argv += ["--batch", "1024"]
    r = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["ranks_seen"] == 2 and d["n_gpus"] == 2
    assert d["value"] > 0 and d["steps"] == 5
    assert d["config"]["parallelism"].startswith("dp2")
    cb = d["cpu_baseline"]
    assert cb is not None and cb["value"] > 0 and cb["cores"] >= 1
