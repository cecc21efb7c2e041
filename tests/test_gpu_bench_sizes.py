"""The benchmarked batch sizes of configs 3, 4 and 5, under test.

test_gpu_bench_path.py checks the bench's output path bit for bit at a few
thousand frames; bench.py times 65,536 (config 3), 1,000,000 (config 4, with
the least-squares refinement) and 16,384 streams (config 5).  At those sizes
the launches take other code paths the small batches never reach: several
persistent frame loops per workgroup in k_frame16, a 7.3 GB compact score
scratch and k_grid_bb grids of 1e6 workgroups at config 4, 16,384-stream
trigger lists and DIRECT batches of thousands of triggered frames at config 5.
So, with the bench's own generator (bench.make_frames, the same seeds):

  configs 3 / 4  the full-batch bench launch (no scores, as timed) writes lags
                 in range, and a strided sample of 4,096 of its frames equals
                 a separate small-batch launch of the same frames bit for bit
                 (lags, gate, cell, xy, max_Lf, xy_ls, ls_rms), whose cells and
                 max_Lf equal the exhaustive float32 scan of a scores run
                 (vga_heatmap.h:99-108 on the engine's own weighted scores);
  config 5       16,384 streams over 10 hops through the hipGraph pipeline;
                 64 sampled streams' records (end, lags, gate, EMA argmax,
                 cell, max_L) and EMA state equal the oracle's sample-by-sample
                 restatement of sample_compute.h:53-146 on those streams.

Reference: sample_compute.h:105-139 (the per-frame path), vga_heatmap.h:99-108.
"""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402  (the bench's generator and configs)
from tdoa import shard, synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402
from tdoa.stream import StreamPipeline  # noqa: E402
from test_gpu_gcc_phat import _grid_f32, _np  # noqa: E402
from test_gpu_stream import compare  # noqa: E402

SAMPLE = 4096
OUT_KEYS = ("lags", "gate", "cell", "xy", "max_Lf", "xy_ls", "ls_rms")


def _bench_batch(config):
    cfg = bench.CONFIGS[config]
    loc = Localizer(engine="gcc_phat", num_mics=cfg["M"], frame_len=cfg["N"], mic_xy=bench.config_mics(cfg))
    P, S = loc.dims.P, loc.dims.S
    B = cfg["batch"]
    fr, _ = bench.make_frames(B, cfg["M"], cfg["N"], loc.lut().reshape(P, -1), S,
                              shard.frame_seed(0x5EED0000 + config, 0, 0), torch.device("cuda", 0))
    return loc, fr


@pytest.mark.timeout(600)
@pytest.mark.parametrize("config", [3, 4])
def test_bench_size_long_frames(config):
    loc, fr = _bench_batch(config)
    B, S = fr.shape[0], loc.dims.S
    ls = config == 4
    assert B == bench.CONFIGS[config]["batch"]
    out = loc.alloc_outputs(B, ls=ls)
    loc.localize_into(fr, out)
    torch.cuda.synchronize()
    lags = out["lags"]
    assert int(lags.abs().max()) <= S
    assert loc.batch_kernel() == "k_frame16"
    # a strided sample, from the first frame to the last, across every
    # workgroup's frame loop
    idx = torch.linspace(0, B - 1, SAMPLE, device="cuda").round().long().unique()
    assert idx.numel() == SAMPLE
    big = {k: v[idx].cpu().numpy() for k, v in out.items() if k in OUT_KEYS}
    del out
    sub = fr[idx].contiguous()
    del fr
    torch.cuda.empty_cache()
    o2 = loc.alloc_outputs(SAMPLE, ls=ls)
    loc.localize_into(sub, o2)
    torch.cuda.synchronize()
    small = _np(o2)
    for k in OUT_KEYS:
        if k in big:
            assert np.array_equal(big[k], small[k], equal_nan=True), (config, k)
    # the sample's cells: the exhaustive f32 scan of its own weighted scores
    checked = _np(loc.localize(sub, scores=True, ls=ls))
    for k in OUT_KEYS:
        if k in big:
            assert np.array_equal(big[k], checked[k], equal_nan=True), (config, k, "scores path")
    cell, mx = _grid_f32(checked["weighted_f"], loc.lut())
    assert np.array_equal(big["cell"], cell), config
    assert np.array_equal(big["max_Lf"], mx), config
    if ls:
        assert np.isfinite(big["xy_ls"]).all()
    loc.close()


@pytest.mark.timeout(600)
def test_bench_size_stream(oracle):
    cfg = bench.CONFIGS[5]
    S, H, hops = cfg["batch"], cfg["hop"], 10
    loc = Localizer(sample_rate_hz=cfg["fs"])
    lut = loc.lut()
    cap = synth.adc_stream(S, hops * H, 3, lut, loc.dims.S, shard.frame_seed(synth.SEEDS[5], 0),
                           device=torch.device("cuda", 0))
    torch.cuda.synchronize()
    pick = np.linspace(0, S - 1, 64).round().astype(np.int64)
    pipe = StreamPipeline(loc, cap, hop=H)  # bench.py's launch form
    recs = {int(s): [] for s in pick}
    total = 0
    for _ in range(hops):
        pipe.step()
        r = pipe.records()
        total += len(r["stream_id"])
        assert (np.abs(r["lags"]) <= loc.dims.S).all()
        for i, s in enumerate(r["stream_id"]):
            if int(s) in recs:
                recs[int(s)].append({k: v[i] for k, v in r.items()})
    pos, est, last = pipe.state()
    assert pos == hops * H
    _, trig, _ = pipe.totals()
    assert trig == total and total > S // 10, (trig, total)
    pipe.close()
    adc = cap[torch.from_numpy(pick).cuda()].cpu().numpy()
    exp = oracle.stream_run(adc, 1024, cfg["fs"], loc.dims.S, loc.window(), lut, max_trig=64)
    assert exp["n_trig"].sum() > 32
    remap = {int(s): i for i, s in enumerate(pick)}
    compare({remap[s]: v for s, v in recs.items()}, est[pick], last[pick], exp, loc.dims.P)
    loc.close()
