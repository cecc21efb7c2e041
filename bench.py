#!/usr/bin/env python3
"""Headline benchmark: localizations/s on BASELINE config 2
(3-mic triangle, 1024-sample int16 frames, batch 4096 per GPU, cross-correlation
-> argmax -> lag prior -> (x, y) grid solve), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--engine gcc_phat|direct]
    torchrun --nproc-per-node N bench.py --gpus N ...     (driver, N > 1)

A step = one fused libtdoa launch over one batch of 4096 frames already
resident in HBM.  Batches rotate through > 256 MiB of frames so the Infinity
Cache cannot serve them.  Frames are independent: each rank owns its own
shard (weak scaling, no data-path collective; the only collectives are the
timing barrier and the max-over-ranks of the elapsed time).

Rank 0 prints one JSON line.  `roofline` prices the dominant kernel against
HBM with ALGORITHMIC bytes (M*N*2 in + 4P lags + 8 xy = 6164 B/loc),
`cpu_baseline` times the oracle (the reference's algorithm restated in C,
OpenMP over frames) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector peak

# BASELINE.json configs 2-4 (per-GPU batch; config 4's 1e6 frames are 125000 per GPU at 8)
CONFIGS = {
    2: dict(desc="BASELINE config 2: 3-mic triangle, 1024-sample frames", M=3, N=1024,
            mics=None, batch=4096),
    3: dict(desc="BASELINE config 3: 4-mic square (0.15 m), 4096-sample frames, 6 pairs",
            M=4, N=4096, mics="square", batch=65536),
    4: dict(desc="BASELINE config 4: 8-mic circle (r 0.15 m), 2048-sample frames, 28 pairs",
            M=8, N=2048, mics="circle", batch=125000),
    # batch = streams per GPU; one step = one 512-sample hop of every stream
    5: dict(desc="BASELINE config 5: streaming 48 kHz, 512-sample hop, 3-mic triangle, "
                 "trigger + DIRECT xcorr + EMA + grid, one hipGraph per hop",
            M=3, N=1024, mics=None, batch=16384, fs=48000, hop=512),
}


def phat_flops(M, N):
    """SURVEY.md 8(d) GCC-PHAT flop model per localization, L = 2N."""
    import math
    L, P = 2 * N, M * (M - 1) // 2
    return M * 2.5 * L * math.log2(L) + P * 10 * (L / 2 + 1) + P * 2.5 * L * math.log2(L)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="default 400 (config 2), 200 (config 5), 20 otherwise")
    ap.add_argument("--warmup", type=int, default=None,
                    help="default 20 (config 2, 5), 3 otherwise")
    ap.add_argument("--engine", default="gcc_phat", choices=["gcc_phat", "direct"])
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--rotate-mib", type=int, default=320,
                    help="frames rotated per rank (> 256 MiB Infinity Cache)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--also", action="store_true", help="also time the other engine")
    ap.add_argument("--no-grid", action="store_true", help="diagnostic: skip the grid solve")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "hbm_traffic.json"))
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    if a.batch is None:
        a.batch = cfg["batch"]
    if a.steps is None:
        a.steps = {2: 400, 5: 200}.get(a.config, 20)
    if a.warmup is None:
        a.warmup = 20 if a.config in (2, 5) else 3
    if a.config == 5:
        a.engine = "direct"  # the streaming loop runs the reference's DIRECT path
    return a


def config_mics(cfg):
    from tdoa import synth
    if cfg["mics"] == "square":
        return synth.square_mics(0.15)
    if cfg["mics"] == "circle":
        return synth.circle_mics(cfg["M"], 0.15)
    return None


def time_engine(engine, args, dev, rank, world, lut_cache):
    from tdoa import synth
    from tdoa.localizer import Localizer
    cfg = CONFIGS[args.config]
    loc = Localizer(engine=engine, num_mics=cfg["M"], frame_len=cfg["N"], mic_xy=config_mics(cfg),
                    device=dev.index)
    M, N, P = loc.dims.M, loc.dims.N, loc.dims.P
    B = args.batch
    lut = loc.lut().reshape(P, 101, 101)
    lut_cache["lut"], lut_cache["window"] = lut, loc.window()
    per_batch = B * M * N * 2
    R = max(1, -(-args.rotate_mib * (1 << 20) // per_batch))
    batches = []
    for r in range(R):
        fr, _, _ = synth.adc_frames(B, M, N, lut, loc.dims.S,
                                    synth.SEEDS[args.config] + 7919 * rank + 104729 * r,
                                    device=dev)
        batches.append(fr)
    out = loc.alloc_outputs(B, grid=not args.no_grid)
    stream = torch.cuda.current_stream(dev)
    for k in range(args.warmup):
        loc.localize_into(batches[k % R], out, stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        loc.localize_into(batches[k % R], out, stream)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ev_ms = ev0.elapsed_time(ev1)  # GPU time of the K launches on the launch stream
    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())
    total = world * B * args.steps
    bytes_per_loc = M * N * 2 + 4 * P + 8
    kern_s = ev_ms / 1e3 / args.steps
    res = {
        "engine": engine,
        "value": total / wall_max,
        "ms_per_step": wall_max * 1e3 / args.steps,
        "kernel_ms": kern_s * 1e3,
        "bytes_per_loc": bytes_per_loc,
        "achieved_gbs": bytes_per_loc * B / kern_s / 1e9,
        "valu_tflops": phat_flops(M, N) * B / kern_s / 1e12,
        "rotate_batches": R,
    }
    # sanity: outputs of the last step are finite / in range
    lags = out["lags"].cpu()
    assert int(lags.abs().max()) <= loc.dims.S
    loc.close()
    return res


def time_stream(args, dev, rank, world, cache):
    """Config 5: S streams per GPU, capture ring resident in HBM (64 hops per
    stream, replayed cyclically); a step = one hop of every stream."""
    from tdoa import synth
    from tdoa.localizer import Localizer
    from tdoa.stream import StreamPipeline
    cfg = CONFIGS[5]
    loc = Localizer(sample_rate_hz=cfg["fs"], device=dev.index)
    S, H = args.batch, cfg["hop"]
    lut = loc.lut()
    cache["lut"], cache["window"], cache["S"] = lut, loc.window(), loc.dims.S
    T = 64 * H
    cap = synth.adc_stream(S, T, 3, lut, loc.dims.S, synth.SEEDS[5] + 7919 * rank, device=dev)
    torch.cuda.synchronize(dev)
    pipe = StreamPipeline(loc, cap, hop=H, use_graph=True)
    st = pipe.stream
    for _ in range(args.warmup):
        pipe.step()
    st.synchronize()
    _, trig0, gated0 = pipe.totals()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(st)
    for _ in range(args.steps):
        pipe.step()
    ev1.record(st)
    st.synchronize()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    _, trig1, gated1 = pipe.totals()
    t = torch.tensor([wall, trig1 - trig0, gated1 - gated0], dtype=torch.float64, device=dev)
    if world > 1:
        mx = t[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t[0] = mx[0]
    wall_max, trig, gated = float(t[0]), float(t[1]), float(t[2])
    samples = world * S * H * args.steps
    pipe.close()
    return {"engine": "direct", "value": trig / wall_max, "ms_per_step": wall_max * 1e3 / args.steps,
            "kernel_ms": gpu_s * 1e3 / args.steps, "triggered": trig, "gated": gated,
            "stream_samples_per_s": samples / wall_max,
            "realtime_streams": samples / wall_max / cfg["fs"],
            "capture_bytes_per_step": world * S * H * 3}


def cpu_baseline_stream(args, lut, window, S_lag):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from tdoa import synth
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    adc = synth.adc_stream(64, 64 * 512, 3, lut, S_lag, synth.SEEDS[5]).numpy()
    O.stream_run(adc[:4, :4096], 1024, 48000, S_lag, window, lut, threads=threads)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        r = O.stream_run(adc, 1024, 48000, S_lag, window, lut, threads=threads, max_trig=64)
        n += int(r["n_trig"].sum())
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "localizations/s", "cores": threads, "kind": "port",
            "sample": f"{n} triggered frames from 64 streams x 32768 samples (config-5 capture "
                      f"bytes) in {dt:.1f} s, oracle orc_stream_run (sample_compute.h:53-146 "
                      f"sample by sample: rings, trigger, DIRECT xcorr, EMA, grid), OpenMP "
                      f"{threads} threads over streams"}


def cpu_baseline(args, lut, window):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from tdoa import synth
    cfg = CONFIGS[args.config]
    M, N = cfg["M"], cfg["N"]
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    nfr = 2048 if args.config == 2 else 128
    fr, _, _ = synth.adc_frames(nfr, M, N, lut, 46, synth.SEEDS[args.config])
    fr = fr.numpy()
    O.localize_batch(fr[:16], 46, window, lut, threads=threads, want_scores=False)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        O.localize_batch(fr, 46, window, lut, threads=threads, want_scores=False)
        n += fr.shape[0]
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "localizations/s", "cores": threads, "kind": "port",
            "sample": f"{n} config-{args.config} frames ({M}x{N} ADC-like, batches of {nfr}) "
                      f"in {dt:.1f} s, "
                      f"oracle/tdoa_oracle.c (reference correlations.c + vga_heatmap.h "
                      f"algorithm, DIRECT integer xcorr), OpenMP {threads} threads"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    cache = {}
    if args.config == 5:
        return main_stream(args, dev, rank, world, cache)
    main_res = time_engine(args.engine, args, dev, rank, world, cache)
    other = None
    if args.also:
        other = time_engine("direct" if args.engine == "gcc_phat" else "gcc_phat", args, dev,
                            rank, world, cache)
    if rank == 0:
        traffic = None
        if args.config == 2 and os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                traffic = tj.get(args.engine, {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        cfg = CONFIGS[args.config]
        shape = f"{cfg['M']}-mic x {cfg['N']}-sample frames"
        line = {
            "metric": f"GCC-PHAT localizations/sec, {shape}"
            if args.engine == "gcc_phat" else
            f"localizations/sec (DIRECT exact xcorr), {shape}",
            "value": main_res["value"],
            "unit": "localizations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": main_res["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if args.engine == "gcc_phat" else "int16->int64",
            "data": "synthetic (ADC-like u8 frames, injected integer delays, resident in HBM, "
                    f"{main_res['rotate_batches']} rotating batches > 256 MiB)",
            "config": {"workload": f"{cfg['desc']}, batch {args.batch} per GPU, "
                                   "xcorr + lag prior + (x,y) grid",
                       "engine": args.engine, "batch_per_gpu": args.batch, "mics": cfg["M"],
                       "frame_len": cfg["N"],
                       "parallelism": f"dp{world} (frame shards, no collective)"},
            "roofline": {"bound": "hbm", "achieved": main_res["achieved_gbs"],
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": main_res["achieved_gbs"] / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "kernel_ms": main_res["kernel_ms"],
                         "bytes_per_loc": main_res["bytes_per_loc"]},
            # the bound that actually binds an fp32 FFT path: FP32 vector issue
            "valu_roofline": {"achieved": main_res["valu_tflops"], "peak": VALU_PEAK_TFLOPS,
                              "unit": "TFLOP/s", "frac": main_res["valu_tflops"] / VALU_PEAK_TFLOPS,
                              "flop_model": "SURVEY.md 8(d) GCC-PHAT model"}
            if args.engine == "gcc_phat" else None,
            "cpu_baseline": None,
        }
        if other is not None:
            line["other_engine"] = other
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(args, cache["lut"], cache["window"])
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main_stream(args, dev, rank, world, cache):
    res = time_stream(args, dev, rank, world, cache)
    if rank == 0:
        cfg = CONFIGS[5]
        line = {
            "metric": "streaming localizations/sec (triggered frames), 3-mic x 1024-sample "
                      "frames, 48 kHz, 512-sample hop",
            "value": res["value"], "unit": "localizations/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "int16->int64",
            "data": "synthetic u8 capture bytes (bursts from a fixed source per stream over a "
                    "quiet floor), 64-hop capture ring per stream resident in HBM",
            "config": {"workload": f"{cfg['desc']}, {args.batch} streams per GPU",
                       "streams_per_gpu": args.batch, "hop": cfg["hop"], "fs": cfg["fs"],
                       "mics": 3, "frame_len": 1024,
                       "parallelism": f"dp{world} (stream shards, no collective)"},
            "stream": {k: res[k] for k in ("kernel_ms", "triggered", "gated",
                                           "stream_samples_per_s", "realtime_streams")},
            "roofline": None,
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline_stream(args, cache["lut"], cache["window"],
                                                       cache["S"])
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
