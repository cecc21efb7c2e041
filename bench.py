#!/usr/bin/env python3
"""Headline benchmark: localizations/s on BASELINE config 2
(3-mic triangle, 1024-sample int16 frames, batch 4096 per GPU, GCC-PHAT
cross-correlation -> argmax -> lag prior -> (x, y) grid solve), one process
per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--engine gcc_phat|direct]
                    [--config 2|3|4|5]
    torchrun --nproc-per-node N bench.py --gpus N ...     (driver, N > 1)

A step = one libtdoa launch over one batch of frames already resident in HBM
(config 5: one 512-sample hop of every stream).  Batches rotate through
> 256 MiB of frames so the Infinity Cache cannot serve them.  Frames are
independent: each rank owns its own frames (weak scaling for configs 2, 3, 5;
config 4 splits one global batch of 1e6 frames, strong scaling) and there is
no data-path collective -- the rank logic (seeds, shard sizes, the timed
bracket with barrier + max-over-ranks) is tdoa/shard.py, which
tests/test_distributed.py runs with gloo.

Rank 0 prints one JSON line.  `roofline` prices the launch against HBM with
ALGORITHMIC bytes (M*N*2 in + 4P lags + 8 xy per localization; 6164 B at
config 2) over the launch's average duration from HIP events on the launch
stream; `parity` reports, on the bench's own first batch, how often the
GCC-PHAT lags / cells equal the DIRECT engine's (the reference's integer
semantics) and the injected delays; `cpu_baseline` times the oracle (the
reference's algorithm restated in C, OpenMP over frames) on a bounded sample
of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tdoa import shard  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CALIB_JSON = os.path.join(ROOT, "profiles", "r05_hbm_calibration.json")


def achievable_hbm():
    """Measured achievable HBM read rate (tools/hbm_copy.hip under rocprofv3,
    profiles/r05_hbm_calibration.json): the denominator of frac_achievable; and the
    faster of its two copies (nontemporal / default-policy stores), read + write."""
    try:
        c = json.load(open(CALIB_JSON))
        cp = max(float(c.get("copy_gbs_rocprof", 0)), float(c.get("copy_plain_gbs_rocprof", 0)))
        return float(c["read_gbs_rocprof"]), cp
    except (OSError, ValueError, KeyError):
        return None, None


VALU_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector peak

# BASELINE.json configs 1-5.  batch: per GPU (weak) or global (strong).
CONFIGS = {
    # config 1: the reference's per-frame plumbing, 2 mics, through the
    # reference-named entry points (one GPU-backed call per stage and buffer)
    1: dict(desc="BASELINE config 1: 2-mic, 1024-sample frames, time-domain cross-correlation through the "
                 "reference-named per-frame entry points (sample_compute.h:105-122 for one pair)",
            M=2, N=1024, mics="two", batch=1, scaling="weak"),
    2: dict(desc="BASELINE config 2: 3-mic triangle, 1024-sample frames", M=3, N=1024,
            mics=None, batch=4096, scaling="weak"),
    3: dict(desc="BASELINE config 3: 4-mic square (0.15 m), 4096-sample frames, 6 pairs",
            M=4, N=4096, mics="square", batch=65536, scaling="weak"),
    4: dict(desc="BASELINE config 4: 8-mic circle (r 0.15 m), 2048-sample frames, 28 pairs, "
                 "global batch 1e6 split over the GPUs",
            M=8, N=2048, mics="circle", batch=1_000_000, scaling="strong"),
    # batch = streams per GPU; one step = one 512-sample hop of every stream
    5: dict(desc="BASELINE config 5: streaming 48 kHz, 512-sample hop, 3-mic triangle, "
                 "trigger + DIRECT xcorr + EMA + grid, two stream launches per hop",
            M=3, N=1024, mics=None, batch=16384, fs=48000, hop=512, scaling="weak"),
}


def dominant_kernel(config: int, engine: str, first: str = "", fused: bool = True) -> str:
    """Name of the kernel(s) a launch runs (the ones `traffic` was measured on);
    `first` is the library's own answer (Localizer.batch_kernel), `fused` whether
    the grid is solved inside it (Localizer.batch_grid_fused)."""
    if config == 2:
        return first or ("k_p1k_lean" if engine == "gcc_phat" else "k_direct_mfma")
    if config in (3, 4) and engine == "gcc_phat":
        return "k_frame16" if fused else "k_frame16 + k_grid_bb"
    return ""


def gpu_clock_mhz(dev, stream):
    """The shader clock the box holds under VALU load, probed right after the
    timed region (tdoa_gpu_clock_mhz: every CU's waves run FMA chains for 2 ms
    and compare s_memtime with the 100 MHz s_memrealtime; median over waves).
    Boxes of the pool differ by several percent on the same build: this tells
    a slow box from a regression.  None if the probe fails."""
    import ctypes as C
    import tdoa
    mhz = C.c_double(0.0)
    rc = tdoa.load().tdoa_gpu_clock_mhz(int(dev.index), C.c_void_p(stream.cuda_stream), 2.0, C.byref(mhz))
    return round(mhz.value, 1) if rc == 0 else None


def settle(launches, R, dev, stream, max_s, join=None):
    """Untimed windows of launches (max(R, 8) each: every rotating batch) until two
    consecutive windows' mean launch time (HIP events on the launch stream) agree
    within 2 %, or max_s has passed.  Returns the windows' means (us) and whether
    they settled."""
    n = max(R, 8)
    means, t0 = [], time.perf_counter()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    while True:
        e0.record(stream)
        for k in range(n):
            launches[k % R]()
        if join:
            join()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        means.append(e0.elapsed_time(e1) * 1e3 / n)
        ok = len(means) >= 2 and abs(means[-1] - means[-2]) <= 0.02 * means[-2]
        if ok or time.perf_counter() - t0 > max_s:
            return {"windows": len(means), "launches_per_window": n, "settled": ok,
                    "last_window_us": [round(m, 2) for m in means[-3:]],
                    "first_window_us": round(means[0], 2)}


def phat_flops(M, N):
    """SURVEY.md 8(d) GCC-PHAT flop model per localization, L = 2N."""
    import math
    L, P = 2 * N, M * (M - 1) // 2
    return M * 2.5 * L * math.log2(L) + P * 10 * (L / 2 + 1) + P * 2.5 * L * math.log2(L)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="default 400 (config 2), 200 (config 5), 5 (config 4), 20 otherwise")
    ap.add_argument("--warmup", type=int, default=None,
                    help="default 20 (config 2, 5), 2 (config 4), 3 otherwise")
    ap.add_argument("--engine", default="gcc_phat", choices=["gcc_phat", "direct"])
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per GPU (weak) / in total (strong); default: the config's")
    ap.add_argument("--rotate-mib", type=int, default=320,
                    help="frames rotated per rank (> 256 MiB Infinity Cache)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--preflight-s", type=float, default=0.25,
                    help="untimed steps for this long before the W warmups (configs 2-4): clocks and "
                         "the rotating batches' translations settle, so a short K-step window "
                         "measures the steady state; 0 disables")
    ap.add_argument("--settle-max-s", type=float, default=8.0,
                    help="longest the preflight waits for a steady launch time (configs 2-4)")
    ap.add_argument("--stream-graph", action="store_true",
                    help="config 5: replay each hop as a hipGraph (default: plain stream launches, faster)")
    ap.add_argument("--streams", type=int, default=0,
                    help="configs 2-4: consecutive steps alternate over this many HIP streams, own outputs each "
                         "(0: 2 where a launch keeps no context scratch, else 1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="no GPU: rehearse the N-process launch, rank logic and JSON line over gloo "
                         "with a stand-in CPU step (tests/test_distributed.py); not a measurement")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend at N > 1 (nccl = RCCL; gloo: the N-rank code on one "
                         "GPU box, e.g. with --rank-device 0; never a measurement of N GPUs)")
    ap.add_argument("--rank-device", type=int, default=-1,
                    help="GPU of every rank (default: LOCAL_RANK, one GPU per rank)")
    ap.add_argument("--also", action="store_true", help="also time the other engine")
    ap.add_argument("--no-grid", action="store_true", help="diagnostic: skip the grid solve")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "hbm_traffic.json"))
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    if a.batch is None:
        a.batch = cfg["batch"]
    if a.steps is None:
        a.steps = {1: 200, 2: 400, 5: 200, 4: 5}.get(a.config, 20)
    if a.warmup is None:
        a.warmup = {1: 10, 2: 20, 5: 20, 4: 2}.get(a.config, 3)
    if a.config in (1, 5):
        a.engine = "direct"  # the reference's integer path (per frame / streaming)
    return a


def config_mics(cfg):
    from tdoa import synth
    if cfg["mics"] == "square":
        return synth.square_mics(0.15)
    if cfg["mics"] == "circle":
        return synth.circle_mics(cfg["M"], 0.15)
    if cfg["mics"] == "two":
        return np.array([[-0.066, 0.0], [0.066, 0.0]], np.float32)
    return None


def make_frames(B, M, N, lut, S, seed, dev, chunk=65536):
    """Synthetic ADC frames generated on the device in chunks (bounded temporaries)."""
    from tdoa import synth
    if B <= chunk:
        fr, _, tau = synth.adc_frames(B, M, N, lut, S, seed, device=dev)
        return fr, tau
    fr = torch.empty((B, M, N), dtype=torch.int16, device=dev)
    tau = torch.empty((B, M), dtype=torch.int64, device=dev)
    for i, lo in enumerate(range(0, B, chunk)):
        hi = min(B, lo + chunk)
        f, _, t = synth.adc_frames(hi - lo, M, N, lut, S, seed + 31 * i, device=dev)
        fr[lo:hi], tau[lo:hi] = f, t
    return fr, tau


def parity_report(engine, loc, frames, tau, out):
    """Agreement of this run's outputs on its first batch with the DIRECT
    engine (the reference's integer semantics, correlations.c:20-23) and with
    the injected integer delays.  Outside the timed region."""
    from tdoa.localizer import Localizer
    B = frames.shape[0]
    P = loc.dims.P
    got = {k: v.cpu().numpy() for k, v in out.items()}
    rep = {"frames": int(B), "sample": "the bench's first batch on rank 0 (first 65536 frames)"}
    # injected delays: pair (0, m) lag = tau_m (synth.adc_frames)
    t = tau.cpu().numpy()
    M = loc.dims.M
    rep["lags_equal_injected_pairs0m"] = float((got["lags"][:, :M - 1] == t[:, 1:]).mean())
    if engine == "gcc_phat":
        d = Localizer(engine="direct", num_mics=M, frame_len=loc.dims.N,
                      mic_xy=None if M == 3 else loc.mics(), device=loc.device)
        dref = {k: v.cpu().numpy() for k, v in d.localize(frames).items()}
        d.close()
        same = got["lags"] == dref["lags"]
        rep["lags_equal_direct"] = float(same.mean())
        rep["frames_all_lags_equal_direct"] = float(same.all(-1).mean())
        if "cell" in got:
            same_c = got["cell"] == dref["cell"]
            rep["cells_equal_direct"] = float(same_c.mean())
            # how far the disagreeing frames' (x, y) lie from DIRECT's, in metres
            d = np.hypot(*(got["xy"] - dref["xy"]).T)
            dd = d[~same_c]
            rep["xy_distance_to_direct_m"] = {
                "p50": float(np.percentile(dd, 50)) if dd.size else 0.0,
                "p99": float(np.percentile(dd, 99)) if dd.size else 0.0,
                "max": float(dd.max()) if dd.size else 0.0,
                "over": "frames whose cell differs from DIRECT's", "frames": int(dd.size)}
        rep["contract"] = ("lags equal DIRECT wherever the fp64 GCC-PHAT top-2 margin exceeds "
                           "2e-4; GCC-PHAT's cell is the grid maximum of its OWN PHAT scores, so "
                           "it agrees with DIRECT's (the reference semantics) at the rate "
                           "cells_equal_direct, each disagreement a near-tie of DIRECT's L "
                           "(gap <= 1 %) at most xy_distance_to_direct_m.max metres away "
                           "(bounds per shape in tests/test_gpu_gcc_phat.py); '(x,y) within 1e-5 "
                           "relative' holds for DIRECT (bit-exact with the oracle) and the LS "
                           "refinement (vs its double oracle), not for GCC-PHAT's cell")
    else:
        rep["contract"] = "DIRECT is bit-exact with the oracle (tests/test_gpu_parity.py)"
    rep["pairs"] = int(P)
    return rep


def time_engine(engine, args, dev, ri, cache):
    from tdoa.localizer import Localizer
    cfg = CONFIGS[args.config]
    loc = Localizer(engine=engine, num_mics=cfg["M"], frame_len=cfg["N"], mic_xy=config_mics(cfg),
                    device=dev.index)
    M, N, P = loc.dims.M, loc.dims.N, loc.dims.P
    B = shard.rank_frames(args.batch, ri.rank, ri.world, cfg["scaling"])
    lut = loc.lut().reshape(P, -1)
    cache["lut"], cache["window"] = lut, loc.window()
    per_batch = B * M * N * 2
    R = max(1, -(-args.rotate_mib * (1 << 20) // per_batch))
    batches, taus = [], []
    for r in range(R):
        fr, tau = make_frames(B, M, N, lut, loc.dims.S,
                              shard.frame_seed(0x5EED0000 + args.config, ri.rank, r), dev)
        batches.append(fr)
        taus.append(tau)
    # config 4 is "28 pairs + least-squares": the LS refinement runs in the timed region
    ls = args.config == 4 and not args.no_grid
    # consecutive steps alternate over Q HIP streams, each with its own output
    # buffers: independent batches, so the next batch's waves start on the CUs
    # the previous one has released instead of waiting for its slowest XCD
    # (config 2: 27.1 vs 29.7 us per 4096-frame step, same box).  Only where a
    # launch keeps no context scratch (the grid solved inside the transform
    # kernel, no least squares): configs 3 / 4's k_grid_bb reads a per-context
    # scratch that concurrent launches would share
    safe = loc.batch_grid_fused() and not ls
    Q = (2 if safe else 1) if args.streams <= 0 else (args.streams if safe else 1)
    outs = [loc.alloc_outputs(B, grid=not args.no_grid, ls=ls) for _ in range(Q)]
    out = outs[0]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(Q - 1)]
    stream = streams[0]
    # preflight (untimed, before the W warmups): every rotating batch once, then
    # until preflight_s has passed (bounded); reported in the line
    # each rotating batch's launch prebuilt (Localizer.prepare: the same
    # tdoa_localize_batch as localize_into, its argument checks and ctypes
    # structs made once), so the timed loop's host Python is one C call per step
    launches = [loc.prepare(batches[k % R], outs[k % Q], streams[k % Q]) for k in range(R * Q)]
    R = R * Q
    pre_n, pre_t0 = 0, time.perf_counter()
    while args.preflight_s > 0 and (pre_n < R or time.perf_counter() - pre_t0 < args.preflight_s) \
            and pre_n < 20000:
        launches[pre_n % R]()
        pre_n += 1
        if pre_n % 64 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    joins = [torch.cuda.Event() for _ in streams[1:]]

    def join():  # the launch stream after every step stream's launches
        for e, st in zip(joins, streams[1:]):
            e.record(st)
            stream.wait_event(e)

    steady = settle(launches, R, dev, stream, args.settle_max_s, join) if args.preflight_s > 0 else None
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)

    def start():  # every step stream after the event (the first steps of each)
        ev0.record(stream)
        for st in streams[1:]:
            st.wait_event(ev0)

    t = shard.timed(lambda k: launches[k % R](), args.steps,
                    args.warmup, sync=lambda: torch.cuda.synchronize(dev), device=dev,
                    on_start=start, on_end=lambda: (join(), ev1.record(stream)))
    kern_s = ev0.elapsed_time(ev1) / 1e3 / args.steps  # GPU time per launch, launch stream
    clock = gpu_clock_mhz(dev, stream)
    total = shard.sum_over_ranks([B * args.steps], device=dev)[0]
    # algorithmic bytes: frames in, lags + (x, y) out (+ xy_ls and its rms with LS)
    bytes_per_loc = M * N * 2 + 4 * P + 8 + (12 if ls else 0)
    res = {
        "engine": engine,
        "kernel": loc.batch_kernel(),
        "grid_fused": loc.batch_grid_fused(),
        "value": total / t["wall_max_s"],
        "ms_per_step": t["wall_max_s"] * 1e3 / args.steps,
        "kernel_ms": kern_s * 1e3,
        "frames_per_rank": B,
        "bytes_per_loc": bytes_per_loc,
        "achieved_gbs": bytes_per_loc * B / kern_s / 1e9,
        "valu_tflops": phat_flops(M, N) * B / kern_s / 1e12,
        "rotate_batches": R // Q,
        "streams": Q,
        "preflight_steps": pre_n,
        "steady": steady,
        "ls": ls,
        "gpu_clock_mhz": clock,
    }
    lags = out["lags"].cpu()
    assert int(lags.abs().max()) <= loc.dims.S
    if ri.rank == 0 and not args.no_parity:
        n = min(B, 65536)
        f0 = batches[0][:n].contiguous()
        res["parity"] = parity_report(engine, loc, f0, taus[0][:n], loc.localize(f0))
    loc.close()
    return res


def time_stream(args, dev, ri, cache):
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
    cap = synth.adc_stream(S, T, 3, lut, loc.dims.S, shard.frame_seed(synth.SEEDS[5], ri.rank),
                           device=dev)
    torch.cuda.synchronize(dev)
    pipe = StreamPipeline(loc, cap, hop=H, use_graph=args.stream_graph)
    st = pipe.stream
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    for _ in range(args.warmup):
        pipe.step()
    st.synchronize()
    _, trig0, gated0 = pipe.totals()
    t = shard.timed(lambda k: pipe.step(), args.steps, 0,
                    sync=lambda: (st.synchronize(), torch.cuda.synchronize(dev)), device=dev,
                    on_start=lambda: ev0.record(st), on_end=lambda: ev1.record(st))
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    clock = gpu_clock_mhz(dev, st)
    _, trig1, gated1 = pipe.totals()
    trig, gated = shard.sum_over_ranks([trig1 - trig0, gated1 - gated0], device=dev)
    # per-hop latency, outside the timed region: one hop in flight at a time,
    # submit -> the hop's device outputs complete (the hop's launches, then
    # a stream synchronise; no copy to the host), and the hop's GPU time from
    # events around it
    lat_host, lat_gpu = [], []
    e_a = torch.cuda.Event(enable_timing=True)
    e_b = torch.cuda.Event(enable_timing=True)
    for _ in range(min(200, max(50, args.steps))):
        t0 = time.perf_counter()
        e_a.record(st)
        pipe.step()
        e_b.record(st)
        st.synchronize()
        lat_host.append(time.perf_counter() - t0)
        lat_gpu.append(e_a.elapsed_time(e_b) / 1e3)
    samples = ri.world * S * H * args.steps
    pipe.close()
    pct = lambda a, q: float(np.percentile(np.asarray(a) * 1e3, q))  # noqa: E731
    return {"engine": "direct", "value": trig / t["wall_max_s"],
            "ms_per_step": t["wall_max_s"] * 1e3 / args.steps,
            "kernel_ms": gpu_s * 1e3 / args.steps, "triggered": trig, "gated": gated,
            "gpu_clock_mhz": clock, "launch": "hipGraph per hop" if args.stream_graph else "stream launches",
            "stream_samples_per_s": samples / t["wall_max_s"],
            "realtime_streams": samples / t["wall_max_s"] / cfg["fs"],
            "capture_bytes_per_step": ri.world * S * H * 3,
            "latency_ms": {"p50": pct(lat_host, 50), "p99": pct(lat_host, 99),
                           "gpu_p50": pct(lat_gpu, 50), "gpu_p99": pct(lat_gpu, 99),
                           "hops": len(lat_host),
                           "kind": "per hop, one hop in flight: submit -> the hop's device outputs "
                                   "complete (the hop's launches, kernels, stream synchronise; no copy to the "
                                   "host) (p50/p99), and the hop's GPU time from events (gpu_*); "
                                   "measured after the timed region"}}


def time_config1(args, dev, ri, path):
    """Config 1: one 2-mic frame per step through the reference-named entry
    points of tdoa_reference_abi.h -- rolling_buffer_write_out, buffer_normalize_range,
    buffer_window for both buffers, then correlations_init (sample_compute.h:105-122
    for one pair): seven per-frame calls on the reference structs.  path "host":
    libtdoa's own host-CPU implementation (tdoa_ref_set_device(-1),
    csrc/tdoa_host_path.cpp; BASELINE config 1 is "on host CPU, no GPU"); path
    "gpu": each call a synchronous GPU round trip.  Every frame's correlations
    and best shift are checked against the oracle after the timed region."""
    import ctypes as C
    import tdoa
    from tdoa import _lib, synth
    from tdoa.localizer import Localizer
    cfg = CONFIGS[1]
    L = tdoa.load()
    loc = Localizer(engine="direct", num_mics=2, frame_len=1024, mic_xy=config_mics(cfg),
                    device=dev.index)
    S = loc.dims.S
    win = loc.window()
    n = args.steps + args.warmup
    fr, _, _ = synth.adc_frames(n, 2, 1024, loc.lut(), S, shard.frame_seed(0x5EED0001, ri.rank))
    fr = fr.numpy()
    loc.close()
    # the two rolling buffers of each frame: full rings, head 0 (oldest first)
    rings = []
    for i in range(n):
        pair = []
        for m in range(2):
            rb = _lib.RollingBuffer()
            rb.head, rb.is_full = 0, True
            C.memmove(rb.buffer, np.ascontiguousarray(fr[i, m]).ctypes.data, 2048)
            pair.append(rb)
        rings.append(pair)
    outs = [_lib.Correlations() for _ in range(n)]
    ba, bb = _lib.Buffer(), _lib.Buffer()
    wo, nr, wi, ci = (L.rolling_buffer_write_out, L.buffer_normalize_range, L.buffer_window,
                      L.correlations_init)

    def step(i):
        ra, rb = rings[i]
        wo(C.byref(ra), C.byref(ba))
        wo(C.byref(rb), C.byref(bb))
        nr(C.byref(ba))
        nr(C.byref(bb))
        wi(C.byref(ba))
        wi(C.byref(bb))
        ci(C.byref(outs[i]), C.byref(ba), C.byref(bb))

    if L.tdoa_ref_set_device(-1 if path == "host" else int(dev.index)) != 0:
        raise RuntimeError("tdoa_ref_set_device failed")
    try:
        for i in range(args.warmup):
            step(i)
        sync = (lambda: None) if path == "host" else (lambda: torch.cuda.synchronize(dev))
        t = shard.timed(lambda k: step(args.warmup + k), args.steps, 0, sync=sync, device=dev)
    finally:
        L.tdoa_ref_set_device(int(dev.index))
    total = shard.sum_over_ranks([args.steps], device=dev)[0]
    # parity: the oracle's DC removal / normalise / window / xcorr / prior per frame
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    ok = 0
    for i in range(args.warmup, n):
        pre = [O.window(O.normalize(O.dc_remove(fr[i, m])[0]), win) for m in range(2)]
        sc, best = O.xcorr(pre[0], pre[1], S)
        got = np.frombuffer(bytes(outs[i].correlations), np.int64)
        ok += int(outs[i].best_shift == best and (got == O.prior(sc, best)).all())
    return {"value": total / t["wall_max_s"], "ms_per_step": t["wall_max_s"] * 1e3 / args.steps,
            "parity": {"frames": args.steps, "bit_exact_frames": ok,
                       "contract": "correlations (int64, after the lag prior) and best_shift equal "
                                   "the oracle's for every timed frame"},
            "S": S, "win": win, "frames": fr}


def cpu_baseline_config1(args, res):
    """The same per-frame sequence on one host core (the oracle's C port)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    fr, win, S = res["frames"], res["win"], res["S"]
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < min(args.cpu_seconds, 5.0):
        f = fr[n % fr.shape[0]]
        pre = [O.window(O.normalize(O.dc_remove(f[m])[0]), win) for m in range(2)]
        sc, best = O.xcorr(pre[0], pre[1], S)
        O.prior(sc, best)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "localizations/s", **_cpu_info(1),
            "threads_source": "one thread (the per-frame path is sequential)", "kind": "port",
            "sample": f"{n} 2-mic frames in {dt:.1f} s: oracle/tdoa_oracle.c dc_remove, normalize, "
                      "window, xcorr, prior per frame (rolling_buffer.c, buffer.c, correlations.c), "
                      "one thread, called from Python like the GPU path"}


def main_config1(args, dev, ri):
    res = time_config1(args, dev, ri, "host")
    gpu = time_config1(args, dev, ri, "gpu")
    world = shard.ranks_seen()
    if ri.rank == 0:
        cfg = CONFIGS[1]
        line = {
            "metric": "localizations/sec (2-mic DIRECT xcorr, reference per-frame entry points, host CPU)",
            "value": res["value"], "unit": "localizations/s", "n_gpus": world, "ranks_seen": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "int16->int64",
            "data": "synthetic (ADC-like u8 frames, injected integer delays) in host rolling-buffer "
                    "structs, as the reference's capture side leaves them",
            "config": {"workload": f"{cfg['desc']}, one frame per step", "mics": 2, "frame_len": 1024,
                       "calls_per_frame": 7, "path": "libtdoa host-CPU path (tdoa_ref_set_device(-1), "
                                                     "csrc/tdoa_host_path.cpp, AVX2), one thread",
                       "parallelism": f"dp{world} (per-frame, no collective)"},
            "parity": res["parity"],
            "roofline": None,
            "gpu_backed": {"value": gpu["value"], "ms_per_step": gpu["ms_per_step"], "parity": gpu["parity"],
                           "note": "the same seven calls with the GPU-backed symbols (default device): "
                                   "latency-bound, three GPU round trips per frame (each write_out's "
                                   "launch also computes the buffer's normalize and window); the batched "
                                   "API is configs 2-5"},
            "note": "BASELINE config 1 is defined on the host CPU: the line's value is libtdoa's own host "
                    "path (no HIP call); cpu_baseline is the oracle port of the same sequence",
            "cpu_baseline": cpu_baseline_config1(args, res) if not args.no_cpu else None,
        }
        print(json.dumps(line), flush=True)
    shard.finalize()


def _cpu_info(threads):
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    return {"cores": threads, "nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_model": model,
            "threads_source": "OMP_NUM_THREADS (the box's CPU share per GPU)"
            if os.environ.get("OMP_NUM_THREADS") else "all CPUs in this process's affinity set"}


def _cpu_threads():
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env > 0:
        return env
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline_stream(args, lut, window, S_lag):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from tdoa import synth
    threads = _cpu_threads()
    adc = synth.adc_stream(64, 64 * 512, 3, lut, S_lag, synth.SEEDS[5]).numpy()
    O.stream_run(adc[:4, :4096], 1024, 48000, S_lag, window, lut, threads=threads)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        r = O.stream_run(adc, 1024, 48000, S_lag, window, lut, threads=threads, max_trig=64)
        n += int(r["n_trig"].sum())
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "localizations/s", **_cpu_info(threads), "kind": "port",
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
    threads = _cpu_threads()
    nfr = 2048 if args.config == 2 else 128
    fr, _, _ = synth.adc_frames(nfr, M, N, lut, 46, synth.SEEDS[args.config])
    fr = fr.numpy()
    O.localize_batch(fr[:16], 46, window, lut, threads=threads, want_scores=False)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        O.localize_batch(fr, 46, window, lut, threads=threads, want_scores=False)
        n += fr.shape[0]
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "localizations/s", **_cpu_info(threads), "kind": "port",
            "sample": f"{n} config-{args.config} frames ({M}x{N} ADC-like, batches of {nfr}) "
                      f"in {dt:.1f} s, oracle/tdoa_oracle.c (reference correlations.c + "
                      f"vga_heatmap.h algorithm, DIRECT integer xcorr), OpenMP {threads} threads"}


def traffic_entry(args, first="", fused=True):
    """HBM bytes per launch from the committed PMC passes, used only when they
    were taken on the kernel this run dispatches."""
    kname = dominant_kernel(args.config, args.engine, first, fused)
    if not kname or not os.path.exists(args.traffic_json):
        return None, None
    try:
        tj = json.load(open(args.traffic_json))
    except (OSError, ValueError):
        return None, None
    e = tj.get(f"c{args.config}_{args.engine}") or {}
    names = kname.split(" + ")
    if e.get("kernel") != names[0]:
        return None, None
    if args.config in (3, 4) and fused and any(k.startswith("k_grid") for k in e.get("kernels", {})):
        return None, None  # a pass taken with the separate grid kernel: not this launch's traffic
    src = (f"{os.path.relpath(args.traffic_json, ROOT)}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
           f"passes on {kname} ({e.get('date', 'undated')}), read = 2 x FETCH_SIZE")
    if len(names) == 1:
        return e.get("hbm_bytes_per_launch"), src
    # several kernels per launch: the sum of theirs (each dispatched once per launch)
    ks = e.get("kernels", {})
    per = [sum(v["hbm_bytes"] for k, v in ks.items() if k.startswith(n + "<") or k == n) for n in names]
    if not all(per):
        return None, None
    return sum(per), src


def stream_traffic(args):
    """Config 5: HBM bytes per hop of the hop's kernels (trigger, DIRECT on the
    triggered batch, update) from the committed PMC passes."""
    try:
        e = json.load(open(args.traffic_json)).get("c5_direct") or {}
    except (OSError, ValueError):
        return None, None
    ks = e.get("kernels", {})
    # k_stream_update runs only for shapes k_direct_mfma does not solve (the
    # config-5 hop fuses the EMA and its grid into k_direct_mfma)
    names = ("k_stream_trigger_p", "k_direct_mfma", "k_stream_update")
    per = [sum(v["hbm_bytes"] for k, v in ks.items() if k.split("<")[0] == n) for n in names]
    if not all(per[:2]):
        return None, None
    names = names if per[2] else names[:2]
    return sum(per), (f"{os.path.relpath(args.traffic_json, ROOT)}: rocprofv3 --pmc FETCH_SIZE / "
                      f"WRITE_SIZE passes on {' + '.join(names)} ({e.get('date', 'undated')}), "
                      "read = 2 x FETCH_SIZE; the trigger re-reads the two previous hops")


def executed_flops(args, frames):
    """FP32 flops a launch of this config actually executes: SQ_INSTS_VALU_FLOPS_FP32 per
    dispatch (tools/summarize_flops.py -> profiles/valu_flops.json) per localization, times
    this launch's frames; (flops per launch, source) or (None, None)."""
    path = os.path.join(ROOT, "profiles", "valu_flops.json")
    try:
        e = json.load(open(path)).get(f"c{args.config}_{args.engine}") or {}
    except (OSError, ValueError):
        return None, None
    if not e.get("executed_fp32_flops_per_loc"):
        return None, None
    return e["executed_fp32_flops_per_loc"] * frames, (
        f"profiles/valu_flops.json: rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 on the launch's kernels "
        f"({e.get('date', 'undated')}), {e['executed_fp32_flops_per_loc']:.4g} flop per localization executed "
        f"against the model's {e['survey_model_flops_per_loc']:.4g}")


def _achievable(achieved_gbs):
    """frac against the measured achievable read rate beside the spec fraction."""
    rd, cp = achievable_hbm()
    if not rd:
        return {"achievable": None, "frac_achievable": None}
    return {"achievable": rd, "frac_achievable": achieved_gbs / rd,
            "achievable_source": f"{os.path.relpath(CALIB_JSON, ROOT)}: 16-B-per-lane read sweep over 1 GiB "
                                 f"(rocprofv3 {rd:.0f} GB/s; the kernels are read-dominated)"}


def launch_workers(args):
    """--gpus N > 1 outside a torch.distributed launch: start the N rank
    processes (one per GPU) through torch.distributed.run as a CHILD process,
    before this process has touched a GPU, and return its exit code.  None:
    this process is a rank of a launch (or N = 1) and runs the bench itself."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess
    # --standalone: the c10d rendezvous store binds a free port itself (no
    # probe-then-rebind race for the port); 127.0.0.1 as the node address
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--local-addr", "127.0.0.1",
           os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def check_world(args, where):
    """The ranks that joined must be the ranks asked for (--gpus)."""
    seen = shard.ranks_seen()
    if seen != args.gpus:
        print(f"bench.py: {where}: {seen} ranks joined, --gpus {args.gpus}", file=sys.stderr)
        sys.exit(3)
    return seen


def rehearse(args):
    """--cpu-rehearsal: the N-rank path without a GPU -- the self-launch, the
    gloo process group, the rank logic of tdoa/shard.py (per-rank batches,
    the timed bracket, max over ranks, sums), the JSON line and the rank-0
    cpu_baseline -- with a stand-in CPU step (a byte sum over the rank's
    frames).  Its value measures nothing and says so."""
    ri = shard.init_distributed("gloo")
    world = check_world(args, "rehearsal")
    cfg = CONFIGS[2]
    B = shard.rank_frames(64, ri.rank, ri.world, cfg["scaling"])
    rng = np.random.default_rng(shard.frame_seed(0x5EED0002, ri.rank))
    fr = rng.integers(0, 256, (B, cfg["M"], cfg["N"]), dtype=np.int16)
    t = shard.timed(lambda k: int(fr.sum()), args.steps, args.warmup)
    total = shard.sum_over_ranks([B * args.steps])[0]
    if ri.rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        import tdoa
        lut = O.build_lut(O.microphones_ref(), fs=50000, max_shift=46)
        line = {"metric": "REHEARSAL (no GPU, stand-in CPU step): rank logic of "
                          "'GCC-PHAT localizations/sec, 3-mic x 1024-sample frames'",
                "value": total / t["wall_max_s"], "unit": "frames/s (stand-in step)",
                "n_gpus": 0, "ranks_seen": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": t["wall_max_s"] * 1e3 / args.steps, "higher_is_better": True,
                "scaling": cfg["scaling"], "vs_baseline": None, "dtype": "none",
                "data": "rehearsal: random bytes, byte-sum step", "rehearsal": True,
                "config": {"workload": "rehearsal of the config-2 rank logic", "batch_per_rank": B,
                           "parallelism": f"dp{world} (gloo, CPU)"},
                "roofline": None,
                "cpu_baseline": None if args.no_cpu else cpu_baseline(
                    args, lut.reshape(3, -1), tdoa.dpss_q15(1024))}
        print(json.dumps(line), flush=True)
    shard.finalize()


def main():
    args = parse()
    rc = launch_workers(args)  # before anything touches a GPU
    if rc is not None:
        sys.exit(rc)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        print(f"bench.py: WORLD_SIZE {env_world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(3)
    if args.cpu_rehearsal:
        return rehearse(args)
    ri = shard.init_distributed(args.dist_backend)
    check_world(args, "process group")
    dev = torch.device("cuda", ri.local_rank if args.rank_device < 0 else args.rank_device)
    torch.cuda.set_device(dev)
    cache = {}
    if args.config == 5:
        return main_stream(args, dev, ri, cache)
    if args.config == 1:
        return main_config1(args, dev, ri)
    main_res = time_engine(args.engine, args, dev, ri, cache)
    other = None
    if args.also:
        other = time_engine("direct" if args.engine == "gcc_phat" else "gcc_phat", args, dev,
                            ri, cache)
    world = shard.ranks_seen()
    if ri.rank == 0:
        traffic, tsrc = traffic_entry(args, main_res.get("kernel", ""), main_res.get("grid_fused", True))
        cfg = CONFIGS[args.config]
        shape = f"{cfg['M']}-mic x {cfg['N']}-sample frames"
        B = main_res["frames_per_rank"]
        line = {
            "metric": f"GCC-PHAT localizations/sec, {shape}"
            if args.engine == "gcc_phat" else
            f"localizations/sec (DIRECT exact xcorr), {shape}",
            "value": main_res["value"],
            "unit": "localizations/s",
            "n_gpus": world,
            "ranks_seen": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "preflight": {"steps": main_res["preflight_steps"], "seconds": args.preflight_s,
                          "steady": main_res["steady"],
                          "note": "untimed, before the warmups: every rotating batch once, then "
                                  "steps until the time has passed, then windows of launches until "
                                  "two consecutive windows' mean launch time agree within 2 % "
                                  "(steady state: a box still clearing a previous job's memory "
                                  "runs the kernels slower for seconds), at most settle_max_s"},
            "ms_per_step": main_res["ms_per_step"],
            "gpu_clock_mhz": main_res["gpu_clock_mhz"],
            "higher_is_better": True,
            "scaling": cfg["scaling"],
            "vs_baseline": None,
            "dtype": "f32" if args.engine == "gcc_phat" else "int16->int64",
            "data": "synthetic (ADC-like u8 frames, injected integer delays, generated on the GPU, "
                    f"resident in HBM, {main_res['rotate_batches']} rotating batches > 256 MiB)"
                    if main_res["rotate_batches"] > 1 else
                    "synthetic (ADC-like u8 frames, injected integer delays, generated on the GPU, "
                    "resident in HBM; one batch larger than the 256 MiB Infinity Cache)",
            "config": {"workload": f"{cfg['desc']}, {B} frames per GPU per step, "
                                   "xcorr + lag prior + (x,y) grid"
                                   + (" + least-squares (x,y)" if main_res["ls"] else ""),
                       "engine": args.engine, "batch_per_gpu": B,
                       "global_batch": args.batch if cfg["scaling"] == "strong" else B * world,
                       "mics": cfg["M"], "frame_len": cfg["N"],
                       "step_streams": main_res["streams"],
                       "parallelism": f"dp{world} (frame shards, no collective)"},
            "roofline": {"bound": "hbm", "achieved": main_res["achieved_gbs"],
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": main_res["achieved_gbs"] / HBM_PEAK_GBS,
                         **_achievable(main_res["achieved_gbs"]),
                         "traffic": traffic,
                         "traffic_source": tsrc,
                         "kernel": dominant_kernel(args.config, args.engine, main_res.get("kernel", ""),
                                                   main_res.get("grid_fused", True))
                         or "all kernels of a launch",
                         "kernel_ms": main_res["kernel_ms"],
                         # step_streams > 1: kernel_ms is the events' span per step with that many
                         # launches in flight; a profiler's per-dispatch duration spans the overlap
                         # (one stream: the two agree, profiles/r06_c2_gcc_phat_kernel_stats_1stream.csv)
                         "concurrent_launches": main_res["streams"],
                         "bytes_per_loc": main_res["bytes_per_loc"]},
            # the bound that actually binds an fp32 FFT path: FP32 vector issue
            "valu_roofline": _valu_roofline(args, main_res) if args.engine == "gcc_phat" else None,
            "parity": main_res.get("parity"),
            "cpu_baseline": None,
        }
        if other is not None:
            other.pop("parity", None)
            line["other_engine"] = other
        if not args.no_cpu:  # rank 0, after the timed region, at every world size
            line["cpu_baseline"] = cpu_baseline(args, cache["lut"], cache["window"])
        print(json.dumps(line), flush=True)
    shard.finalize()


def _valu_roofline(args, res):
    """FP32 VALU roofline of the launch: SURVEY.md 8(d)'s flop model (forward FFTs, PHAT
    and FULL inverse FFTs per localization) and, where a counter pass exists for this
    batch, the flops the kernels actually executed (the pruned inverse as built)."""
    r = {"achieved": res["valu_tflops"], "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
         "frac": res["valu_tflops"] / VALU_PEAK_TFLOPS, "flop_model": "SURVEY.md 8(d) GCC-PHAT model"}
    fl, src = executed_flops(args, res["frames_per_rank"])
    if fl:
        t = fl / (res["kernel_ms"] * 1e-3) / 1e12
        r["executed"] = {"achieved": t, "frac": t / VALU_PEAK_TFLOPS, "flops_per_launch": fl,
                         "source": src}
    return r


def main_stream(args, dev, ri, cache):
    res = time_stream(args, dev, ri, cache)
    world = shard.ranks_seen()
    if ri.rank == 0:
        cfg = CONFIGS[5]
        line = {
            "metric": "streaming localizations/sec (triggered frames), 3-mic x 1024-sample "
                      "frames, 48 kHz, 512-sample hop",
            "value": res["value"], "unit": "localizations/s", "n_gpus": world,
            "ranks_seen": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
            "gpu_clock_mhz": res["gpu_clock_mhz"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "int16->int64",
            "data": "synthetic u8 capture bytes (bursts from a fixed source per stream over a "
                    "quiet floor), 64-hop capture ring per stream resident in HBM",
            "config": {"workload": f"{cfg['desc']}, {args.batch} streams per GPU",
                       "streams_per_gpu": args.batch, "hop": cfg["hop"], "fs": cfg["fs"],
                       "mics": 3, "frame_len": 1024,
                       "parallelism": f"dp{world} (stream shards, no collective)"},
            "stream": {k: res[k] for k in ("kernel_ms", "triggered", "gated", "launch",
                                           "stream_samples_per_s", "realtime_streams")},
            "latency_ms": res["latency_ms"],
            # the hop's algorithmic bytes: every stream's 512 capture samples (M bytes
            # each) read once, over the hop's GPU time (memset + trigger + DIRECT +
            # update, HIP events on the pipeline stream)
            "roofline": {"bound": "hbm", "achieved": res["capture_bytes_per_step"] / ri.world /
                         (res["kernel_ms"] * 1e-3) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": res["capture_bytes_per_step"] / ri.world / (res["kernel_ms"] * 1e-3) / 1e9
                         / HBM_PEAK_GBS,
                         **dict(zip(("traffic", "traffic_source"), stream_traffic(args))),
                         "kernel": "all kernels of a hop (trigger + DIRECT)", "kernel_ms": res["kernel_ms"],
                         "bytes_per_step": res["capture_bytes_per_step"] // ri.world,
                         # what the sliding trigger must read per hop: the half-window
                         # sums after every sample need the entering sample (this hop),
                         # the one crossing the window's middle (N/2 = one hop back) and
                         # the leaving one (N = two hops back): 3 x the hop's capture
                         # bytes (rolling_buffer.c:16-41 per sample, sample_compute.h:75-91)
                         "sliding": {
                             "bytes_per_step": 3 * res["capture_bytes_per_step"] // ri.world,
                             "achieved": 3 * res["capture_bytes_per_step"] / ri.world /
                             (res["kernel_ms"] * 1e-3) / 1e9,
                             "frac": 3 * res["capture_bytes_per_step"] / ri.world /
                             (res["kernel_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                             "note": "the trigger's algorithmic reads (current hop + the two hops "
                                     "leaving the half-windows); `traffic` counts these plus the "
                                     "triggered frames DIRECT reads and the EMA states"}},
            "cpu_baseline": None,
        }
        if not args.no_cpu:  # rank 0, after the timed region, at every world size
            line["cpu_baseline"] = cpu_baseline_stream(args, cache["lut"], cache["window"],
                                                       cache["S"])
        print(json.dumps(line), flush=True)
    shard.finalize()


if __name__ == "__main__":
    main()
