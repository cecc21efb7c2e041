#!/usr/bin/env python3
"""Per-step GPU timeline of a short config-2 timed region (diagnostic only).

    python3 tools/diag_first_steps.py [--steps 20] [--streams 2] [--reps 5]

The bench's driver shape (--steps 20 --warmup 5) runs ~1.5 us per step slower
than 400 steps.  This replays that region -- warmups, sync, then K launches
alternating over the step streams -- with a HIP event before and after every
launch on its own stream, and prints each step's start (relative to step 0's)
and duration, so the first and last steps' share of the gap can be read off.
The events add host calls between launches, so absolute numbers run a little
above the bench's; compare the steps with each other.
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))

import bench  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS[2]
    loc = Localizer(engine="gcc_phat", num_mics=cfg["M"], frame_len=cfg["N"],
                    mic_xy=bench.config_mics(cfg), device=0)
    M, N, P = loc.dims.M, loc.dims.N, loc.dims.P
    B = 4096
    lut = loc.lut().reshape(P, -1)
    R = 8
    batches = [bench.make_frames(B, M, N, lut, loc.dims.S, 0x5EED0100 + r, dev)[0] for r in range(R)]
    Q = args.streams
    outs = [loc.alloc_outputs(B, grid=True, ls=False) for _ in range(Q)]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(device=dev) for _ in range(Q - 1)]
    launches = [loc.prepare(batches[k % R], outs[k % Q], streams[k % Q]) for k in range(R * Q)]
    for k in range(2000):  # settle the clock
        launches[k % len(launches)]()
    torch.cuda.synchronize(dev)
    K = args.steps
    starts = np.zeros((args.reps, K))
    durs = np.zeros((args.reps, K))
    for rep in range(args.reps):
        for k in range(args.warmup):
            launches[k % len(launches)]()
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        for k in range(K):
            st = streams[k % Q]
            ev[k][0].record(st)
            launches[k % len(launches)]()
            ev[k][1].record(st)
        torch.cuda.synchronize(dev)
        for k in range(K):
            starts[rep, k] = ev[0][0].elapsed_time(ev[k][0]) * 1e3
            durs[rep, k] = ev[k][0].elapsed_time(ev[k][1]) * 1e3
    end = np.median(starts[:, -1] + durs[:, -1])
    print(f"steps {K} streams {Q} reps {args.reps}: region (first start -> last end) p50 {end:.1f} us, "
          f"{end / K:.2f} us per step")
    print("step  start_us  duration_us   (medians over reps)")
    for k in range(K):
        print(f"{k:4d} {np.median(starts[:, k]):9.1f} {np.median(durs[:, k]):11.2f}")
    loc.close()


if __name__ == "__main__":
    main()
