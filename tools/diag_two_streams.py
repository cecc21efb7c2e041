#!/usr/bin/env python3
"""Config 2: steps on one stream vs alternating over two or four streams (each
with its own outputs), wall time per step.  Diagnostic only.

    python tools/diag_two_streams.py [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))
import torch  # noqa: E402

from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 400
loc = Localizer(engine="gcc_phat")
lut = loc.lut().reshape(3, 101, 101)
R = 14
batches = [synth.adc_frames(4096, 3, 1024, lut, 46, 100 + r, device="cuda")[0] for r in range(R)]
for ns in (1, 2, 4, 1, 2, 4):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    outs = [loc.alloc_outputs(4096) for _ in range(ns)]
    for k in range(200):
        loc.localize_into(batches[k % R], outs[k % ns], streams[k % ns])
    torch.cuda.synchronize()
    for window in (20, K):
        t0 = time.perf_counter()
        for k in range(window):
            loc.localize_into(batches[k % R], outs[k % ns], streams[k % ns])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / window
        print(f"streams {ns} steps {window}: {dt * 1e6:.2f} us per step, {4096 / dt:.4g} loc/s")
