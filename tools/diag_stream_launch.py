#!/usr/bin/env python3
"""Config 5 hop time by launch form: the per-hop hipGraph (the bench's form)
against plain stream launches of the same two kernels, interleaved, same box.
Diagnostic only.

    python tools/diag_stream_launch.py [S] [hops]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))
import torch  # noqa: E402

from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402
from tdoa.stream import StreamPipeline  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
K = int(sys.argv[2]) if len(sys.argv) > 2 else 400
H = 512
loc = Localizer(sample_rate_hz=48000)
cap = synth.adc_stream(S, 64 * H, 3, loc.lut(), loc.dims.S, synth.SEEDS[5], device="cuda")
torch.cuda.synchronize()
pipes = {g: StreamPipeline(loc, cap, hop=H, use_graph=g) for g in (True, False)}
for rnd in range(3):
    for g, p in pipes.items():
        for _ in range(20):
            p.step()
        p.stream.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            p.step()
        p.stream.synchronize()
        dt = (time.perf_counter() - t0) / K
        print(f"round {rnd} graph={int(g)}: {dt * 1e6:.2f} us per hop")
for p in pipes.values():
    p.close()
