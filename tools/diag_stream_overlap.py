#!/usr/bin/env python3
"""Config 5: can a hop's DIRECT and another hop's trigger share the GPU?  Two
independent StreamPipelines (own capture, state and HIP stream) stepped
alternately, against one pipeline alone: the pair's time per hop-pair vs twice
one pipeline's hop.  An upper bound on what overlapping hop h's DIRECT with hop
h + 1's trigger inside one pipeline could gain.  Diagnostic only.

    python tools/diag_stream_overlap.py [S] [hops] [S_half]

With S_half: also one pipeline of S streams against two of S_half each
(the same streams as two shards on two HIP streams).
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
K = int(sys.argv[2]) if len(sys.argv) > 2 else 300
H = 512
loc = Localizer(sample_rate_hz=48000)
caps = [synth.adc_stream(S, 64 * H, 3, loc.lut(), loc.dims.S, synth.SEEDS[5] + i, device="cuda") for i in range(2)]
torch.cuda.synchronize()
pipes = [StreamPipeline(loc, c, hop=H) for c in caps]


def run(ps, k):
    for p in ps:
        for _ in range(10):
            p.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        for p in ps:
            p.step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k


for rnd in range(3):
    one = run(pipes[:1], K)
    two = run(pipes, K)
    print(f"round {rnd}: one pipeline {one * 1e6:.2f} us per hop; two pipelines {two * 1e6:.2f} us per hop pair "
          f"({two / 2 * 1e6:.2f} per hop, {100 * (1 - two / (2 * one)):.1f} % saved)")
if len(sys.argv) > 3:
    Sh = int(sys.argv[3])
    halves = [StreamPipeline(loc, caps[0][i * Sh:(i + 1) * Sh].contiguous(), hop=H) for i in range(2)]
    for rnd in range(3):
        one = run(pipes[:1], K)
        two = run(halves, K)
        print(f"round {rnd}: {S} streams as one pipeline {one * 1e6:.2f} us per hop; as two shards of {Sh} "
              f"{two * 1e6:.2f} us per hop")
    for p in halves:
        p.close()
for p in pipes:
    p.close()
