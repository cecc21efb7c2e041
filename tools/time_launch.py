#!/usr/bin/env python3
"""Time a GCC-PHAT batch launch (the bench's no-scores outputs) for A/B builds whose
outputs are not meaningful (timing-only switches): HIP events around K launches.
Diagnostic only.

    TDOA_LIB=... python tools/time_launch.py <config 2|3|4> [B] [K] [nogrid]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))
import torch  # noqa: E402

from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402

cfg = int(sys.argv[1])
M, N, xy = {2: (3, 1024, None), 3: (4, 4096, synth.square_mics(0.15)), 4: (8, 2048, synth.circle_mics(8, 0.15))}[cfg]
B = int(sys.argv[2]) if len(sys.argv) > 2 else {2: 4096, 3: 65536, 4: 131072}[cfg]
K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
kw = dict(num_mics=M, frame_len=N, sample_rate_hz=50000)
if xy is not None:
    kw["mic_xy"] = xy
loc = Localizer(engine="gcc_phat", **kw)
fr, _, _ = synth.adc_frames(B, M, N, loc.lut(), loc.dims.S, 7, device="cuda")
out = loc.alloc_outputs(B, grid=not (len(sys.argv) > 4 and sys.argv[4] == "nogrid"))
for _ in range(3):
    loc.localize_into(fr, out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(K):
    loc.localize_into(fr, out)
e1.record()
torch.cuda.synchronize()
print(f"config {cfg} B={B}: {e0.elapsed_time(e1) / K:.4f} ms per launch ({os.path.basename(os.environ.get('TDOA_LIB', 'libtdoa.so'))})")
