#!/usr/bin/env python3
"""Where k_grid_bb's time goes: per-wave s_memtime cycles accumulated by phase
in libtdoa_diag.so (tdoa_grid_bb.h BB_MARK), averaged per frame.  Diagnostic only.

    python tools/diag_grid_bb.py [config 3|4] [B]
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("TDOA_LIB", os.path.join(ROOT, "audio-triangulation_amd", "tdoa", "libtdoa_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tdoa  # noqa: E402
from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
M, N, xy = (4, 4096, synth.square_mics(0.15)) if cfg == 3 else (8, 2048, synth.circle_mics(8, 0.15))
loc = Localizer(engine="gcc_phat", num_mics=M, frame_len=N, sample_rate_hz=50000, mic_xy=xy)
fr, _, _ = synth.adc_frames(B, M, N, loc.lut(), loc.dims.S, 5, device="cuda")
out = loc.alloc_outputs(B)
for _ in range(2):
    loc.localize_into(fr, out)
torch.cuda.synchronize()
L = tdoa.load()
L.tdoa_diag_fetch_bb.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(8192 * 8, np.uint64)
assert L.tdoa_diag_fetch_bb(buf.ctypes.data_as(C.c_void_p), 8192 * 8) == 0
st = buf.reshape(-1, 8).astype(np.float64)
st = st[st[:, 5] > 0]
frames = st[:, 5].sum()
print(f"config {cfg}: B={B}, waves {len(st)}, frames seen {int(frames)}, P={loc.dims.P} K={loc.dims.K}")
names = ["frame load", "bounds", "seed + eval", "other evals"]
tot = st[:, :4].sum()
for i, n in enumerate(names):
    print(f"  {n:12s} {st[:, i].sum() / frames:9.0f} cycles/frame  ({100 * st[:, i].sum() / tot:4.1f} %)")
ev = st[:, 4].sum() / frames
print(f"  evaluations per frame: {ev:.2f} (incl. the seed)")
per_wave = st[:, :4].sum(axis=1)
print("  wave busy cycles: p10 %.3g  p50 %.3g  p90 %.3g  max %.3g" %
      tuple(np.percentile(per_wave, [10, 50, 90, 100])))
