#!/usr/bin/env python3
"""Phase timeline of k_frame16 (the fused long-frame GCC-PHAT kernel) from
libtdoa_diag.so's per-wave s_memtime stamps.  Diagnostic only.

    python tools/diag_frame16.py [config 3|4] [B]
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
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
M, N, xy = (4, 4096, synth.square_mics(0.15)) if cfg == 3 else (8, 2048, synth.circle_mics(8, 0.15))
loc = Localizer(engine="gcc_phat", num_mics=M, frame_len=N, sample_rate_hz=50000, mic_xy=xy)
fr, _, _ = synth.adc_frames(B, M, N, loc.lut(), loc.dims.S, 5, device="cuda")
out = loc.alloc_outputs(B)
for _ in range(5):
    loc.localize_into(fr, out)
torch.cuda.synchronize()
L = tdoa.load()
L.tdoa_diag_fetch_f16.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(1 << 16, np.uint64)
assert L.tdoa_diag_fetch_f16(buf.ctypes.data_as(C.c_void_p), 1 << 16) == 0
wave_kernel = cfg == 4 and os.environ.get("TDOA_F16", "grp") == "w"  # k_frame16w
W = 32 if wave_kernel else 48  # stamps per wave record; the last three: end memtime, start / end realtime
st = buf[:(len(buf) // W) * W].reshape(-1, W).astype(np.int64)
st = st[st[:, 0] > 0]
G = 16384 // N
P = M * (M - 1) // 2
R = (P + G - 1) // G
if wave_kernel:
    # k_frame16w: start, forward, split, then one stamp per pair of the wave
    # (waves 0-11 run two pairs, 12-15 one: their stamp 4 stays 0)
    names = ["start", "forward", "split", "pair 1"]
    w = np.arange(len(st)) % 16
    two = st[w < P - 16]
    d = two[:, 4] - two[:, 3]
    print("k_frame16w second pair (waves with two): p10 / p50 / p90 %.0f %.0f %.0f" %
          (np.percentile(d, 10), np.median(d), np.percentile(d, 90)))
    print("per wave: median cycles after the split barrier to the end of pair 1 / pair 2")
    for wi in range(16):
        sw = st[w == wi]
        e1 = np.median(sw[:, 3] - sw[:, 2])
        e2 = np.median(sw[:, 4] - sw[:, 2]) if wi < P - 16 else float("nan")
        print(f"  wave {wi:2d}: {e1:8.0f} {e2:8.0f}")
else:
    # the forward's six barriers (DC sum, pass 1 .. 3 reads / writes), then
    # its closing mark
    names = ["start", "fw dc", "fw p1", "fw p2 dft", "fw p2 wr", "fw p3 dft", "fw p3 wr", "forward",
             "U regs"] + sum([[f"r{r} Y", f"r{r} p1 dft", f"r{r} p1 wr", f"r{r} p2 dft",
                                                   f"r{r} p2 wr", f"r{r} p3"] for r in range(R)], [])
    dm = os.environ.get("TDOA_F16_DEFER", "1" if R >= 2 else "0")
    if dm == "1":
        names.append("epilogue")  # the deferred pair outputs (DM 1)
n = len(names)
print(f"config {cfg}: M={M} N={N} P={P} G={G} rounds={R}, waves {len(st)}")
life = st[:, W - 3] - st[:, 0]
print("wave life (cycles): p50 %.0f; clock %.2f GHz" % (np.median(life),
      np.median(life / ((st[:, W - 1] - st[:, W - 2]) / 100e6)) / 1e9))
print("phase durations (cycles): p10 / p50 / p90")
for i in range(1, n):
    d = st[:, i] - st[:, i - 1]
    print(f"  {names[i]:9s} {np.percentile(d, 10):8.0f} {np.median(d):8.0f} {np.percentile(d, 90):8.0f}")
d = st[:, W - 3] - st[:, n - 1] if not wave_kernel else st[:, W - 3] - np.where(st[:, 4] > 0, st[:, 4], st[:, 3])
print(f"  {'tail':9s} {np.percentile(d, 10):8.0f} {np.median(d):8.0f} {np.percentile(d, 90):8.0f}")
