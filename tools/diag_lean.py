#!/usr/bin/env python3
"""Timeline of k_p1k_lean (libtdoa_diag.so: absolute s_memtime stamps per wave
at its phase boundaries).  Diagnostic only; never used by tests or bench.py.

    python tools/diag_lean.py [B]
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

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
loc = Localizer(engine="gcc_phat")
fr, _, _ = synth.adc_frames(B, 3, 1024, loc.lut(), 46, 1, device="cuda")
out = loc.alloc_outputs(B)
for _ in range(20):
    loc.localize_into(fr, out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
loc.localize_into(fr, out)
e1.record()
torch.cuda.synchronize()
L = tdoa.load()
L.tdoa_diag_fetch_p1k.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(1 << 16, np.uint64)
assert L.tdoa_diag_fetch_p1k(buf.ctypes.data_as(C.c_void_p), 1 << 16) == 0
st = buf.reshape(-1, 16).astype(np.int64)
st = st[st[:, 0] > 0]
names = ["start", "staged", "mic0", "mic1", "pair01", "mic2+cross", "pair02", "pair12",
         "grid-wsc", "grid-loop", "grid-argmax", "grid-out"]
n = len(names)
t = st[:, :n] - st[:, 0].min()
print(f"B={B} waves={len(st)} kernel {e0.elapsed_time(e1) * 1e3:.1f} us (event, one launch)")
print("absolute (cycles from the first wave's start): p0 / p50 / p90 / max")
for i, nm in enumerate(names):
    c = t[:, i]
    print(f"  {nm:11s} {c.min():8d} {np.median(c):8.0f} {np.percentile(c, 90):8.0f} {c.max():8d}")
clk = (st[:, 13] - st[:, 0]) / ((st[:, 15] - st[:, 14]) / 100e6) / 1e9
print(f"shader clock over a wave's life (s_memtime / s_memrealtime): p10 {np.percentile(clk, 10):.2f} "
      f"p50 {np.median(clk):.2f} p90 {np.percentile(clk, 90):.2f} GHz")
rt = st[:, 14] - st[:, 14].min()  # memrealtime is one chip-wide 100 MHz clock
print(f"wave start (realtime, us): p50 {np.median(rt) / 100:.2f} max {rt.max() / 100:.2f}; "
      f"wave end p50 {np.median(st[:, 15] - st[:, 14].min()) / 100:.2f} max {(st[:, 15] - st[:, 14].min()).max() / 100:.2f}")
print("phase durations: p10 / p50 / p90")
for i in range(1, n):
    d = t[:, i] - t[:, i - 1]
    print(f"  {names[i]:11s} {np.percentile(d, 10):8.0f} {np.median(d):8.0f} {np.percentile(d, 90):8.0f}")
life = (st[:, 15] - st[:, 14]) / 100.0  # us
end = (st[:, 15] - st[:, 14].min()) / 100.0
blk = np.nonzero(buf.reshape(-1, 16)[:, 0] > 0)[0]  # global wave index = block * 8 + wave
wv = blk % 8
xcd = (blk // 8) % 8
print("wave life (us): p10 %.2f p50 %.2f p90 %.2f p99 %.2f max %.2f" % tuple(np.percentile(life, [10, 50, 90, 99, 100])))
print("wave end  (us): p10 %.2f p50 %.2f p90 %.2f p99 %.2f max %.2f" % tuple(np.percentile(end, [10, 50, 90, 99, 100])))
print("end by wave-in-workgroup:", " ".join(f"{np.median(end[wv == w]):.1f}" for w in range(8)))
print("end by block % 8 (XCD):  ", " ".join(f"{np.median(end[xcd == x]):.1f}" for x in range(8)))
m0 = t[:, 2] - t[:, 1]
print("mic0 phase by wave-in-workgroup (kcyc):", " ".join(f"{np.median(m0[wv == w]) / 1e3:.1f}" for w in range(8)))
