#!/usr/bin/env python3
"""Per-phase cycle split of k_phat1024 (libtdoa_diag.so s_memtime stamps).
Diagnostic only; never used by tests or bench.py.

    TDOA_PHAT1024_WAVES=4 python tools/diag_p1k.py [B]
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
for _ in range(5):
    loc.localize_into(fr, out)
torch.cuda.synchronize()
L = tdoa.load()
L.tdoa_diag_fetch_p1k.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(1 << 16, np.uint64)
assert L.tdoa_diag_fetch_p1k(buf.ctypes.data_as(C.c_void_p), 1 << 16) == 0
st = buf.reshape(-1, 16).astype(np.int64)
st = st[st[:, 15] > 0]
names = ["tables", "fwd0|fwd1", "split0,1", "inv01|fwd2", "split2+cross", "inv02|inv12",
         "grid outputs", "grid wsc", "grid loop", "grid reduce"]
tot = st[:, :len(names)].sum(1)
it = np.median(st[:, 15])
print(f"B={B} waves={len(st)} iters/wave median {it}  total median {np.median(tot):.0f} cyc")
for i, nm in enumerate(names):
    print(f"  {nm:12s} {np.median(st[:, i]):9.0f} cyc  ({np.median(st[:, i] / tot) * 100:5.1f}%)"
          f"  p90 {np.percentile(st[:, i], 90):9.0f}")
print("  total per wave: p50 %.0f p90 %.0f p99 %.0f max %.0f" % tuple(np.percentile(tot, [50, 90, 99, 100])))
for i in range(6, 10):
    print(f"  {names[i]:14s} p99 {np.percentile(st[:, i], 99):9.0f} max {st[:, i].max():9.0f}")
