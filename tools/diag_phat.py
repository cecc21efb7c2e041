#!/usr/bin/env python3
"""Per-phase cycle split of k_gcc_phat_1024 (libtdoa_diag.so stamps).
Diagnostic only; never used by tests or bench.py."""
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
for _ in range(3):
    loc.localize_into(fr, out)
torch.cuda.synchronize()
L = tdoa.load()
L.tdoa_diag_fetch_phat.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(1 << 16, np.uint64)
assert L.tdoa_diag_fetch_phat(buf.ctypes.data_as(C.c_void_p), 1 << 16) == 0
st = buf.reshape(-1, 8).astype(np.int64)
st = st[st[:, 7] > 0]
names = ["load+prep+fwd FFT", "split+PHAT", "inv FFT+argmax", "gate", "grid"]
tot = st[:, :5].sum(1)
print(f"B={B} workgroups={len(st)} iters/wg median {np.median(st[:, 7])}")
for i, nm in enumerate(names):
    print(f"  {nm:18s} {np.median(st[:, i]) / np.median(st[:, 7]):9.0f} cyc/iter ({np.median(st[:, i] / tot) * 100:5.1f}%)")
print(f"  total              {np.median(tot) / np.median(st[:, 7]):9.0f} cyc/iter (2 frames)")
