#!/usr/bin/env python3
"""Where a k_frame16 wave's frame time goes: barrier waits vs the rest, per
phase.  Diagnostic only (libtdoa_diag.so: per-wave s_memtime stamps after each
phase boundary of the stamped frame, g_diag_f16, and each wave's arrival at the
frame's barriers, g_diag_f16b).

    python tools/diag_frame16_bar.py [config 3|4] [B]

Per wave: every arrival is matched with the first phase stamp after it (the
stamps sit right behind the barriers), so stamp - arrival is the wave's wait at
that barrier and arrival - previous stamp its work (VALU issue, LDS and memory
waits) in the interval.  Printed per interval: median over waves of work and
barrier wait, and the frame totals.  SQ counters give the same totals for the
whole launch (SQ_WAIT_ANY = waitcnt + barrier parking): tools/gpu/run.sh sq.
"""
import ctypes as C
import json
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
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
M, N, xy = (4, 4096, synth.square_mics(0.15)) if cfg == 3 else (8, 2048, synth.circle_mics(8, 0.15))
loc = Localizer(engine="gcc_phat", num_mics=M, frame_len=N, sample_rate_hz=50000, mic_xy=xy)
fr, _, _ = synth.adc_frames(B, M, N, loc.lut(), loc.dims.S, 5, device="cuda")
out = loc.alloc_outputs(B)
for _ in range(5):
    loc.localize_into(fr, out)
torch.cuda.synchronize()
L = tdoa.load()
W = 48
bufs = []
for fn in ("tdoa_diag_fetch_f16", "tdoa_diag_fetch_f16b"):
    f = getattr(L, fn)
    f.argtypes = [C.c_void_p, C.c_int]
    b = np.zeros(1 << 16, np.uint64)
    assert f(b.ctypes.data_as(C.c_void_p), 1 << 16) == 0
    bufs.append(b[:(len(b) // W) * W].reshape(-1, W).astype(np.int64))
st, ar = bufs
keep = st[:, 0] > 0
st, ar = st[keep], ar[keep]
waves = len(st)
rows = []
frame_t, bar_t = [], []
per_interval = {}
for w in range(waves):
    s = st[w, :W - 3]
    s = s[s > 0]
    a = ar[w]
    a = a[a > 0]
    total = s[-1] - s[0]
    bw = 0
    prev = s[0]
    for i, t in enumerate(a):
        nxt = s[s > t]
        if not len(nxt):
            continue
        wait = nxt[0] - t
        work = t - prev
        per_interval.setdefault(i, []).append((work, wait, w % 16))
        bw += wait
        prev = nxt[0]
    frame_t.append(total)
    bar_t.append(bw)
frame_t, bar_t = np.array(frame_t), np.array(bar_t)
res = {"config": cfg, "waves": waves, "frame_cycles_p50": float(np.median(frame_t)),
       "barrier_wait_cycles_p50": float(np.median(bar_t)),
       "barrier_wait_frac_p50": float(np.median(bar_t / frame_t)),
       "intervals": []}
print(f"config {cfg}: {waves} waves; stamped frame p50 {np.median(frame_t):.0f} cycles, "
      f"barrier wait p50 {np.median(bar_t):.0f} ({100 * np.median(bar_t / frame_t):.1f} %)")
print("interval  work p50  barrier-wait p50  (cycles; work = VALU issue + LDS / memory waits)")
for i in sorted(per_interval):
    v = np.array(per_interval[i])
    wk, wt = float(np.median(v[:, 0])), float(np.median(v[:, 1]))
    res["intervals"].append({"barrier": i, "work_p50": wk, "wait_p50": wt})
    print(f"  {i:3d}   {wk:8.0f}   {wt:8.0f}")
# which waves are late: median work per interval by wave index (wave % 16:
# SIMD = wave % 4), for the intervals with the largest waits
top = sorted(per_interval, key=lambda i: -np.median(np.array(per_interval[i])[:, 1]))[:8]
print("median work by wave index (rows: interval; columns: waves 0..15)")
res["work_by_wave"] = {}
for i in sorted(top):
    v = np.array(per_interval[i])
    row = [float(np.median(v[v[:, 2] == wi, 0])) if (v[:, 2] == wi).any() else float("nan") for wi in range(16)]
    res["work_by_wave"][i] = row
    print(f"  {i:3d} " + " ".join(f"{x:6.0f}" for x in row))
print(json.dumps(res))
