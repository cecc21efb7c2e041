#!/usr/bin/env python3
"""Diagnostic (round 6): the packed compact range (lo | w << 8 | off << 16)
every k_frame16 thread holds for the four-pairs epilogue, dumped by a build
with -DF16_RNG_DUMP over the first 1024 lag slots, against the host's kp.wc_*
(recomputed here from the LUT as tdoa_capi.cpp does).

    TDOA_LIB=.../libtdoa_X.so python3 tools/diag_rng.py [3|4]

The lane -> pair map is k_frame16's f16_epi_pair: packed (the default) or,
with EPI_SPREAD=1 in the environment here for a -DF16_EPI_SPREAD=1 build,
spread over a multiple of four waves.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))
from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
M, N, mics = (4, 4096, synth.square_mics(0.15)) if cfg == 3 else (8, 2048, synth.circle_mics(8, 0.15))
loc = Localizer(engine="gcc_phat", num_mics=M, frame_len=N, mic_xy=mics)
P, K = loc.dims.P, loc.dims.K
lut = loc.lut().reshape(P, -1)
lo, hi = lut.min(1).astype(int), lut.max(1).astype(int)
if P > 8:
    lo &= ~3
w = hi - lo + 1
off = np.concatenate([[0], np.cumsum((w + 3) & ~3)[:-1]])
fr, _, _ = synth.adc_frames(2048, M, N, lut, loc.dims.S, 5, device="cuda")
out = loc.alloc_outputs(2048)
loc.localize_into(fr.contiguous(), out)
torch.cuda.synchronize()
got = out["lags"].reshape(-1)[:1024].cpu().numpy().astype(np.uint32)
bad = 0
rows = set()
spread = os.environ.get("EPI_SPREAD", "0") != "0"
EW = min(16, (((P + 3) // 4 + 3) & ~3)) if spread else (P + 3) // 4
for t in range(1024):
    wv, q = t >> 6, (t >> 4) & 3
    p = (wv + EW * q if spread else 4 * wv + q) if wv < EW else P
    if p >= P:
        continue
    exp = int(lo[p]) | int(w[p]) << 8 | int(off[p]) << 16
    if int(got[t]) != exp:
        if bad < 12:
            print(f"thread {t} pair {p}: got lo {got[t] & 255} w {(got[t] >> 8) & 255} off {got[t] >> 16}"
                  f" expected lo {lo[p]} w {w[p]} off {off[p]}")
        bad += 1
        rows.add((t >> 6, (t >> 4) & 3))
print("wrong (wave, row):", sorted(rows))
print(f"config {cfg}: {bad} of {16 * P} epilogue threads hold a wrong range")
