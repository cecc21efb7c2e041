#!/usr/bin/env python3
"""Why frames miss the grid settle path (configs 3/4): from the scores path's
outputs, per frame the settle test of k_settle (tdoa_grid.hip) restated in
numpy -- margin m_p - b_p > 2^-17 A and the peak tuple on the grid.
Diagnostic only; never used by tests or bench.py.

    python tools/diag_settle.py [cfg3|cfg4] [B]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))
import numpy as np  # noqa: E402

from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "cfg3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
M, N, xy = (4, 4096, synth.square_mics(0.15)) if shape == "cfg3" else (8, 2048, synth.circle_mics(8, 0.15))
loc = Localizer(engine="gcc_phat", num_mics=M, frame_len=N, mic_xy=xy)
P, K, S = loc.dims.P, loc.dims.K, loc.dims.S
lut = loc.lut().reshape(P, -1)
fr, cells, tau = synth.adc_frames(B, M, N, lut.reshape(P, 101, 101), S, 97, device="cuda")
o = {k: v.cpu().numpy() for k, v in loc.localize(fr, scores=True).items()}
prior = loc.prior()
best = o["lags"] + S
sc = o["scores_f"]
m = np.take_along_axis(sc, best[..., None], -1)[..., 0] * np.float32(prior[0])
s2 = np.where(np.arange(K)[None, None, :] == best[..., None], -np.inf, sc).max(-1)
b2 = np.maximum(s2, 0).astype(np.float32)
A = (np.abs(m) + np.abs(b2)).sum(-1)
margin_ok = ((m - b2).min(-1) * 131072.0 > A)
tuples = {tuple(t) for t in lut.T.tolist()}
on_grid = np.array([tuple(b) in tuples for b in best.tolist()])
inj = np.array([[lut[p][c] for p in range(P)] for c in np.asarray(cells.cpu() if hasattr(cells, "cpu") else cells)])
lag_inj = (best == inj).all(-1)
print(f"{shape}: B={B} margin ok {margin_ok.mean():.4f}  peak tuple on grid {on_grid.mean():.4f}  "
      f"settle {np.mean(margin_ok & on_grid):.4f}  lags == injected {lag_inj.mean():.4f}")
bad = ~margin_ok
if bad.any():
    r = (m - b2).min(-1)[bad] / A[bad]
    print("  margin-failing frames: min (m - b) / A p50 %.3g max %.3g" % (np.median(r), r.max()))
    pw = ((m - b2) * 131072.0 <= A[:, None])[bad].mean(0)
    print("  per pair failing fraction:", np.round(pw, 3).tolist())
