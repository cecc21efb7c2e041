#!/usr/bin/env python3
"""GCC-PHAT vs DIRECT lag agreement on the config-2 bench batch and the
nature of the disagreements (diagnostic for the test contract)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import gcc_phat_oracle as G  # noqa: E402
from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402

ph = Localizer(engine="gcc_phat")
lut = ph.lut().reshape(3, 101, 101)
for seed in (synth.SEEDS[2], 0x5EED0002 + 104729):
    fr, cells, tau = synth.adc_frames(4096, 3, 1024, lut, 46, seed, device="cuda")
    g = {k: v.cpu().numpy() for k, v in ph.localize(fr, scores=True).items()}
    d = {k: v.cpu().numpy() for k, v in Localizer(engine="direct").localize(fr, scores=True).items()}
    e = G.gcc_phat_batch(fr.cpu().numpy(), 46, ph.window(), lut)
    same = g["lags"] == d["lags"]
    print(f"seed {seed:#x}: lags equal DIRECT {same.mean():.5f}, frames all-equal {same.all(-1).mean():.5f}, "
          f"cells equal {(g['cell'] == d['cell']).mean():.5f}, gpu==fp64 lags {(g['lags'] == e['lags']).mean():.5f}")
    srt = np.sort(e["scores_f"], axis=-1)
    m64 = srt[..., -1] - srt[..., -2]
    dsc = d["scores"].astype(np.float64)
    ds = np.sort(dsc, axis=-1)
    dm = (ds[..., -1] - ds[..., -2]) / np.maximum(np.abs(ds[..., -1]), 1)
    bad = np.argwhere(~same)
    print("  disagreements:", len(bad))
    for b, p in bad[:12]:
        # fp64 GCC score at DIRECT's lag vs at its own best
        kd = d["lags"][b, p] + 46
        kg = g["lags"][b, p] + 46
        print(f"   frame {b} pair {p}: gcc {g['lags'][b, p]} direct {d['lags'][b, p]} tau {tau[b].tolist()} "
              f"| fp64 gcc margin {m64[b, p]:.2e} gcc(best)-gcc(direct lag) {e['scores_f'][b, p, kg] - e['scores_f'][b, p, kd]:.2e} "
              f"| direct rel margin {dm[b, p]:.2e}")
    if len(bad):
        kd = d["lags"][~same] + 46
        kg = g["lags"][~same] + 46
        gap = e["scores_f"][~same, kg] - e["scores_f"][~same, kd] if False else \
            np.array([e["scores_f"][b, p, g["lags"][b, p] + 46] - e["scores_f"][b, p, d["lags"][b, p] + 46] for b, p in bad])
        print("  fp64 GCC gap (own best - at DIRECT's lag): max %.3e p50 %.3e" % (gap.max(), np.median(gap)))
        print("  DIRECT rel margin at disagreements: max %.3e p50 %.3e" % (dm[~same].max(), np.median(dm[~same])))
