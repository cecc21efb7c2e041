"""The long-frame GCC-PHAT kernel variants the library selects once per process
(environment, tdoa_phat_r16.hip), each in a child process against the fp64
oracle (oracle/gcc_phat_oracle.py) with test_gpu_gcc_phat.py's tolerances:

  TDOA_F16=w          k_frame16w, one wave per pair (config 4's shape)
  TDOA_F16_DEFER=0    k_frame16 with every pair's outputs in its round (config 3
                      and 4 shapes)
  TDOA_F16_DEFER=1    k_frame16 with the deferred per-frame epilogue (at
                      C = 4096 the window table leaves no LDS for it: in-round)
  TDOA_F16_FG=1       the grid solved inside k_frame16 by the last pair round's
                      idle waves (the previous frame's compact scores kept in
                      LDS: one buffer with the deferred epilogue, two with
                      in-round outputs) instead of by k_grid_bb after it (the
                      default: measured faster at both shapes)
Every case also checks the cell / max_Lf bit for bit against the exhaustive
float32 scan of the run's own weighted scores (vga_heatmap.h:99-108).

The defaults (k_frame16, deferred lagged epilogue at configs 3 and 4) run in
test_gpu_gcc_phat.py itself.  k_frame16w and the fused grid are A/B paths that
measured slower: they are built only into tdoa/libtdoa_ab.so (Makefile "ab",
TDOA_AB=1), which those children load through TDOA_LIB; libtdoa.so has neither.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AB_LIB = os.path.join(ROOT, "audio-triangulation_amd", "tdoa", "libtdoa_ab.so")

CHILD = r"""
import sys
sys.path[:0] = [{pkg!r}, {orc!r}, {tests!r}]
import numpy as np
import gcc_phat_oracle as G
from tdoa import synth
from tdoa.localizer import Localizer
from test_gpu_gcc_phat import check_phat, _np, _grid_f32
M, N = {M}, {N}
xy = synth.square_mics(0.15) if M == 4 else synth.circle_mics(8, 0.15)
kw = dict(num_mics=M, frame_len=N, sample_rate_hz=50000, mic_xy=xy)
ph = Localizer(engine="gcc_phat", **kw)
S = ph.dims.S
fr, _, _ = synth.adc_frames(300, M, N, ph.lut(), S, 0x5A + M, device="cuda")
fr2 = synth.full_range_frames(4, M, N, 11, device="cuda")
import torch
fr = torch.cat([fr, fr2]).contiguous()
got = _np(ph.localize(fr, scores=True))
exp = G.gcc_phat_batch(fr.cpu().numpy(), S, ph.window(), ph.lut())
check_phat(got, exp)
cell, mx = _grid_f32(got["weighted_f"], ph.lut())
assert (got["cell"] == cell).all() and (got["max_Lf"] == mx).all()
lean = _np(ph.localize(fr))  # no scores requested: the bench's path
for k in lean:
    assert np.array_equal(lean[k], got[k]), k
print("variant ok", ph.batch_kernel(), "grid_fused", ph.batch_grid_fused())
"""


@pytest.mark.parametrize("env,M,N", [
    ({"TDOA_F16": "w"}, 8, 2048),
    ({"TDOA_F16_DEFER": "0"}, 8, 2048),
    ({"TDOA_F16_DEFER": "0"}, 4, 4096),  # config 3 with in-round outputs
    ({"TDOA_F16_DEFER": "1"}, 4, 2048),  # one pair round, epilogue forced
    ({"TDOA_F16_FG": "1"}, 8, 2048),  # config 4, deferred epilogue: one score buffer
    ({"TDOA_F16_FG": "1"}, 4, 4096),  # config 3 with the fused grid (in-round outputs)
    ({"TDOA_F16_FG": "1", "TDOA_F16_DEFER": "0"}, 8, 2048),  # in-round outputs: double-buffered scores
])
def test_frame16_variant_vs_fp64(env, M, N):
    code = CHILD.format(pkg=os.path.join(ROOT, "audio-triangulation_amd"), orc=os.path.join(ROOT, "oracle"),
                        tests=os.path.join(ROOT, "tests"), M=M, N=N)
    e = dict(os.environ, **env)
    if "TDOA_F16" in env or "TDOA_F16_FG" in env:  # the A/B kernels live in the A/B library
        e["TDOA_LIB"] = AB_LIB
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "variant ok" in r.stdout
    if env.get("TDOA_F16") == "w":
        assert "variant ok k_frame16w" in r.stdout, r.stdout
    if env.get("TDOA_F16_FG") == "1":
        assert "grid_fused True" in r.stdout, r.stdout
