"""The remaining environment-selected kernel variants (INTEGRATION.md "Kernel
selection switches"), each in a child process -- the library reads its
switches once per process -- against the same oracles as the defaults:

  TDOA_P1K=w64       k_p1k_w64 (config 2 at one frame per 64-lane wave):
                     fp64 GCC-PHAT oracle with test_gpu_gcc_phat.py's
                     tolerances, its cell / max_Lf bit-equal to the exhaustive
                     float32 grid scan of its own weighted scores, and its
                     no-scores outputs equal to its scores run
  TDOA_EMA_WAVES=12  the 12-wave streaming DIRECT + EMA workgroup (config 5):
                     bit-exact against the oracle's sample-by-sample
                     sample_compute.h:53-146 (test_gpu_stream.py's compare)
  TDOA_DIRECT_XC3=0  DIRECT's xcorr one MFMA tile per pair instead of per
                     (frame, first mic) at three mics: config 2's batch bit-exact
                     against the oracle, and the streaming run above

The frame16 switches are tests/test_gpu_frame16_variants.py; TDOA_NO_COMPACT
is tests/test_gpu_bench_path.py.  k_p1k_w64 measured slower and is built only
into the A/B library tdoa/libtdoa_ab.so (Makefile "ab"), loaded here through
TDOA_LIB; libtdoa.so does not contain it.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
AB_LIB = os.path.join(ROOT, "audio-triangulation_amd", "tdoa", "libtdoa_ab.so")
PATHS = [os.path.join(ROOT, "audio-triangulation_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

W64 = r"""
import numpy as np, torch
import gcc_phat_oracle as G
from tdoa import synth
from tdoa.localizer import Localizer
from test_gpu_gcc_phat import check_phat, _np, _grid_f32
ph = Localizer(engine="gcc_phat")
assert ph.batch_kernel() == "k_p1k_w64", ph.batch_kernel()
lut = ph.lut()
g = np.load({golden!r})
cases = [torch.from_numpy(g["frames"]).cuda(),
         synth.adc_frames(4096, 3, 1024, lut.reshape(3, 101, 101), 46, synth.SEEDS[2], device="cuda")[0],
         synth.adc_frames(4093, 3, 1024, lut.reshape(3, 101, 101), 46, 0x77, device="cuda")[0],
         synth.full_range_frames(256, 3, 1024, 0xBEE, device="cuda"),
         torch.randint(0, 256, (512, 3, 1024), generator=torch.Generator().manual_seed(5),
                       dtype=torch.int16).cuda()]
for fr in cases:
    fr = fr.contiguous()
    got = _np(ph.localize(fr, scores=True))
    check_phat(got, G.gcc_phat_batch(fr.cpu().numpy(), 46, ph.window(), lut))
    cell, mx = _grid_f32(got["weighted_f"], lut)
    assert (got["cell"] == cell).all() and (got["max_Lf"] == mx).all()
    lean = _np(ph.localize(fr))
    for k in lean:
        assert np.array_equal(lean[k], got[k]), k
const = torch.full((3, 3, 1024), 77, dtype=torch.int16, device="cuda")
got = _np(ph.localize(const, scores=True))
assert (got["scores_f"] == 0).all() and (got["lags"] == -46).all()
print("variant ok", ph.batch_kernel())
"""

EMA12 = r"""
import oracle as O
if not __import__("os").path.exists(O.LIB_PATH):
    O.build()
from tdoa import synth
from tdoa.localizer import Localizer
from test_gpu_stream import run_pipeline, compare
loc = Localizer(sample_rate_hz=48000)
lut = loc.lut()
adc = synth.adc_stream(40, 512 * 40, 3, lut, loc.dims.S, 0x5EED0005).numpy()
recs, est, last = run_pipeline(loc, adc, 512)
exp = O.stream_run(adc, 1024, 48000, loc.dims.S, loc.window(), lut, max_trig=64)
assert exp["n_trig"].sum() > 200 and exp["gate"].sum() > 100
compare(recs, est, last, exp, loc.dims.P)
adc = synth.adc_stream(6, 512 * 24, 3, lut, loc.dims.S, 23).numpy()
recs, est, last = run_pipeline(loc, adc, 512, capture_len=2049)
compare(recs, est, last, O.stream_run(adc, 1024, 48000, loc.dims.S, loc.window(), lut), loc.dims.P)
print("variant ok streaming")
"""


XC3_OFF = r"""
import numpy as np
import oracle as O
if not __import__("os").path.exists(O.LIB_PATH):
    O.build()
from tdoa import synth
from tdoa.localizer import Localizer
loc3 = Localizer()
lut = loc3.lut().reshape(3, 101, 101)
for B, seed in ((4096, synth.SEEDS[2]), (33, 1033)):
    fr, _, _ = synth.adc_frames(B, 3, 1024, lut, 46, seed, device="cuda")
    got = {k: v.cpu().numpy() for k, v in loc3.localize(fr, scores=True).items()}
    exp = O.localize_batch(fr.cpu().numpy(), 46, loc3.window(), lut, threads=8)
    for k in ("lags", "gate", "cell", "max_L", "xy", "scores", "weighted"):
        assert np.array_equal(got[k], exp[k]), k
""" + EMA12.replace('print("variant ok streaming")', 'print("variant ok xc3 off")')


def _child(code, env):
    pre = f"import sys\nsys.path[:0] = {PATHS!r}\n"
    r = subprocess.run([sys.executable, "-c", pre + code], env=dict(os.environ, **env), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "variant ok" in r.stdout
    return r.stdout


def test_p1k_w64_vs_fp64_and_exhaustive_grid():
    _child(W64.format(golden=os.path.join(ROOT, "tests", "golden", "pipeline_cfg2.npz")), {"TDOA_P1K": "w64", "TDOA_LIB": AB_LIB})


def test_ema_waves_12_stream_bit_exact():
    _child(EMA12, {"TDOA_EMA_WAVES": "12"})


def test_direct_xc3_off_bit_exact():
    _child(XC3_OFF, {"TDOA_DIRECT_XC3": "0"})
