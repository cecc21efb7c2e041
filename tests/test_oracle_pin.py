"""Pin the CPU oracle (oracle/tdoa_oracle.c) before trusting it.

Pinned by the reference itself:
  - window tables vs window_function.h:5-70 and window.ipynb:73-202
    (sha256 recorded in tests/golden/window_pins.json at generation time,
    re-checked live when /root/reference exists);
  - ring / write_out / normalize / window / microphones vs the outputs of the
    reference's own buffer.c, rolling_buffer.c, microphones.c compiled
    unchanged (tests/golden/ref_components.npz, and live via oracle/_ref).
Not pinnable by reference output (correlations.c, vga_heatmap.h need Pico SDK
headers): checked against an independent numpy restatement and known-answer
injected delays.
"""
import ctypes as C
import hashlib
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, golden

REF = "/root/reference"


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.int32).tobytes()).hexdigest()


# ------------------------------------------------------------------ windows
def test_window_pins_recorded():
    pins = json.load(open(os.path.join(GOLDEN, "window_pins.json")))
    assert pins["window_function_h_1024_equals_dpss"]
    assert pins["notebook_output_2048_equals_dpss"]
    w = golden("window_q15.npz")
    assert _sha(w["n1024"]) == pins["window_function_h_1024_sha256"]
    assert _sha(w["n2048"]) == pins["notebook_output_2048_sha256"]


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent")
def test_window_live_against_reference_sources():
    txt = open(os.path.join(REF, "src/components/window_function.h")).read()
    ref = np.array([int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]+", txt[txt.index("{"):])])
    assert ref.size == 1024
    assert (ref == golden("window_q15.npz")["n1024"]).all()
    nb = json.load(open(os.path.join(REF, "window.ipynb")))
    out = "".join(nb["cells"][3]["outputs"][0]["text"])
    vals = np.array([int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]+", out)])
    assert (vals == golden("window_q15.npz")["n2048"]).all()


# ------------------------------------------------------- ring / buffer ops
def test_oracle_ring_matches_reference_fixture(oracle):
    g = golden("ref_components.npz")
    storage = np.zeros(1024, np.int16)
    r = oracle.orc_ring()
    lib = oracle.lib()
    lib.orc_ring_init.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    lib.orc_ring_push.argtypes = [C.c_void_p, C.c_int16]
    lib.orc_ring_incoming_power.argtypes = [C.c_void_p]
    lib.orc_ring_incoming_power.restype = C.c_int64
    lib.orc_ring_outgoing_power.argtypes = [C.c_void_p]
    lib.orc_ring_outgoing_power.restype = C.c_int64
    lib.orc_ring_write_out.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.orc_ring_init(C.byref(r), storage.ctypes.data_as(C.c_void_p), 1024)
    snaps = list(g["snap_index"])
    k = 0
    for i, v in enumerate(g["pushes"]):
        lib.orc_ring_push(C.byref(r), int(v))
        assert lib.orc_ring_incoming_power(C.byref(r)) == g["incoming_power"][i]
        assert lib.orc_ring_outgoing_power(C.byref(r)) == g["outgoing_power"][i]
        assert r.head == g["heads"][i]
        if i in snaps:
            out = np.zeros(1024, np.int16)
            pw = np.zeros(1, np.int64)
            lib.orc_ring_write_out(C.byref(r), out.ctypes.data_as(C.c_void_p),
                                   pw.ctypes.data_as(C.c_void_p))
            assert (out == g["write_out"][k]).all()
            assert pw[0] == g["write_out_power"][k]
            n = oracle.normalize(out)
            assert (n == g["normalized"][k]).all()
            w = oracle.window(n, golden("window_q15.npz")["n1024"])
            assert (w == g["windowed"][k]).all()
            k += 1
    assert k == len(snaps)


def test_oracle_buffer_ops_full_range_fixture(oracle):
    g = golden("ref_components.npz")
    win = golden("window_q15.npz")["n1024"]
    for row, n_ref, w_ref in zip(g["frames"], g["frames_normalized"], g["frames_windowed"]):
        assert (oracle.normalize(row) == n_ref).all()
        assert (oracle.window(row, win) == w_ref).all()


def test_oracle_microphones_fixture(oracle):
    g = golden("ref_components.npz")
    assert (oracle.microphones_ref() == g["mics"]).all()  # bit-exact float32


def test_oracle_vs_live_reference_components(oracle, ref_lib):
    rng = np.random.default_rng(7)
    win = golden("window_q15.npz")["n1024"]
    for trial in range(20):
        hi = 256 if trial % 2 == 0 else 32768
        lo = 0 if trial % 2 == 0 else -32768
        x = rng.integers(lo, hi, 1024).astype(np.int16)
        b = oracle.RefBuffer()
        C.memmove(b.buffer, x.ctypes.data, 2048)
        ref_lib.buffer_normalize_range(C.byref(b))
        assert (np.frombuffer(bytes(b.buffer), np.int16) == oracle.normalize(x)).all()
        C.memmove(b.buffer, x.ctypes.data, 2048)
        ref_lib.buffer_window(C.byref(b))
        assert (np.frombuffer(bytes(b.buffer), np.int16) == oracle.window(x, win)).all()
        rb = oracle.RefRollingBuffer()
        ref_lib.rolling_buffer_init(C.byref(rb))
        pushes = rng.integers(lo, hi, 1024 + int(rng.integers(0, 1500))).astype(np.int16)
        for v in pushes:
            ref_lib.rolling_buffer_push(C.byref(rb), int(v))
        ref_lib.rolling_buffer_write_out(C.byref(rb), C.byref(b))
        out, pw = oracle.dc_remove(pushes[-1024:])
        assert (np.frombuffer(bytes(b.buffer), np.int16) == out).all() and b.power == pw


# ------------------------------------------- unpinned stages: numpy restatement
def np_xcorr(a, b, S):
    a = a.astype(np.int64)
    b = b.astype(np.int64)
    n = a.size
    sc = np.zeros(2 * S + 1, np.int64)
    for s in range(-S, S + 1):
        if s >= 0:
            sc[s + S] = int(np.dot(a[: n - s], b[s:]))
        else:
            sc[s + S] = int(np.dot(a[-s:], b[: n + s]))
    best = int(np.argmax(sc)) - S  # argmax returns the first max
    return sc, best


def np_prior(sc, best):
    S = (sc.size - 1) // 2
    s = np.arange(-S, S + 1)
    d2 = (s - best) ** 2
    arg = (-d2).astype(np.float32) / np.float32(36.0)       # float division
    scale = np.exp(arg.astype(np.float64)).astype(np.float32)  # double exp, narrowed
    return (sc.astype(np.float32) * scale).astype(np.int64)  # float32 RN mult, trunc


def test_xcorr_prior_vs_numpy(oracle):
    rng = np.random.default_rng(11)
    win = golden("window_q15.npz")["n1024"]
    for trial in range(12):
        if trial < 6:
            a = rng.integers(-32767, 32512, 1024).astype(np.int16)
            b = rng.integers(-32767, 32512, 1024).astype(np.int16)
        else:
            base = rng.normal(0, 40, 1200)
            d = int(rng.integers(-40, 41))
            a = np.clip(np.round(128 + base[100:1124]), 0, 255).astype(np.int16)
            b = np.clip(np.round(128 + base[100 - d:1124 - d]), 0, 255).astype(np.int16)
            a = oracle.window(oracle.normalize(oracle.dc_remove(a)[0]), win)
            b = oracle.window(oracle.normalize(oracle.dc_remove(b)[0]), win)
        sc, best = oracle.xcorr(a, b, 46)
        sc2, best2 = np_xcorr(a, b, 46)
        assert (sc == sc2).all() and best == best2
        assert (oracle.prior(sc, best) == np_prior(sc, best)).all()


def test_xcorr_first_max_tie_break(oracle):
    a = np.zeros(1024, np.int16)
    b = np.zeros(1024, np.int16)
    sc, best = oracle.xcorr(a, b, 46)
    assert (sc == 0).all() and best == -46  # all equal -> most negative lag


def test_known_answer_injected_delay(oracle):
    """b delayed by d relative to a -> best = +d (correlations.c sign)."""
    win = golden("window_q15.npz")["n1024"]
    rng = np.random.default_rng(5)
    for d in (-30, -7, 0, 3, 19, 41):
        src = rng.normal(0, 40, 1200)
        a = np.clip(np.round(128 + src[100:1124]), 0, 255).astype(np.int16)
        b = np.clip(np.round(128 + src[100 - d:1124 - d]), 0, 255).astype(np.int16)
        pa = oracle.window(oracle.normalize(oracle.dc_remove(a)[0]), win)
        pb = oracle.window(oracle.normalize(oracle.dc_remove(b)[0]), win)
        assert oracle.xcorr(pa, pb, 46)[1] == d


def np_roundf(x):
    t = np.trunc(x)
    return (t + np.where(np.abs(x - t) >= np.float32(0.5), np.sign(x), 0)).astype(np.int64)


def test_lut_vs_numpy_float32(oracle):
    mics = oracle.microphones_ref()
    lut = oracle.build_lut(mics)
    f = np.float32
    y, x = np.meshgrid(np.arange(101), np.arange(101), indexing="ij")
    xm = (x - 50).astype(f) / f(24.0)
    ym = (50 - y).astype(f) / f(24.0)
    zm = np.full_like(xm, f(1.2))
    k = f(1.2) / np.sqrt(zm * zm + xm * xm + ym * ym)
    xm, ym, zm = xm * k, ym * k, zm * k
    d = [np.sqrt(zm * zm + (xm - mx) * (xm - mx) + (ym - my) * (ym - my)) for mx, my in mics]
    p = 0
    for i in range(3):
        for j in range(i + 1, 3):
            s = np_roundf((d[j] - d[i]) / f(343.0) * f(50000.0))
            s = np.clip(s, -46, 46) + 46
            assert (s.astype(np.uint8) == lut[p]).all()
            p += 1


def test_grid_solve_vs_numpy(oracle):
    mics = oracle.microphones_ref()
    lut = oracle.build_lut(mics)
    rng = np.random.default_rng(3)
    for _ in range(10):
        w = rng.integers(-(1 << 38), 1 << 38, (3, 93)).astype(np.int64)
        L = sum(w[p][lut[p].reshape(-1)] for p in range(3))
        mL, cell = oracle.grid_solve(w, lut)
        assert mL == L.max() and cell == int(np.argmax(L))


# ------------------------------------------------------------ regression
def test_oracle_pipeline_fixture(oracle):
    g = golden("pipeline_cfg2.npz")
    win = golden("window_q15.npz")["n1024"]
    res = oracle.localize_batch(g["frames"], 46, win, g["lut"], threads=2)
    for k in ("lags", "gate", "cell", "max_L", "xy", "scores", "weighted"):
        assert (res[k] == g[k]).all(), k


def test_oracle_ema_fixture(oracle):
    g = golden("ema_sequence.npz")
    est = np.zeros(93, np.int64)
    last = 0
    for i in range(g["fresh"].shape[0]):
        d = oracle.decay(int(g["t_us"][i]), last)
        assert np.float32(d) == g["decay"][i]
        est, b = oracle.average(est, g["fresh"][i], d)
        last = int(g["t_us"][i])
        assert (est == g["est"][i]).all() and b == g["best"][i]


def test_ema_vs_numpy(oracle):
    rng = np.random.default_rng(9)
    est = rng.integers(-(1 << 40), 1 << 40, 93).astype(np.int64)
    fresh = rng.integers(-(1 << 40), 1 << 40, 93).astype(np.int64)
    dec = np.float32(oracle.decay(1_700_000, 1_000_000))
    exp = (est.astype(np.float32) + (fresh - est).astype(np.float32) * dec).astype(np.int64)
    got, best = oracle.average(est, fresh, float(dec))
    assert (got == exp).all() and best == int(np.argmax(exp)) - 46


# ------------------------------------------------------- GCC-PHAT oracle
def test_gcc_phat_prep_equals_c_oracle(oracle):
    import gcc_phat_oracle as G
    g = golden("pipeline_cfg2.npz")
    win = golden("window_q15.npz")["n1024"]
    fr = g["frames"][:20]
    got = G.prep(fr, win)
    for b in range(fr.shape[0]):
        for m in range(3):
            exp = oracle.window(oracle.normalize(oracle.dc_remove(fr[b, m])[0]), win)
            assert (got[b, m] == exp).all()


def test_gcc_phat_oracle_recovers_injected_delays():
    import gcc_phat_oracle as G
    g = golden("pipeline_cfg2.npz")
    win = golden("window_q15.npz")["n1024"]
    res = G.gcc_phat_batch(g["frames"][:64], 46, win, g["lut"])
    # ADC-like frames: the (0,m) pairs peak at the injected delays, like DIRECT
    agree = (res["lags"][:, :2] == g["tau"][:, 1:]).mean()
    assert agree > 0.95
    assert (res["lags"] == g["lags"][:64]).mean() > 0.9
