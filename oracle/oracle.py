"""ctypes wrapper over the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It loads ``oracle/liboracle.so`` (the clean-room restatement in
``tdoa_oracle.c``) and, when present, ``oracle/_ref/libref_components.so``
(the reference's own buffer.c / rolling_buffer.c / microphones.c compiled
unchanged).  See tdoa_oracle.h for what is pinned and what is not.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# TDOA_ORACLE_LIB: another build of the same restatement (the sanitizer build,
# tests/test_sanitizers.py)
LIB_PATH = os.environ.get("TDOA_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libref_components.so")

_lib = None


def build(quiet: bool = True) -> None:
    """Compile liboracle.so (and _ref when /root/reference exists)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.orc_dc_remove.argtypes = [P, P, C.c_int, P]
        L.orc_normalize.argtypes = [P, C.c_int]
        L.orc_window.argtypes = [P, P, C.c_int]
        L.orc_xcorr.argtypes = [P, P, C.c_int, C.c_int, P, P]
        L.orc_prior_scale.argtypes = [C.c_int]
        L.orc_prior_scale.restype = C.c_float
        L.orc_prior.argtypes = [P, C.c_int, C.c_int]
        L.orc_decay.argtypes = [C.c_uint64, C.c_uint64]
        L.orc_decay.restype = C.c_float
        L.orc_average.argtypes = [P, P, C.c_int, C.c_float, P]
        L.orc_microphones_ref.argtypes = [P]
        L.orc_build_lut.argtypes = [P, C.c_int, C.c_int, C.c_int, C.c_float,
                                    C.c_float, C.c_float, C.c_int, C.c_int, P]
        L.orc_grid_solve.argtypes = [P, C.c_int, C.c_int, P, C.c_int, P, P]
        L.orc_localize_batch.argtypes = [P, C.c_int64, C.c_int, C.c_int, C.c_int,
                                         P, P, C.c_int, C.c_int, C.c_float,
                                         C.c_int, C.c_int, P]
        L.orc_localize_batch.restype = C.c_int
        L.orc_stream_run.argtypes = [P, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int,
                                     C.c_int, P, P, C.c_int, C.c_int, C.c_int, C.c_int, P]
        L.orc_stream_run.restype = C.c_int
        L.orc_heatmap.argtypes = [P, C.c_int, C.c_int, P, C.c_int, P]
        L.orc_ls_refine.argtypes = [P, P, C.c_int, C.c_int, P, C.c_int32, C.c_int, C.c_int,
                                    C.c_double, C.c_double, C.c_double, C.c_double, C.c_int,
                                    P, P, P]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"], "oracle needs C-contiguous arrays"
    return a.ctypes.data_as(C.c_void_p)


class orc_ring(C.Structure):
    """struct orc_ring (tdoa_oracle.h)."""
    _fields_ = [("head", C.c_int), ("incoming_power", C.c_int64),
                ("incoming_total", C.c_int64), ("outgoing_power", C.c_int64),
                ("outgoing_total", C.c_int64), ("is_full", C.c_int), ("n", C.c_int),
                ("buf", C.c_void_p)]


class _BatchOut(C.Structure):
    _fields_ = [("scores", C.c_void_p), ("weighted", C.c_void_p),
                ("lags", C.c_void_p), ("gate", C.c_void_p),
                ("cell", C.c_void_p), ("max_L", C.c_void_p), ("xy", C.c_void_p)]


class _StreamOut(C.Structure):
    _fields_ = [("n_trig", C.c_void_p), ("end", C.c_void_p), ("lags", C.c_void_p),
                ("gate", C.c_void_p), ("ema_best", C.c_void_p), ("cell", C.c_void_p),
                ("max_L", C.c_void_p), ("est", C.c_void_p), ("last", C.c_void_p)]


def stream_run(adc: np.ndarray, N: int, fs: int, max_shift: int, win: np.ndarray,
               lut: np.ndarray | None, max_trig: int = 64, half_w=50, half_h=50, threads=0):
    """sample_compute.h:53-146 over S streams of u8 ADC bytes [S][T][M].
    Returns per-stream lists of trigger records plus the final EMA state."""
    a = np.ascontiguousarray(adc, dtype=np.uint8)
    S, T, M = a.shape
    P, K = M * (M - 1) // 2, 2 * max_shift + 1
    w = np.ascontiguousarray(win, dtype=np.int32)
    r = {"n_trig": np.zeros(S, np.int32), "end": np.zeros((S, max_trig), np.int64),
         "lags": np.zeros((S, max_trig, P), np.int32), "gate": np.zeros((S, max_trig), np.uint8),
         "ema_best": np.zeros((S, max_trig, P), np.int32),
         "cell": np.zeros((S, max_trig), np.int32), "max_L": np.zeros((S, max_trig), np.int64),
         "est": np.zeros((S, P, K), np.int64), "last": np.zeros(S, np.uint64)}
    o = _StreamOut(*[_p(r[k]).value for k in ("n_trig", "end", "lags", "gate", "ema_best",
                                                "cell", "max_L", "est", "last")])
    lut_c = np.ascontiguousarray(lut, dtype=np.uint8) if lut is not None else None
    rc = lib().orc_stream_run(_p(a), S, T, M, N, fs, max_shift, _p(w),
                              _p(lut_c) if lut_c is not None else None, half_w, half_h,
                              max_trig, int(threads), C.byref(o))
    if rc != 0:
        raise ValueError("orc_stream_run rejected the shape")
    return r


def heatmap(weighted: np.ndarray, lut: np.ndarray) -> np.ndarray:
    """vga_heatmap.h:97-130 classes for one frame: weighted int64 [P][K], lut [P][G]."""
    w = np.ascontiguousarray(weighted, dtype=np.int64)
    P, K = w.shape
    lt = np.ascontiguousarray(lut, dtype=np.uint8).reshape(P, -1)
    out = np.zeros(lt.shape[1], np.uint8)
    lib().orc_heatmap(_p(w), P, K, _p(lt), lt.shape[1], _p(out))
    return out


def ls_refine(scores, best, mic_xy, cell, half_w=50, half_h=50, grid_scale=24.0,
              height=1.2, fs=50000.0, c=343.0, iters=10):
    """a15 least squares for B frames: scores [B][P][K] raw (any numeric dtype),
    best [B][P], cell [B] -> (uv [B][2] float64, rms [B])."""
    sc = np.ascontiguousarray(scores, dtype=np.float64)
    B, P, K = sc.shape
    M = int(round((1 + np.sqrt(1 + 8 * P)) / 2))
    bst = np.ascontiguousarray(best, dtype=np.int32)
    mic = np.ascontiguousarray(mic_xy, dtype=np.float32).reshape(-1)
    uv = np.zeros((B, 2), np.float64)
    rms = np.zeros(B, np.float64)
    u, v, r = C.c_double(), C.c_double(), C.c_double()
    for f in range(B):
        lib().orc_ls_refine(_p(sc[f]), _p(bst[f]), M, K, _p(mic), int(cell[f]), half_w, half_h,
                            grid_scale, height, fs, c, iters, C.byref(u), C.byref(v), C.byref(r))
        uv[f] = (u.value, v.value)
        rms[f] = r.value
    return uv, rms


# ---------------------------------------------------------------- stages
def dc_remove(x: np.ndarray):
    x = np.ascontiguousarray(x, dtype=np.int16)
    out = np.empty_like(x)
    pw = np.zeros(1, np.int64)
    lib().orc_dc_remove(_p(x), _p(out), x.size, _p(pw))
    return out, int(pw[0])


def normalize(x: np.ndarray) -> np.ndarray:
    x = np.array(x, dtype=np.int16, copy=True, order="C")
    lib().orc_normalize(_p(x), x.size)
    return x


def window(x: np.ndarray, w: np.ndarray) -> np.ndarray:
    x = np.array(x, dtype=np.int16, copy=True, order="C")
    w = np.ascontiguousarray(w, dtype=np.int32)
    assert w.size == x.size
    lib().orc_window(_p(x), _p(w), x.size)
    return x


def xcorr(a: np.ndarray, b: np.ndarray, max_shift: int):
    a = np.ascontiguousarray(a, dtype=np.int16)
    b = np.ascontiguousarray(b, dtype=np.int16)
    sc = np.zeros(2 * max_shift + 1, np.int64)
    best = np.zeros(1, np.int32)
    lib().orc_xcorr(_p(a), _p(b), a.size, max_shift, _p(sc), _p(best))
    return sc, int(best[0])


def prior_scale(d2: int) -> float:
    return float(lib().orc_prior_scale(int(d2)))


def prior(scores: np.ndarray, best: int) -> np.ndarray:
    s = np.array(scores, dtype=np.int64, copy=True)
    lib().orc_prior(_p(s), (s.size - 1) // 2, int(best))
    return s


def decay(now_us: int, last_us: int) -> float:
    return float(lib().orc_decay(int(now_us), int(last_us)))


def average(est: np.ndarray, fresh: np.ndarray, dec: float):
    e = np.array(est, dtype=np.int64, copy=True)
    f = np.ascontiguousarray(fresh, dtype=np.int64)
    best = np.zeros(1, np.int32)
    lib().orc_average(_p(e), _p(f), e.size, C.c_float(dec), _p(best))
    return e, int(best[0])


def microphones_ref() -> np.ndarray:
    xy = np.zeros(6, np.float32)
    lib().orc_microphones_ref(_p(xy))
    return xy.reshape(3, 2)


def build_lut(mic_xy, half_w=50, half_h=50, grid_scale=24.0, height=1.2,
              speed=343.0, fs=50000, max_shift=46) -> np.ndarray:
    mic = np.ascontiguousarray(mic_xy, dtype=np.float32).reshape(-1, 2)
    M = mic.shape[0]
    P = M * (M - 1) // 2
    H, W = 2 * half_h + 1, 2 * half_w + 1
    lut = np.zeros((P, H, W), np.uint8)
    lib().orc_build_lut(_p(mic), M, half_w, half_h, grid_scale, height, speed,
                        fs, max_shift, _p(lut))
    return lut


def grid_solve(weighted: np.ndarray, lut: np.ndarray):
    w = np.ascontiguousarray(weighted, dtype=np.int64)
    P, K = w.shape
    l2 = np.ascontiguousarray(lut.reshape(P, -1), dtype=np.uint8)
    mL = np.zeros(1, np.int64)
    cell = np.zeros(1, np.int32)
    lib().orc_grid_solve(_p(w), P, K, _p(l2), l2.shape[1], _p(mL), _p(cell))
    return int(mL[0]), int(cell[0])


def localize_batch(frames: np.ndarray, max_shift: int, win: np.ndarray,
                   lut: np.ndarray | None, half_w=50, half_h=50,
                   grid_scale=24.0, threads=0, want_scores=True):
    """Stateless batch pipeline; frames int16 [B][M][N] raw (pre-DC)."""
    fr = np.ascontiguousarray(frames, dtype=np.int16)
    B, M, N = fr.shape
    P, K = M * (M - 1) // 2, 2 * max_shift + 1
    w = np.ascontiguousarray(win, dtype=np.int32)
    assert w.size == N
    res = {
        "lags": np.zeros((B, P), np.int32),
        "gate": np.zeros(B, np.uint8),
        "cell": np.zeros(B, np.int32),
        "max_L": np.zeros(B, np.int64),
        "xy": np.zeros((B, 2), np.float32),
    }
    if want_scores:
        res["scores"] = np.zeros((B, P, K), np.int64)
        res["weighted"] = np.zeros((B, P, K), np.int64)
    o = _BatchOut(
        _p(res["scores"]).value if want_scores else None,
        _p(res["weighted"]).value if want_scores else None,
        _p(res["lags"]).value, _p(res["gate"]).value, _p(res["cell"]).value,
        _p(res["max_L"]).value, _p(res["xy"]).value)
    do_grid = lut is not None
    lut_c = np.ascontiguousarray(lut, dtype=np.uint8) if do_grid else np.zeros(1, np.uint8)
    rc = lib().orc_localize_batch(_p(fr), B, M, N, max_shift, _p(w), _p(lut_c),
                                  half_w, half_h, grid_scale, int(do_grid),
                                  int(threads), C.byref(o))
    if rc != 0:
        raise ValueError("orc_localize_batch rejected the shape")
    return res


# ------------------------------------------------------- reference (_ref) TUs
_ref = None


def ref_available() -> bool:
    return os.path.exists(REF_PATH)


class RefRollingBuffer(C.Structure):
    """struct rolling_buffer_t, rolling_buffer.h:13-25 (x86-64 ABI layout)."""
    _fields_ = [("head", C.c_int), ("incoming_power", C.c_int64),
                ("incoming_total", C.c_int64), ("outgoing_power", C.c_int64),
                ("outgoing_total", C.c_int64), ("is_full", C.c_bool),
                ("buffer", C.c_int16 * 1024)]


class RefBuffer(C.Structure):
    """struct buffer_t, buffer.h:8-12."""
    _fields_ = [("buffer", C.c_int16 * 1024), ("power", C.c_int64)]


class RefPoint(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float)]


def ref():
    """The reference's own component TUs (only where oracle/_ref was built)."""
    global _ref
    if _ref is None:
        if not ref_available():
            return None
        R = C.CDLL(REF_PATH)
        R.rolling_buffer_init.argtypes = [C.POINTER(RefRollingBuffer)]
        R.rolling_buffer_push.argtypes = [C.POINTER(RefRollingBuffer), C.c_int16]
        R.rolling_buffer_write_out.argtypes = [C.POINTER(RefRollingBuffer), C.POINTER(RefBuffer)]
        R.rolling_buffer_get_incoming_power.argtypes = [C.POINTER(RefRollingBuffer)]
        R.rolling_buffer_get_incoming_power.restype = C.c_int64
        R.rolling_buffer_get_outgoing_power.argtypes = [C.POINTER(RefRollingBuffer)]
        R.rolling_buffer_get_outgoing_power.restype = C.c_int64
        R.buffer_window.argtypes = [C.POINTER(RefBuffer)]
        R.buffer_normalize_range.argtypes = [C.POINTER(RefBuffer)]
        R.microphones_init.argtypes = []
        _ref = R
    return _ref
