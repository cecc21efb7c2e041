"""The reference-named per-frame symbols (include/tdoa_reference_abi.h) checked
against the reference's own compiled components (tests/golden/ref_components.npz:
rolling_buffer.c / buffer.c outputs) and the oracle (correlations.c:4-63), on
whichever path libtdoa currently routes them to (GPU, or the host-CPU path of
tdoa_ref_set_device(-1)).  Shared by test_gpu_parity.py and test_ref_host_path.py."""
import ctypes as C

import numpy as np

from conftest import golden
from tdoa import _lib


def check_reference_symbols(L, oracle):
    g = golden("ref_components.npz")
    win = golden("window_q15.npz")["n1024"]
    # replay the ring, then write_out / normalize / window on the routed path
    rb = _lib.RollingBuffer()
    L.rolling_buffer_init(C.byref(rb))
    k = 0
    for i, v in enumerate(g["pushes"]):
        L.rolling_buffer_push(C.byref(rb), int(v))
        if i in list(g["snap_index"]):
            b = _lib.Buffer()
            L.rolling_buffer_write_out(C.byref(rb), C.byref(b))
            assert (np.frombuffer(bytes(b.buffer), np.int16) == g["write_out"][k]).all()
            assert b.power == g["write_out_power"][k]
            L.buffer_normalize_range(C.byref(b))
            assert (np.frombuffer(bytes(b.buffer), np.int16) == g["normalized"][k]).all()
            L.buffer_window(C.byref(b))
            assert (np.frombuffer(bytes(b.buffer), np.int16) == g["windowed"][k]).all()
            # the fused write_out records its normalised / windowed output; a
            # buffer changed after write_out must take its own launch
            b2 = _lib.Buffer()
            L.rolling_buffer_write_out(C.byref(rb), C.byref(b2))
            x = np.frombuffer(bytes(b2.buffer), np.int16).copy()
            x[k % 1024] ^= 0x35
            C.memmove(b2.buffer, x.ctypes.data, 2048)
            L.buffer_normalize_range(C.byref(b2))
            y = oracle.normalize(x)
            assert (np.frombuffer(bytes(b2.buffer), np.int16) == y).all()
            L.buffer_window(C.byref(b2))
            assert (np.frombuffer(bytes(b2.buffer), np.int16) == oracle.window(y, win)).all()
            k += 1
    # correlations_init / correlations_average with a deterministic clock
    clock = {"t": 5_000_000}

    @_lib.CLOCK_FN
    def now():
        clock["t"] += 20_000
        return clock["t"]

    L.tdoa_ref_set_clock(now)
    rng = np.random.default_rng(8)
    est = _lib.Correlations()
    est_ref = np.zeros(93, np.int64)
    last = 0
    for it in range(6):
        a = oracle.window(oracle.normalize(oracle.dc_remove(rng.integers(0, 256, 1024))[0]), win)
        d = int(rng.integers(-30, 31))
        bsig = np.roll(a, d)
        ba, bb = _lib.Buffer(), _lib.Buffer()
        C.memmove(ba.buffer, a.ctypes.data, 2048)
        C.memmove(bb.buffer, np.ascontiguousarray(bsig).ctypes.data, 2048)
        new = _lib.Correlations()
        L.correlations_init(C.byref(new), C.byref(ba), C.byref(bb))
        sc, best = oracle.xcorr(a, bsig, 46)
        assert new.best_shift == best
        assert (np.frombuffer(bytes(new.correlations), np.int64) == oracle.prior(sc, best)).all()
        L.correlations_average(C.byref(est), C.byref(new))
        dec = oracle.decay(est.last_update, last)
        est_ref, b = oracle.average(est_ref, oracle.prior(sc, best), dec)
        last = est.last_update
        assert (np.frombuffer(bytes(est.correlations), np.int64) == est_ref).all()
        assert est.best_shift == b
    L.tdoa_ref_set_clock(_lib.CLOCK_FN())
