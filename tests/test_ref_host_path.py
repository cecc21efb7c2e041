"""libtdoa's host-CPU path for the reference's per-frame symbols
(tdoa_ref_set_device(-1), csrc/tdoa_host_path.cpp; BASELINE config 1, "on host
CPU, no GPU").  It makes no HIP call, so it runs in the CPU suite: bit-exact
against the reference's own compiled ring/buffer code (golden fixture), the
oracle's correlations.c restatement, and the int16 wrap / extreme cases.

This is the product's own code (not oracle/): the oracle is only the checker."""
import ctypes as C

import numpy as np
import pytest

import tdoa
from conftest import golden
from ref_symbols_check import check_reference_symbols
from tdoa import _lib


@pytest.fixture()
def host_lib():
    L = tdoa.load()
    assert L.tdoa_ref_set_device(-1) == 0
    yield L
    assert L.tdoa_ref_set_device(0) == 0


def test_reference_symbols_host_path(host_lib, oracle):
    check_reference_symbols(host_lib, oracle)


def _buf(x):
    b = _lib.Buffer()
    C.memmove(b.buffer, np.ascontiguousarray(x, np.int16).ctypes.data, 2048)
    return b


def _arr(b):
    return np.frombuffer(bytes(b.buffer), np.int16).copy()


@pytest.mark.parametrize("kind", ["full_range", "adc", "extreme", "zeros"])
def test_frame_path_bit_exact(host_lib, oracle, kind):
    """write_out (random head) -> normalize -> window -> correlations_init for
    two rings, against the oracle, on wrap-heavy full-range samples, ADC-like
    bytes, the extreme products (|x| = 32767 after the window) and all-zero
    frames (every score ties: the first lag, -46)."""
    L = host_lib
    rng = np.random.default_rng({"full_range": 1, "adc": 2, "extreme": 3, "zeros": 4}[kind])
    win = golden("window_q15.npz")["n1024"]
    for it in range(8):
        pre = []
        for m in range(2):
            if kind == "full_range":
                ring = rng.integers(-32768, 32768, 1024).astype(np.int16)
            elif kind == "adc":
                ring = rng.integers(0, 256, 1024).astype(np.int16)
            elif kind == "zeros":
                ring = np.zeros(1024, np.int16)
            else:
                ring = None
            head = int(rng.integers(0, 1024))
            if ring is None:  # prepared buffers straight into correlations_init
                x = np.where(rng.integers(0, 2, 1024) > 0, 32767, -32767).astype(np.int16)
                pre.append(x if m == 0 else (x if it % 2 else -x))
                continue
            rb = _lib.RollingBuffer()
            rb.head, rb.is_full = head, True
            C.memmove(rb.buffer, ring.ctypes.data, 2048)
            b = _lib.Buffer()
            L.rolling_buffer_write_out(C.byref(rb), C.byref(b))
            lin = np.concatenate([ring[head:], ring[:head]])
            dc, pw = oracle.dc_remove(lin)
            assert (_arr(b) == dc).all() and b.power == pw
            L.buffer_normalize_range(C.byref(b))
            assert (_arr(b) == oracle.normalize(dc)).all()
            L.buffer_window(C.byref(b))
            w = oracle.window(oracle.normalize(dc), win)
            assert (_arr(b) == w).all()
            pre.append(w)
        corr = _lib.Correlations()
        L.correlations_init(C.byref(corr), C.byref(_buf(pre[0])), C.byref(_buf(pre[1])))
        sc, best = oracle.xcorr(pre[0], pre[1], 46)
        assert corr.best_shift == best
        assert (np.frombuffer(bytes(corr.correlations), np.int64) == oracle.prior(sc, best)).all()
        if kind == "zeros":
            assert best == -46


def test_average_sequence(host_lib, oracle):
    """correlations_average's float EMA (compound-assignment rounding, no FMA)
    and re-argmax over a clocked sequence, against the oracle."""
    L = host_lib
    clock = {"t": 1_000_000}

    @_lib.CLOCK_FN
    def now():
        clock["t"] += 13_337
        return clock["t"]

    L.tdoa_ref_set_clock(now)
    try:
        rng = np.random.default_rng(9)
        est = _lib.Correlations()
        ref = np.zeros(93, np.int64)
        last = 0
        for _ in range(20):
            fresh = _lib.Correlations()
            new = rng.integers(-(1 << 40), 1 << 40, 93)
            C.memmove(fresh.correlations, np.ascontiguousarray(new, np.int64).ctypes.data, 93 * 8)
            L.correlations_average(C.byref(est), C.byref(fresh))
            ref, b = oracle.average(ref, new, oracle.decay(est.last_update, last))
            last = est.last_update
            assert (np.frombuffer(bytes(est.correlations), np.int64) == ref).all()
            assert est.best_shift == b
    finally:
        L.tdoa_ref_set_clock(_lib.CLOCK_FN())


def test_gpu_device_switch_rules():
    """-1 selects the host path at any time; 0 restores the default device."""
    L = tdoa.load()
    assert L.tdoa_ref_set_device(-1) == 0
    assert L.tdoa_ref_set_device(-7) == 0  # any negative: the host path
    assert L.tdoa_ref_set_device(0) == 0


@pytest.mark.parametrize("case", ["runs", "all_min", "alternating", "random_with_min"])
def test_correlations_init_int16_min(host_lib, oracle, case):
    """correlations_init takes any buffer_t, not only windowed ones:
    adjacent INT16_MIN samples in both buffers make a vpmaddwd pair sum
    (-32768)^2 * 2 = 2^31, which wraps in an int32 lane; the reference
    multiplies in int32 and sums in int64 (correlations.c:9-18).  Bit-exact
    against the oracle for raw buffers with runs of -32768."""
    L = host_lib
    rng = np.random.default_rng(0x3276)
    n = 1024
    if case == "runs":
        a = rng.integers(-32768, 32768, n).astype(np.int16)
        b = rng.integers(-32768, 32768, n).astype(np.int16)
        for lo in (0, 100, 511, 1000):
            a[lo:lo + 24] = -32768
            b[lo + 3:lo + 30] = -32768
    elif case == "all_min":
        a = np.full(n, -32768, np.int16)
        b = np.full(n, -32768, np.int16)
    elif case == "alternating":
        a = np.where(np.arange(n) % 4 < 2, -32768, 32767).astype(np.int16)
        b = a.copy()
    else:
        a = rng.choice(np.array([-32768, -32767, 0, 32767], np.int16), n)
        b = rng.choice(np.array([-32768, 32767], np.int16), n)
    for x, y in ((a, b), (b, a), (a, a)):
        corr = _lib.Correlations()
        L.correlations_init(C.byref(corr), C.byref(_buf(x)), C.byref(_buf(y)))
        sc, best = oracle.xcorr(x, y, 46)
        assert corr.best_shift == best, case
        assert (np.frombuffer(bytes(corr.correlations), np.int64) == oracle.prior(sc, best)).all(), case
