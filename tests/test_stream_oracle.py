"""Streaming loop (sample_compute.h:53-146) on the CPU: the oracle's
orc_stream_run against the REFERENCE's own rolling_buffer.c / buffer.c
(tests/golden/stream_trace.npz, made by tools/gen_golden.py through
oracle/_ref; live when _ref is built here), and the hop decomposition the GPU
trigger kernel uses (prefix sums over [pos+1-N, pos+H), first firing sample at
least N after the last trigger) against the sequential ring semantics."""
import ctypes as C

import numpy as np
import pytest

from conftest import golden


def _mics(oracle):
    m = np.zeros(6, np.float32)
    oracle.lib().orc_microphones_ref(m.ctypes.data_as(C.c_void_p))
    return m.reshape(3, 2)


def _win():
    return golden("window_q15.npz")["n1024"]


def test_oracle_triggers_match_reference_trace(oracle):
    g = golden("stream_trace.npz")
    r = oracle.stream_run(g["adc"], 1024, int(g["fs"]), int(g["max_shift"]), _win(), g["lut"],
                          max_trig=32)
    ends = [(s, int(r["end"][s, i])) for s in range(len(r["n_trig"]))
            for i in range(r["n_trig"][s])]
    assert ends == [tuple(x) for x in g["ref_ends"]]
    for k in ("n_trig", "end", "lags", "gate", "ema_best", "cell", "max_L", "est", "last"):
        assert (r[k] == g["orc_" + k]).all(), k


def test_oracle_prepared_frames_match_reference_trace(oracle):
    g = golden("stream_trace.npz")
    adc = g["adc"]
    for (s, end), ref in zip(g["ref_ends"], g["ref_prepared"]):
        raw = adc[s, end - 1024:end].T.astype(np.int16)  # [3][1024]
        for m in range(3):
            x, _ = oracle.dc_remove(raw[m])
            x = oracle.normalize(x)
            x = oracle.window(x, _win())
            assert (x == ref[m]).all()


def _ref_triggers(R, oracle, adc):
    thr = 2 << 18
    out = []
    for s in range(adc.shape[0]):
        rb = [oracle.RefRollingBuffer() for _ in range(adc.shape[2])]
        for r in rb:
            R.rolling_buffer_init(C.byref(r))
        for t in range(adc.shape[1]):
            for m, r in enumerate(rb):
                R.rolling_buffer_push(C.byref(r), int(adc[s, t, m]))
            if not all(r.is_full for r in rb):
                continue
            po = sum(R.rolling_buffer_get_outgoing_power(C.byref(r)) for r in rb)
            pi = sum(R.rolling_buffer_get_incoming_power(C.byref(r)) for r in rb)
            if po > thr + pi:
                out.append((s, t + 1))
                for r in rb:
                    R.rolling_buffer_init(C.byref(r))
    return out


def test_oracle_triggers_vs_live_reference(oracle, ref_lib):
    from tdoa import synth
    lut = oracle.build_lut(_mics(oracle), fs=50000, max_shift=46)
    adc = synth.adc_stream(2, 9000, 3, lut, 46, 321, burst_len=500, gap=(1100, 2600)).numpy()
    r = oracle.stream_run(adc, 1024, 50000, 46, _win(), lut)
    ends = [(s, int(r["end"][s, i])) for s in range(2) for i in range(r["n_trig"][s])]
    assert ends == _ref_triggers(ref_lib, oracle, adc)
    assert len(ends) >= 6


def hop_triggers(adc, N, H):
    """The GPU trigger kernel's algorithm (tdoa_stream.hip) in numpy."""
    S, T, M = adc.shape
    hb = int(np.log2(N)) - 1
    thr = 2 << (2 * hb)
    out = []
    for s in range(S):
        x = adc[s].astype(np.int64)  # [T][M]
        ring_start, pos = 0, 0
        while pos + H <= T:
            base = pos + 1 - N
            L = N + H - 1
            idx = np.arange(base, base + L)
            w = np.where(idx[:, None] >= 0, x[np.clip(idx, 0, None)], 0)  # [L][M]
            Q1 = np.concatenate([np.zeros((1, M), np.int64), np.cumsum(w, 0)])
            Q2 = np.concatenate([np.zeros((1, M), np.int64), np.cumsum(w * w, 0)])
            a = np.arange(H)
            h = N // 2
            so1, so2 = Q1[a + h] - Q1[a], Q2[a + h] - Q2[a]
            si1, si2 = Q1[a + N] - Q1[a + h], Q2[a + N] - Q2[a + h]
            po = ((so2 << hb) - so1 * so1).sum(1)
            pi = ((si2 << hb) - si1 * si1).sum(1)
            ok = (a >= ring_start + N - pos - 1) & (po > thr + pi)
            if ok.any():
                e = pos + 1 + int(np.argmax(ok))
                out.append((s, e))
                ring_start = e
            pos += H
    return out


@pytest.mark.parametrize("H", [512, 256, 1024, 300])
def test_hop_decomposition_equals_sequential_rings(oracle, H):
    from tdoa import synth
    lut = oracle.build_lut(_mics(oracle), fs=48000, max_shift=44)
    adc = synth.adc_stream(4, 14000, 3, lut, 44, 99 + H).numpy()
    T = (14000 // H) * H
    r = oracle.stream_run(adc[:, :T], 1024, 48000, 44, _win(), lut)
    ends = [(s, int(r["end"][s, i])) for s in range(4) for i in range(r["n_trig"][s])]
    assert ends == hop_triggers(adc[:, :T], 1024, H)
    assert len(ends) >= 12
