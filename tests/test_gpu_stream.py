"""Streaming pipeline (tdoa_stream_*, BASELINE config 5) against the oracle's
sample-by-sample restatement of sample_compute.h:53-146 (itself pinned to the
reference's rolling_buffer.c / buffer.c in test_stream_oracle.py).
Everything is integer or reference-rounded float: exact equality."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402
from tdoa.stream import StreamPipeline  # noqa: E402


def run_pipeline(loc, adc, hop, use_graph=True, capture_len=None):
    """Feed all full hops; returns per-stream record lists and the final state."""
    S, T, M = adc.shape
    steps = T // hop
    if capture_len is None:
        cap = torch.from_numpy(adc).cuda()
    else:  # producer-fed capture ring
        # + 4 spare bytes: an unaligned last ring may be read word-wise
        flat = torch.zeros(S * capture_len * M + 4, dtype=torch.uint8, device="cuda")
        cap = flat[:S * capture_len * M].view(S, capture_len, M)
        src = torch.from_numpy(adc).cuda()
    pipe = StreamPipeline(loc, cap, hop=hop, use_graph=use_graph)
    recs = {s: [] for s in range(S)}
    for h in range(steps):
        if capture_len is not None:
            with torch.cuda.stream(pipe.stream):
                t0 = h * hop
                idx = torch.arange(t0, t0 + hop, device="cuda") % capture_len
                cap[:, idx] = src[:, t0:t0 + hop]
        pipe.step()
        r = pipe.records()
        for i, s in enumerate(r["stream_id"]):
            recs[int(s)].append({k: v[i] for k, v in r.items()})
    pos, est, last = pipe.state()
    assert pos == steps * hop
    pipe.close()
    return recs, est, last


def compare(recs, est, last, exp, lut_P):
    for s, lst in recs.items():
        n = exp["n_trig"][s]
        assert len(lst) == n, (s, len(lst), n)
        for i, r in enumerate(lst):
            assert r["end"] == exp["end"][s, i]
            assert (r["lags"] == exp["lags"][s, i]).all()
            assert r["gate"] == exp["gate"][s, i]
            if r["gate"]:
                assert (r["ema_best"] == exp["ema_best"][s, i]).all()
                assert r["cell"] == exp["cell"][s, i]
                assert r["max_L"] == exp["max_L"][s, i]
            else:
                assert r["cell"] == -1
    assert (est == exp["est"]).all()
    assert (last == exp["last"]).all()


@pytest.fixture(scope="module")
def loc48():
    return Localizer(sample_rate_hz=48000)


def test_stream_vs_oracle(loc48, oracle):
    S_lag = loc48.dims.S
    lut = loc48.lut()
    adc = synth.adc_stream(40, 512 * 40, 3, lut, S_lag, 0x5EED0005).numpy()
    recs, est, last = run_pipeline(loc48, adc, 512)
    exp = oracle.stream_run(adc, 1024, 48000, S_lag, loc48.window(), lut, max_trig=64)
    assert exp["n_trig"].sum() > 200 and exp["gate"].sum() > 100
    compare(recs, est, last, exp, loc48.dims.P)


def test_stream_graph_equals_eager(loc48):
    lut = loc48.lut()
    adc = synth.adc_stream(8, 512 * 16, 3, lut, loc48.dims.S, 17).numpy()
    a = run_pipeline(loc48, adc, 512, use_graph=True)
    b = run_pipeline(loc48, adc, 512, use_graph=False)
    assert (a[1] == b[1]).all() and (a[2] == b[2]).all()
    for s in a[0]:
        assert len(a[0][s]) == len(b[0][s])
        for x, y in zip(a[0][s], b[0][s]):
            assert all((x[k] == y[k]).all() for k in x)


@pytest.mark.parametrize("capture_len", [2048, 2049, 2051])
def test_stream_capture_ring_wraps(loc48, oracle, capture_len):
    """A producer-fed ring; odd lengths make every stream's ring start
    unaligned (stride capture_len * 3 bytes), which the register trigger scan
    reads word-wise (byte shift from the absolute address)."""
    lut = loc48.lut()
    adc = synth.adc_stream(6, 512 * 24, 3, lut, loc48.dims.S, 23).numpy()
    recs, est, last = run_pipeline(loc48, adc, 512, capture_len=capture_len)
    exp = oracle.stream_run(adc, 1024, 48000, loc48.dims.S, loc48.window(), lut)
    compare(recs, est, last, exp, loc48.dims.P)


@pytest.mark.parametrize("hop", [256, 1024, 384])
def test_stream_other_hops(loc48, oracle, hop):
    lut = loc48.lut()
    T = (9000 // hop) * hop
    adc = synth.adc_stream(6, T, 3, lut, loc48.dims.S, 40 + hop).numpy()
    recs, est, last = run_pipeline(loc48, adc, hop)
    exp = oracle.stream_run(adc, 1024, 48000, loc48.dims.S, loc48.window(), lut)
    compare(recs, est, last, exp, loc48.dims.P)


def test_stream_reference_trace_fixture(loc48, oracle):
    """The fixture's triggers came from the reference's own ring code."""
    g = golden("stream_trace.npz")
    adc = g["adc"]
    T = (adc.shape[1] // 512) * 512
    recs, _, _ = run_pipeline(loc48, np.ascontiguousarray(adc[:, :T]), 512)
    got = [(s, int(r["end"])) for s in sorted(recs) for r in recs[s]]
    assert got == [tuple(x) for x in g["ref_ends"] if x[1] <= T]
    for s in recs:
        for i, r in enumerate(recs[s]):
            assert (r["lags"] == g["orc_lags"][s, i]).all()
            if r["gate"]:
                assert r["cell"] == g["orc_cell"][s, i]


@pytest.mark.parametrize("N,hop,M", [(512, 256, 3), (2048, 1024, 3), (1024, 512, 4), (1024, 512, 2)])
def test_stream_register_trigger_shapes(oracle, N, hop, M):
    """frame_len = 2 x hop runs the register trigger scan (k_stream_trigger_p)
    for each (G = hop/64, M) it is instantiated for; config 5 is N 1024 / hop 512
    / 3 mics (test_stream_vs_oracle).  M = 2: a sample's two bytes gathered by
    the squares' v_perm (zeros above), M = 4: the word itself."""
    mics = {4: synth.square_mics(0.15),
            2: np.array([[-0.066, 0], [0.066, 0]], np.float32)}.get(M)
    loc = Localizer(sample_rate_hz=48000, frame_len=N, num_mics=M, mic_xy=mics)
    lut = loc.lut()
    T = (12 * N // hop) * hop
    adc = synth.adc_stream(6, T, M, lut, loc.dims.S, 70 + N + M).numpy()
    recs, est, last = run_pipeline(loc, adc, hop)
    exp = oracle.stream_run(adc, N, 48000, loc.dims.S, loc.window(), lut)
    compare(recs, est, last, exp, loc.dims.P)
    loc.close()
