"""Least-squares refinement (a15, north-star extension absent in the
reference; definition in oracle/tdoa_oracle.h).  CPU: the double-precision
oracle recovers known source positions from exact continuous lags.  GPU:
libtdoa's k_ls against the oracle on the same raw scores / lags / cells.
Tolerance (BASELINE north star): (x, y) within 1e-5 relative."""
import numpy as np
import pytest
import torch

from tdoa import synth

TOL = 1e-5


def _lags_at(mics, u, v, h=1.2, fs=50000.0, c=343.0):
    n = np.sqrt(u * u + v * v + h * h)
    P3 = np.array([u * h / n, v * h / n, h * h / n])
    d = np.sqrt(((P3[None, :2] - mics) ** 2).sum(1) + P3[2] ** 2)
    M = len(mics)
    return np.array([(d[j] - d[i]) * fs / c for i in range(M) for j in range(i + 1, M)])


@pytest.mark.parametrize("M", [3, 4, 8])
def test_oracle_ls_known_answer(oracle, M):
    mics = synth.circle_mics(M, 0.15) if M != 4 else synth.square_mics(0.15)
    K, S = 93, 46
    rng = np.random.default_rng(M)
    for _ in range(6):
        u, v = rng.uniform(-1.8, 1.8, 2)
        tau = _lags_at(mics, u, v)
        best = np.round(tau).astype(np.int32)[None]
        k = np.arange(K) - S
        sc = (1e9 - 1e6 * (k[None, :] - tau[:, None]) ** 2)[None]  # vertex at tau
        cell = (50 - int(round(v * 24))) * 101 + int(round(u * 24)) + 50
        uv, rms = oracle.ls_refine(sc, best, mics, [cell])
        assert np.abs(uv[0] - [u, v]).max() < 1e-9
        assert rms[0] < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("engine,M,N", [("direct", 3, 1024), ("gcc_phat", 3, 1024),
                                        ("direct", 8, 2048), ("gcc_phat", 4, 4096),
                                        ("gcc_phat", 8, 2048)])
def test_gpu_ls_vs_oracle(oracle, engine, M, N):
    from tdoa.localizer import Localizer
    mics = None if M == 3 else (synth.circle_mics(8, 0.15) if M == 8 else synth.square_mics(0.15))
    loc = Localizer(engine=engine, num_mics=M, frame_len=N, mic_xy=mics)
    lut = loc.lut()
    fr, _, _ = synth.adc_frames(64, M, N, lut, loc.dims.S, 11 + M, device="cuda")
    got = {k: v.cpu().numpy() for k, v in loc.localize(fr, scores=True, ls=True).items()}
    raw = got["scores"] if engine == "direct" else got["scores_f"]
    uv, rms = oracle.ls_refine(raw, got["lags"], loc.mics(), got["cell"])
    err = np.abs(got["xy_ls"] - uv) / np.maximum(1.0, np.abs(uv))
    assert err.max() <= TOL
    assert np.abs(got["ls_rms"] - rms).max() <= 1e-4 * max(1.0, rms.max())
    # without scores / cell requested the scratch path (the long-frame kernels:
    # the three peak scores per pair written by k_frame16) gives the same answer
    lean = loc.localize(fr, grid=False, ls=True)
    assert (lean["xy_ls"].cpu().numpy() == got["xy_ls"]).all()
    loc.close()


@pytest.mark.gpu
def test_gpu_ls_refines_toward_true_position(oracle):
    """Integer-delay frames from random cells: the refined point stays within
    a cell or so of the source cell's coordinates."""
    from tdoa.localizer import Localizer
    loc = Localizer(num_mics=8, frame_len=2048, mic_xy=synth.circle_mics(8, 0.15))
    lut = loc.lut()
    fr, cells, _ = synth.adc_frames(128, 8, 2048, lut, loc.dims.S, 77, device="cuda")
    got = loc.localize(fr, ls=True)
    xy_true = loc.cell_xy(cells.cpu().numpy())
    d_grid = np.linalg.norm(got["xy"].cpu().numpy() - xy_true, axis=1)
    d_ls = np.linalg.norm(got["xy_ls"].cpu().numpy() - xy_true, axis=1)
    assert np.median(d_ls) <= np.median(d_grid) + 1.0 / 24
    loc.close()
