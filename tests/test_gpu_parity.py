"""Parity of libtdoa's gfx950 kernels (through the C ABI) with the oracle.

DIRECT engine: bit-exact for every integer output (scores, weighted scores,
lags, gate, grid max, argmax cell) and exact float32 (x, y).
"""
import ctypes as C

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

import tdoa  # noqa: E402
from tdoa import _lib, synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402


def _np(d):
    return {k: v.cpu().numpy() for k, v in d.items()}


def _cmp(got, exp, keys=("lags", "gate", "cell", "max_L", "xy", "scores", "weighted")):
    for k in keys:
        if k in exp and k in got:
            g, e = got[k], exp[k]
            bad = np.argwhere(g != e) if g.shape == e.shape else None
            assert g.shape == e.shape and bad.size == 0, \
                f"{k}: {0 if bad is None else len(bad)} mismatches, first {None if bad is None else bad[:3].tolist()}"


@pytest.fixture(scope="module")
def loc3():
    return Localizer()


def test_golden_pipeline_cfg2(loc3):
    g = golden("pipeline_cfg2.npz")
    assert (loc3.lut().reshape(g["lut"].shape) == g["lut"]).all()
    fr = torch.from_numpy(g["frames"]).cuda()
    got = _np(loc3.localize(fr, scores=True))
    _cmp(got, dict(g))


def test_cfg2_batch_vs_oracle(loc3, oracle):
    lut = loc3.lut().reshape(3, 101, 101)
    fr, cells, tau = synth.adc_frames(4096, 3, 1024, lut, 46, synth.SEEDS[2], device="cuda")
    got = _np(loc3.localize(fr, scores=True))
    exp = oracle.localize_batch(fr.cpu().numpy(), 46, loc3.window(), lut, threads=8)
    _cmp(got, exp)
    # known answer: pair (0, m) lags recover the injected integer delays
    agree = (got["lags"][:, :2] == tau.cpu().numpy()[:, 1:]).mean()
    assert agree > 0.95


def test_full_range_int16_wrap(loc3, oracle):
    fr = synth.full_range_frames(512, 3, 1024, 0xABC, device="cuda")
    got = _np(loc3.localize(fr, scores=True))
    exp = oracle.localize_batch(fr.cpu().numpy(), 46, loc3.window(), loc3.lut().reshape(3, 101, 101),
                                threads=8)
    _cmp(got, exp)


@pytest.mark.parametrize("B", [1, 2, 3, 5, 7, 9, 33])
def test_ragged_batches(loc3, oracle, B):
    lut = loc3.lut().reshape(3, 101, 101)
    fr, _, _ = synth.adc_frames(B, 3, 1024, lut, 46, 1000 + B, device="cuda")
    got = _np(loc3.localize(fr, scores=True))
    exp = oracle.localize_batch(fr.cpu().numpy(), 46, loc3.window(), lut)
    _cmp(got, exp)


def test_empty_batch(loc3):
    fr = torch.empty((0, 3, 1024), dtype=torch.int16, device="cuda")
    out = loc3.localize(fr)
    assert out["lags"].shape == (0, 3)


def test_constant_frames_tie_break(loc3, oracle):
    # all-equal frames: every score 0 -> first lag (-S) wins, as in correlations.c:20
    fr = torch.full((4, 3, 1024), 128, dtype=torch.int16, device="cuda")
    got = _np(loc3.localize(fr, scores=True))
    exp = oracle.localize_batch(fr.cpu().numpy(), 46, loc3.window(), loc3.lut().reshape(3, 101, 101))
    _cmp(got, exp)
    assert (got["lags"] == -46).all()


CONFIGS = [
    # (M, N, fs, max_shift, mics, half)
    (2, 1024, 50000, 0, np.array([[-0.066, 0.0], [0.066, 0.0]], np.float32), 50),
    (3, 1024, 48000, 0, None, 50),            # 48 kHz -> S = 44
    (3, 1024, 50000, 45, None, 50),           # odd S: lag tiles start at -S-1
    (3, 256, 50000, 0, None, 20),
    (3, 512, 50000, 0, None, 50),
    (4, 4096, 50000, 0, synth.square_mics(0.15), 50),
    (8, 2048, 50000, 0, synth.circle_mics(8, 0.15), 50),
    (5, 2048, 50000, 63, synth.circle_mics(5, 0.3), 30),
    # 3 mics, S = 63, a triangle twice the reference's: 6510 distinct lag tuples,
    # more than the keyed grid holds in registers (the generic grid solve)
    (3, 1024, 67600, 63, np.array([[-0.132, -0.076], [0.132, -0.076], [0.0, 0.152]], np.float32), 50),
    # a 261 x 261 grid: more cells than the keyed grid's 16 index bits
    (3, 1024, 50000, 0, None, 130),
    # 2 mics x 4096: frames exceed k_direct_mfma's staging registers -> the VALU
    # k_direct and the separate int64 branch-and-bound grid (k_grid_bb<int64_t>)
    (2, 4096, 50000, 0, np.array([[-0.066, 0.0], [0.066, 0.0]], np.float32), 50),
]


@pytest.mark.parametrize("M,N,fs,S_cfg,mics,half", CONFIGS)
def test_configs_vs_oracle(oracle, M, N, fs, S_cfg, mics, half):
    loc = Localizer(num_mics=M, frame_len=N, sample_rate_hz=fs, max_shift=S_cfg, mic_xy=mics,
                    grid_half_w=half, grid_half_h=half)
    S = loc.dims.S
    lut = loc.lut()
    mic_xy = loc.mics()
    exp_lut = oracle.build_lut(mic_xy, half_w=half, half_h=half, fs=fs, max_shift=S)
    assert (lut == exp_lut.reshape(lut.shape)).all()
    exp_win = tdoa.dpss_q15(1024)[::1024 // N] if N <= 1024 else tdoa.dpss_q15(N)
    assert (loc.window() == exp_win).all()
    B = 48 if N <= 2048 else 24
    fr, _, _ = synth.adc_frames(B, M, N, exp_lut, S, 77 + M + N, device="cuda")
    fr2 = synth.full_range_frames(8, M, N, 99 + N, device="cuda")
    fr = torch.cat([fr, fr2]).contiguous()
    got = _np(loc.localize(fr, scores=True))
    exp = oracle.localize_batch(fr.cpu().numpy(), S, loc.window(), exp_lut,
                                half_w=half, half_h=half, threads=8)
    _cmp(got, exp)


def test_prepared_path_arbitrary_int16(oracle):
    loc = Localizer(num_mics=2, mic_xy=np.array([[-0.066, 0], [0.066, 0]], np.float32))
    g = torch.Generator().manual_seed(5)
    fr = torch.randint(-32768, 32768, (64, 2, 1024), generator=g, dtype=torch.int32).to(torch.int16)
    fr[0, :, :] = -32768   # extreme products
    fr[1, 0, :] = 32767
    fr[1, 1, :] = -32768
    out = _np(loc.correlate_prepared(fr.cuda().contiguous(), scores=True, grid=False))
    for b in range(fr.shape[0]):
        sc, best = oracle.xcorr(fr[b, 0].numpy(), fr[b, 1].numpy(), 46)
        assert (out["scores"][b, 0] == sc).all(), b
        assert out["lags"][b, 0] == best
        assert (out["weighted"][b, 0] == oracle.prior(sc, best)).all()


def test_ema_streams_vs_oracle(oracle):
    loc = Localizer()
    Sn, steps = 16, 24
    rng = np.random.default_rng(21)
    est = torch.zeros((Sn, 3, 93), dtype=torch.int64, device="cuda")
    best = torch.zeros((Sn, 3), dtype=torch.int32, device="cuda")
    est_ref = np.zeros((Sn, 3, 93), np.int64)
    last = np.zeros(Sn, np.uint64)
    lut = loc.lut()
    for t in range(steps):
        fresh = rng.integers(-(1 << 40), 1 << 40, (Sn, 3, 93)).astype(np.int64)
        now = last + rng.integers(1000, 900000, Sn).astype(np.uint64)
        dec = np.array([tdoa.decay_us(int(n), int(l)) for n, l in zip(now, last)], np.float32)
        solve = {"cell": torch.empty(Sn, dtype=torch.int32, device="cuda"),
                 "max_L": torch.empty(Sn, dtype=torch.int64, device="cuda"),
                 "xy": torch.empty((Sn, 2), dtype=torch.float32, device="cuda")}
        loc.average(est, torch.from_numpy(fresh).cuda(), torch.from_numpy(dec).cuda(), best, solve)
        for s in range(Sn):
            for p in range(3):
                est_ref[s, p], b = oracle.average(est_ref[s, p], fresh[s, p], float(dec[s]))
                assert best[s, p].item() == b
            mL, cell = oracle.grid_solve(est_ref[s], lut.reshape(3, 101, 101))
            assert solve["cell"][s].item() == cell and solve["max_L"][s].item() == mL
        assert (est.cpu().numpy() == est_ref).all()
        last = now


def test_ema_solve_many_pairs_branch_and_bound(oracle):
    """tdoa_average_batch's grid solve at the config-4 geometry (8 mics, 28
    pairs): the int64 k_grid_bb with the grouped running maxima of the bound
    pass (P > 8), against the oracle's exhaustive scan, bit for bit -- random
    EMA scores (weak bounds) and one stream of all-equal scores (ties)."""
    loc = Localizer(num_mics=8, frame_len=2048, mic_xy=synth.circle_mics(8, 0.15))
    P, K = loc.dims.P, loc.dims.K
    lut = loc.lut().reshape(P, 101, 101)
    Sn, steps = 12, 4
    rng = np.random.default_rng(28)
    est = torch.zeros((Sn, P, K), dtype=torch.int64, device="cuda")
    best = torch.zeros((Sn, P), dtype=torch.int32, device="cuda")
    est_ref = np.zeros((Sn, P, K), np.int64)
    for t in range(steps):
        fresh = rng.integers(-(1 << 40), 1 << 40, (Sn, P, K)).astype(np.int64)
        fresh[0] = 12345  # every tuple ties: the first cell
        dec = rng.uniform(0.05, 1.0, Sn).astype(np.float32)
        solve = {"cell": torch.empty(Sn, dtype=torch.int32, device="cuda"),
                 "max_L": torch.empty(Sn, dtype=torch.int64, device="cuda"),
                 "xy": torch.empty((Sn, 2), dtype=torch.float32, device="cuda")}
        loc.average(est, torch.from_numpy(fresh).cuda(), torch.from_numpy(dec).cuda(), best, solve)
        for s in range(Sn):
            for p in range(P):
                est_ref[s, p], _ = oracle.average(est_ref[s, p], fresh[s, p], float(dec[s]))
            mL, cell = oracle.grid_solve(est_ref[s], lut)
            assert solve["cell"][s].item() == cell and solve["max_L"][s].item() == mL, (t, s)
        assert (est.cpu().numpy() == est_ref).all()
    loc.close()


@pytest.mark.parametrize("path", ["gpu", "host"])
def test_reference_symbols_gpu_backed(oracle, path):
    """The reference-named per-frame entry points (tdoa_reference_abi.h) on the
    GPU (the default) and on libtdoa's host-CPU path (tdoa_ref_set_device(-1),
    BASELINE config 1), bit-exact with the reference's components and the oracle."""
    from ref_symbols_check import check_reference_symbols
    L = tdoa.load()
    assert L.tdoa_ref_set_device(-1 if path == "host" else 0) == 0
    try:
        check_reference_symbols(L, oracle)
    finally:
        assert L.tdoa_ref_set_device(0) == 0


def test_plain_c_host_program():
    """host/tdoa_host.c: the reference loop through the reference-named
    symbols, then the batched GCC-PHAT API, from plain C."""
    import os
    import subprocess
    from conftest import PKG
    exe = os.path.join(PKG, "host", "tdoa_host")
    assert os.path.exists(exe), "build with `make -C audio-triangulation_amd host`"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "lags ab=5 ac=9 bc=4" in r.stdout
    assert "recovered all three injected lags" in r.stdout


@pytest.mark.parametrize("N", [256, 512, 1024])
def test_default_window_is_reference_table(N):
    """N <= 1024: the 1024-point table subsampled as buffer.c:8 indexes it,
    WINDOW_FUNCTION[i << (10 - BUFFER_SIZE_BITS)] (pinned to window_function.h
    in test_oracle_pin.py)."""
    loc = Localizer(frame_len=N)
    w1k = golden("window_q15.npz")["n1024"]
    assert (loc.window() == w1k[::1024 // N]).all()
    loc.close()


def test_correlate_prepared_on_gcc_phat_context_returns_direct_outputs(oracle):
    """correlations_init inputs run the reference's integer path whatever the
    context's engine: the call returns the int64 outputs it filled."""
    loc = Localizer(engine="gcc_phat")
    g = torch.Generator(device="cpu").manual_seed(11)
    fr = torch.randint(-32768, 32768, (8, 3, 1024), generator=g, dtype=torch.int32)
    fr = fr.to(torch.int16).cuda()
    got = _np(loc.correlate_prepared(fr))
    assert "scores" in got and "weighted" in got and "max_L" in got
    frn = fr.cpu().numpy()
    for b in range(frn.shape[0]):
        for p, (i, j) in enumerate([(0, 1), (0, 2), (1, 2)]):
            sc, best = oracle.xcorr(frn[b, i], frn[b, j], 46)
            assert (got["scores"][b, p] == sc).all()
            assert got["lags"][b, p] == best
    loc.close()
