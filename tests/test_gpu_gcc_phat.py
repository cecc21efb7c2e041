"""GCC_PHAT engine (fp32 FFT on gfx950) against the float64 oracle
(oracle/gcc_phat_oracle.py).

Tolerances (stated here, checked below):
  scores_f, weighted_f   |gpu - fp64| <= 3e-5 absolute (PHAT scores lie in [-1, 1])
  lags, gate             equal wherever the fp64 top-2 score margin > 2e-4
  cell / xy              equal wherever the fp64 grid max beats every other
                         tuple's L by > 1e-3 (xy is the cell's coordinates)
  max_Lf                 |gpu - fp64| <= 1e-3
On clean integer-delay frames the lags equal DIRECT's (the reference's).
"""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

import gcc_phat_oracle as G  # noqa: E402
from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402

TOL_SCORE = 3e-5
TOL_LAG_MARGIN = 2e-4
TOL_CELL_MARGIN = 1e-3
# GCC-PHAT vs DIRECT (the reference's integer xcorr, correlations.c:20-23) lag
# agreement on integer-delay frames: measured 100 % of pairs on the config-2
# batch (two seeds, tools/diag_agree.py) and on the first 65536 frames of the
# config-3/4 bench batches (bench.py "parity").  Contract: the measured rate
# minus a 1e-3 slack, and every disagreement a near-tie of the fp64 GCC-PHAT
# scores (its score at DIRECT's lag within TOL_DISAGREE of its own best).
AGREE_MIN = 1.0 - 1e-3
TOL_DISAGREE = 2e-3


def _np(d):
    return {k: v.cpu().numpy() for k, v in d.items()}


def check_phat(got, exp, grid=True):
    s_exp = exp["scores_f"]
    assert np.abs(got["scores_f"] - s_exp).max() <= TOL_SCORE
    srt = np.sort(s_exp, axis=-1)
    margin = srt[..., -1] - srt[..., -2]
    sure = margin > TOL_LAG_MARGIN
    assert (got["lags"][sure] == exp["lags"][sure]).all()
    lag_ok = (got["lags"] == exp["lags"]).all(-1)
    assert (got["gate"][lag_ok] == exp["gate"][lag_ok]).all()
    same = got["lags"] == exp["lags"]
    assert np.abs(got["weighted_f"] - exp["weighted_f"])[same].max(initial=0) <= TOL_SCORE
    if grid:
        Lg = exp["L"]
        top = Lg.max(-1)
        cells = got["cell"]
        # margin of the fp64 max over every cell whose L differs from it
        second = np.where(Lg >= top[:, None] - 1e-12, -np.inf, Lg).max(-1)
        sure_c = (top - second > TOL_CELL_MARGIN) & lag_ok
        Lsel = Lg[np.arange(len(cells)), cells]
        assert (np.abs(Lsel[sure_c] - top[sure_c]) < 1e-9).all()
        assert np.abs(got["max_Lf"] - exp["max_Lf"])[lag_ok].max(initial=0) <= 1e-3
        W = 101
        xy = np.stack([(cells % W - 50).astype(np.float32) / np.float32(24.0),
                       (50 - cells // W).astype(np.float32) / np.float32(24.0)], -1)
        assert (got["xy"] == xy).all()
    return sure.mean()


@pytest.fixture(scope="module")
def phat3():
    return Localizer(engine="gcc_phat")


def test_golden_frames_vs_fp64(phat3):
    g = golden("pipeline_cfg2.npz")
    fr = torch.from_numpy(g["frames"]).cuda()
    got = _np(phat3.localize(fr, scores=True))
    exp = G.gcc_phat_batch(g["frames"], 46, phat3.window(), phat3.lut())
    check_phat(got, exp)


def test_cfg2_batch_vs_fp64_and_direct(phat3):
    lut = phat3.lut().reshape(3, 101, 101)
    fr, cells, tau = synth.adc_frames(4096, 3, 1024, lut, 46, synth.SEEDS[2], device="cuda")
    got = _np(phat3.localize(fr, scores=True))
    exp = G.gcc_phat_batch(fr.cpu().numpy(), 46, phat3.window(), lut)
    frac_sure = check_phat(got, exp)
    assert frac_sure > 0.95
    # the north-star lag contract: on integer-delay frames GCC-PHAT lags match
    # the injected delays and DIRECT's (the reference's) lags
    direct = Localizer(engine="direct")
    d = _np(direct.localize(fr))
    assert (got["lags"][:, :2] == tau.cpu().numpy()[:, 1:]).mean() >= AGREE_MIN
    check_agreement(got, d, exp, 46)


def check_agreement(got, d, exp, S):
    """GCC-PHAT lags vs DIRECT's: rate >= AGREE_MIN, disagreements near-ties."""
    same = got["lags"] == d["lags"]
    assert same.mean() >= AGREE_MIN, same.mean()
    for b, p in np.argwhere(~same):
        s64 = exp["scores_f"][b, p]
        gap = s64.max() - s64[d["lags"][b, p] + S]
        assert gap <= TOL_DISAGREE, (b, p, gap)
    return same.mean()


@pytest.mark.parametrize("M,N,mics", [(4, 4096, "square"), (8, 2048, "circle")])
def test_long_frames_agree_with_direct(M, N, mics):
    # BASELINE configs 3 and 4 shapes: the two-pass kernels (and the fused
    # per-frame kernel when TDOA_PHAT_FUSED=1) against DIRECT and fp64
    xy = synth.square_mics(0.15) if mics == "square" else synth.circle_mics(8, 0.15)
    kw = dict(num_mics=M, frame_len=N, sample_rate_hz=50000, mic_xy=xy)
    ph = Localizer(engine="gcc_phat", **kw)
    S = ph.dims.S
    fr, _, _ = synth.adc_frames(384, M, N, ph.lut(), S, 0xA6 + M, device="cuda")
    got = _np(ph.localize(fr, scores=True))
    exp = G.gcc_phat_batch(fr.cpu().numpy(), S, ph.window(), ph.lut())
    check_phat(got, exp)
    direct = Localizer(engine="direct", **kw)
    check_agreement(got, _np(direct.localize(fr)), exp, S)
    ph.close()
    direct.close()


def test_full_range_frames(phat3):
    fr = synth.full_range_frames(256, 3, 1024, 0xBEE, device="cuda")
    got = _np(phat3.localize(fr, scores=True))
    exp = G.gcc_phat_batch(fr.cpu().numpy(), 46, phat3.window(), phat3.lut())
    check_phat(got, exp)


def test_constant_frames_tie_break(phat3):
    fr = torch.full((3, 3, 1024), 77, dtype=torch.int16, device="cuda")
    got = _np(phat3.localize(fr, scores=True))
    assert (got["scores_f"] == 0).all() and (got["lags"] == -46).all()


def test_empty_and_ragged(phat3):
    out = phat3.localize(torch.empty((0, 3, 1024), dtype=torch.int16, device="cuda"))
    assert out["lags"].shape == (0, 3)
    lut = phat3.lut().reshape(3, 101, 101)
    fr, _, _ = synth.adc_frames(5, 3, 1024, lut, 46, 3, device="cuda")
    got = _np(phat3.localize(fr, scores=True))
    check_phat(got, G.gcc_phat_batch(fr.cpu().numpy(), 46, phat3.window(), lut))


TWO = np.array([[-0.066, 0.0], [0.066, 0.0]], np.float32)
PHAT_CONFIGS = [
    # (M, N, fs, mics, batch): fused kernels for M <= 3, N <= 2048 ...
    (2, 1024, 50000, TWO, 96), (3, 256, 50000, None, 96), (3, 512, 48000, None, 96),
    (3, 2048, 50000, None, 96), (2, 2048, 48000, TWO, 96),
    # ... two-pass spectra/pairs kernels beyond (BASELINE configs 3 and 4 shapes)
    (4, 4096, 50000, synth.square_mics(0.15), 40),
    (8, 2048, 50000, synth.circle_mics(8, 0.15), 40),
    (3, 4096, 48000, None, 40),
    (2, 4096, 50000, TWO, 40),                             # long-frame kernels, 1 pair
    (4, 2048, 67600, synth.square_mics(0.15), 40),         # S = 63: lags -63..63, the widest K
    (5, 1024, 50000, synth.circle_mics(5, 0.15), 64),
    (4, 256, 50000, synth.square_mics(0.15), 64),
    # the reference triangle doubled, S = 63: 6510 distinct lag tuples, more
    # than k_p1k_lean's LDS tail holds -> the generic fused k_gcc_phat_1024
    (3, 1024, 67600, np.array([[-0.132, -0.076], [0.132, -0.076], [0.0, 0.152]], np.float32), 64),
]


@pytest.mark.parametrize("M,N,fs,mics,B", PHAT_CONFIGS)
def test_configs(M, N, fs, mics, B):
    loc = Localizer(engine="gcc_phat", num_mics=M, frame_len=N, sample_rate_hz=fs, mic_xy=mics)
    S = loc.dims.S
    lut = loc.lut()
    fr, _, _ = synth.adc_frames(B, M, N, lut, S, 40 + N + M, device="cuda")
    fr2 = synth.full_range_frames(4, M, N, 7 + N, device="cuda")
    fr = torch.cat([fr, fr2]).contiguous()
    got = _np(loc.localize(fr, scores=True))
    exp = G.gcc_phat_batch(fr.cpu().numpy(), S, loc.window(), lut)
    sure = check_phat(got, exp)
    assert sure > 0.5
    loc.close()


def test_split_path_chunking_matches_one_chunk():
    """The two-pass path runs in chunks of its spectrum scratch; a batch spanning
    several chunks must equal the per-frame results."""
    M, N = 8, 2048
    loc = Localizer(engine="gcc_phat", num_mics=M, frame_len=N, mic_xy=synth.circle_mics(8, 0.15))
    lut = loc.lut()
    # 128 MiB scratch / (8 * 2048 * 8 B) = 1024 frames per chunk
    fr, _, _ = synth.adc_frames(1100, M, N, lut, loc.dims.S, 5, device="cuda")
    big = _np(loc.localize(fr))
    part = _np(loc.localize(fr[1020:1030].contiguous()))
    for k in ("lags", "gate", "cell", "xy", "max_Lf"):
        assert (big[k][1020:1030] == part[k]).all(), k
    loc.close()


def _grid_f32(weighted, lut):
    """vga_heatmap.h:99-108 on the engine's own float weighted scores, in float32
    with the kernel's association ((w0 + w1) + w2): max L and the first cell."""
    w = np.asarray(weighted, np.float32)
    lut2 = np.asarray(lut).reshape(w.shape[1], -1).astype(np.int64)
    L = w[:, 0][:, lut2[0]]
    for p in range(1, w.shape[1]):
        L = (L + w[:, p][:, lut2[p]]).astype(np.float32)
    return L.argmax(-1).astype(np.int32), L.max(-1)


@pytest.mark.parametrize("kind", ["adc", "adc_3iter", "adc_ragged", "full_range", "noise_only",
                                  "constant", "mixed"])
def test_grid_exact_on_own_scores(phat3, kind):
    """The config-2 kernel scans the 2469 distinct lag tuples for a wave's two
    frames at once; its cell and max L must equal the exhaustive float32 scan
    of its own weighted scores bit for bit (ties to the first row-major cell):
    peaked, flat noisy and all-equal scores (every tuple ties), and waves whose
    two frames are one peaked and one constant.  6144 / 6151 frames: several
    workgroups per CU, a ragged last workgroup."""
    lut = phat3.lut()
    if kind.startswith("adc"):
        B = {"adc": 2048, "adc_3iter": 6144, "adc_ragged": 6151}[kind]
        fr, _, _ = synth.adc_frames(B, 3, 1024, lut.reshape(3, 101, 101), 46, 77, device="cuda")
    elif kind == "full_range":
        fr = synth.full_range_frames(512, 3, 1024, 0x51, device="cuda")
    elif kind == "constant":
        fr = torch.full((64, 3, 1024), 77, dtype=torch.int16, device="cuda")
    elif kind == "mixed":  # frames 2w peaked, 2w + 1 constant: one wave, both extremes
        fr, _, _ = synth.adc_frames(256, 3, 1024, lut.reshape(3, 101, 101), 46, 78, device="cuda")
        fr[1::2] = 77
    else:  # uncorrelated mics: flat, noisy scores, weak bounds
        g = torch.Generator(device="cpu").manual_seed(5)
        fr = (torch.randint(0, 256, (512, 3, 1024), generator=g, dtype=torch.int16)).cuda()
    got = _np(phat3.localize(fr, scores=True))
    cell, mx = _grid_f32(got["weighted_f"], lut)
    assert (got["cell"] == cell).all()
    assert (got["max_Lf"] == mx).all()


@pytest.mark.parametrize("shape", ["cfg3", "cfg4", "wide"])
@pytest.mark.parametrize("kind", ["adc", "noise_only", "constant"])
def test_grid_bb_exact_on_own_scores(shape, kind):
    """Configs 3/4 solve the grid by exact branch and bound (k_grid_bb: entries
    of <= 64 tuples from one 8 x 8 block of cells, skipped when their bound is
    below the best L found).  Cell and max L must equal the exhaustive float32
    scan of the engine's own weighted scores bit for bit: peaked scores (ADC
    frames, strong pruning), flat noisy scores (weak bounds) and all-equal
    scores (every entry ties: first cell).  "wide": a 0.3 m square, whose
    entries span lag ranges wider than the sparse-table queries encode (> 15
    lags): the table is marked wide and the exhaustive k_grid solves it."""
    M, N, xy = {"cfg3": (4, 4096, synth.square_mics(0.15)), "cfg4": (8, 2048, synth.circle_mics(8, 0.15)),
                "wide": (4, 2048, synth.square_mics(0.3))}[shape]
    loc = Localizer(engine="gcc_phat", num_mics=M, frame_len=N, mic_xy=xy)
    lut = loc.lut()
    B = 300
    if kind == "adc":
        fr, _, _ = synth.adc_frames(B, M, N, lut.reshape(-1, 101, 101), loc.dims.S, 91, device="cuda")
    elif kind == "noise_only":
        g = torch.Generator(device="cpu").manual_seed(6)
        fr = torch.randint(0, 256, (B, M, N), generator=g, dtype=torch.int16).cuda()
    else:
        fr = torch.full((8, M, N), 77, dtype=torch.int16, device="cuda")
    got = _np(loc.localize(fr, scores=True))
    cell, mx = _grid_f32(got["weighted_f"], lut)
    assert (got["cell"] == cell).all()
    assert (got["max_Lf"] == mx).all()


# ---- GCC-PHAT cell / (x, y) contract against DIRECT (the reference semantics:
# the first row-major maximum of vga_heatmap.h:99-108 on the int64 weighted
# scores of correlations.c:20-33).  The two engines score lags differently
# (PHAT-whitened fp32 vs raw integer products), so their grid maxima can fall
# on different cells where DIRECT's own L is nearly flat.  Contract per shape,
# on ADC-like integer-delay frames (synth.adc_frames, the bench's seeds):
#   agreement rate >= CELL_AGREE[shape]: measured 0.9995 (cfg2, 4096 frames),
#     0.9644 (cfg3, 2048), 0.9453 (cfg4, 2048), minus a 0.001-0.01 slack
#   every disagreeing frame is a near-tie of DIRECT's own L: (max L - L[gcc
#     cell]) / |max L| <= CELL_L_GAP (measured max 0.0066; median 0.0009-0.0033),
#     the cells lying 1-2 grid cells apart at the median (max 7)
CELL_SHAPES = {
    "cfg2": dict(M=3, N=1024, mics=None, B=4096),
    "cfg3": dict(M=4, N=4096, mics="square", B=2048),
    "cfg4": dict(M=8, N=2048, mics="circle", B=2048),
}
CELL_AGREE = {"cfg2": 0.9985, "cfg3": 0.955, "cfg4": 0.935}
CELL_L_GAP = 0.01
# the disagreeing frames' (x, y) distance to DIRECT's, metres: measured max
# 0.093 (cfg2), 0.317 (cfg3), 0.358 (cfg4) over the bench's 4096 / 65536 /
# 65536 frames (profiles/r03_c*_gcc_phat_bench.json `parity`).  "(x, y) within
# 1e-5 relative" of the reference semantics holds for DIRECT (bit-exact) and for
# the LS refinement against its double oracle, not for GCC-PHAT's cell.
XY_MAX_M = {"cfg2": 0.12, "cfg3": 0.40, "cfg4": 0.40}


def _direct_L_at(weighted, lut, cells):
    """DIRECT's int64 L (sum over pairs of weighted[p][lut[p][cell]]) at given cells."""
    P = weighted.shape[1]
    lut2 = np.asarray(lut).reshape(P, -1).astype(np.int64)
    idx = lut2[:, cells].T  # [B][P]
    return np.take_along_axis(weighted, idx[:, :, None], axis=2)[:, :, 0].sum(-1)


@pytest.mark.parametrize("shape", sorted(CELL_SHAPES))
def test_cell_contract_vs_direct(shape):
    c = CELL_SHAPES[shape]
    xy = {None: None, "square": synth.square_mics(0.15), "circle": synth.circle_mics(8, 0.15)}[c["mics"]]
    kw = dict(num_mics=c["M"], frame_len=c["N"], mic_xy=xy)
    ph = Localizer(engine="gcc_phat", **kw)
    direct = Localizer(engine="direct", **kw)
    lut = ph.lut()
    fr, _, _ = synth.adc_frames(c["B"], c["M"], c["N"], lut.reshape(ph.dims.P, 101, 101), ph.dims.S,
                                synth.SEEDS[{"cfg2": 2, "cfg3": 3, "cfg4": 4}[shape]], device="cuda")
    got = _np(ph.localize(fr))
    d = _np(direct.localize(fr, scores=True))
    same = got["cell"] == d["cell"]
    rate = same.mean()
    L_gcc = _direct_L_at(d["weighted"], lut, got["cell"])
    gap = (d["max_L"] - L_gcc) / np.maximum(np.abs(d["max_L"]), 1)
    W = 101
    cheb = np.maximum(np.abs(got["cell"] % W - d["cell"] % W), np.abs(got["cell"] // W - d["cell"] // W))
    bad = ~same & ~(gap <= CELL_L_GAP)
    print(f"{shape}: cells equal {rate:.4f}; disagreements {int((~same).sum())}: "
          f"L gap p50 {np.median(gap[~same]) if (~same).any() else 0:.4f} max {gap.max():.4f}, "
          f"cells apart p50 {np.median(cheb[~same]) if (~same).any() else 0} max {cheb.max()}")
    assert (gap >= 0).all()  # DIRECT's cell is DIRECT's maximum
    assert rate >= CELL_AGREE[shape], rate
    assert not bad.any(), np.argwhere(bad)[:5].ravel().tolist()
    dist = np.hypot(*(got["xy"] - d["xy"]).T)
    assert (dist[same] == 0).all()
    assert dist.max() <= XY_MAX_M[shape], float(dist.max())
    ph.close()
    direct.close()


def test_long_frames_big_grid_exhaustive():
    """A 261 x 261 grid at 4 mics x 2048: more 8 x 8 blocks than k_grid_bb's
    table holds -> the exhaustive float grid (k_grid) after k_frame16."""
    loc = Localizer(engine="gcc_phat", num_mics=4, frame_len=2048, mic_xy=synth.square_mics(0.15),
                    grid_half_w=130, grid_half_h=130)
    lut = loc.lut()
    fr, _, _ = synth.adc_frames(64, 4, 2048, lut.reshape(6, 261, 261), loc.dims.S, 0x261, device="cuda")
    got = _np(loc.localize(fr, scores=True))
    cell, mx = _grid_f32(got["weighted_f"], lut)
    assert (got["cell"] == cell).all()
    assert (got["max_Lf"] == mx).all()
    loc.close()


def test_prepared_launch_matches_localize_into(phat3):
    """Localizer.prepare (bench.py's timed loop) enqueues the same launch as
    localize_into: identical outputs on the same batch."""
    lut = phat3.lut().reshape(3, 101, 101)
    fr, _, _ = synth.adc_frames(512, 3, 1024, lut, 46, 0x9E, device="cuda")
    a = phat3.alloc_outputs(512)
    b = phat3.alloc_outputs(512)
    phat3.localize_into(fr, a)
    run = phat3.prepare(fr, b)
    run()
    run()  # a second enqueue of the same prebuilt launch
    torch.cuda.synchronize()
    for k in a:
        assert torch.equal(a[k], b[k]), k
