"""Heat-map colour classes of vga_draw_heatmap (vga_heatmap.h:97-130), §8(f)
item 4: the oracle against a numpy restatement on the golden pipeline frames,
libtdoa's k_heatmap against the oracle (int64, exact) and a float32 numpy
restatement (GCC_PHAT scores, same summation order: exact)."""
import numpy as np
import pytest
import torch

from conftest import golden


def np_classes(w, lut):
    P = w.shape[0]
    L = np.zeros(lut.shape[1], np.int64)
    for p in range(P):
        L += w[p][lut[p]]
    hi = L.max()
    t = [(hi * 63) >> 6, (hi * 31) >> 5, (hi * 15) >> 4, (hi * 7) >> 3]
    return np.select([L >= t[0], L >= t[1], L >= t[2], L >= t[3]], [4, 3, 2, 1], 0).astype(np.uint8)


def test_oracle_heatmap_vs_numpy(oracle):
    g = golden("pipeline_cfg2.npz")
    lut = g["lut"].reshape(3, -1)
    for f in range(0, 80, 7):
        c = oracle.heatmap(g["weighted"][f], lut)
        assert (c == np_classes(g["weighted"][f], lut)).all()
        assert (c == 4).any()


@pytest.mark.gpu
def test_gpu_heatmap_direct_vs_oracle(oracle):
    from tdoa.localizer import Localizer
    loc = Localizer()
    g = golden("pipeline_cfg2.npz")
    out = loc.localize(torch.from_numpy(g["frames"]).cuda(), scores=True)
    cls = loc.heatmap(out["weighted"], out["max_L"]).cpu().numpy().reshape(len(g["frames"]), -1)
    lut = loc.lut()
    w = out["weighted"].cpu().numpy()
    for f in range(len(g["frames"])):
        assert (cls[f] == oracle.heatmap(w[f], lut)).all(), f
    loc.close()


@pytest.mark.gpu
def test_gpu_heatmap_float():
    from tdoa import synth
    from tdoa.localizer import Localizer
    loc = Localizer(engine="gcc_phat")
    lut = loc.lut()
    fr, _, _ = synth.adc_frames(16, 3, 1024, lut, 46, 4, device="cuda")
    out = loc.localize(fr, scores=True)
    cls = loc.heatmap(out["weighted_f"], out["max_Lf"]).cpu().numpy().reshape(16, -1)
    w = out["weighted_f"].cpu().numpy()
    mx = out["max_Lf"].cpu().numpy()
    for f in range(16):
        L = np.zeros(lut.shape[1], np.float32)
        for p in range(3):
            L = (L + w[f, p][lut[p]]).astype(np.float32)
        assert L.max() == mx[f]
        t = [np.float32(mx[f]) * np.float32(n / 2 ** b) for n, b in ((63, 6), (31, 5), (15, 4), (7, 3))]
        exp = np.select([L >= t[0], L >= t[1], L >= t[2], L >= t[3]], [4, 3, 2, 1], 0)
        assert (cls[f] == exp).all()
    loc.close()
