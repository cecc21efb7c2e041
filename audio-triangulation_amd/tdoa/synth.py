"""Synthetic multi-mic frames of the BASELINE shapes.

ADC-like frames: int16 holding u8 samples around 128 (dma_sampler.c:17-20,
sample_compute.h:67-69 read 8-bit ADC bytes into sample_t).  A broadband
N(0, src_std) source reaches mic m delayed by an integer tau_m taken from the
grid LUT of a random cell (tau_0 = 0, tau_m = LUT_(0,m)[cell] - S), plus
N(0, noise_std) noise, rounded and clipped to [0, 255].

`full_range` frames are uniform over all of int16 and exercise the
reference's int16 wrap paths (rolling_buffer.c:65-66, buffer.c:16).
"""
from __future__ import annotations

import numpy as np
import torch

SEEDS = {1: 0x5EED0001, 2: 0x5EED0002, 3: 0x5EED0003, 4: 0x5EED0004, 5: 0x5EED0005}


def adc_frames(B: int, M: int, N: int, lut: np.ndarray, S: int, seed: int,
               device: str | torch.device = "cpu", src_std: float = 40.0,
               noise_std: float = 8.0, mean: float = 128.0):
    """Returns (frames int16 [B][M][N], cells int64 [B], tau int64 [B][M])."""
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    P, G = lut.shape[0], lut.reshape(lut.shape[0], -1).shape[1]
    lut_t = torch.as_tensor(lut.reshape(P, -1).astype(np.int64), device=dev)
    cells = torch.randint(0, G, (B,), generator=g, device=dev)
    tau = torch.zeros((B, M), dtype=torch.int64, device=dev)
    for m in range(1, M):
        tau[:, m] = lut_t[m - 1][cells] - S  # pair (0, m) is index m-1
    pad = S + 1
    src = torch.randn((B, N + 2 * pad), generator=g, device=dev) * src_std
    idx = torch.arange(N, device=dev).view(1, 1, N) + pad - tau.view(B, M, 1)
    x = torch.gather(src.view(B, 1, -1).expand(B, M, -1), 2, idx)
    x = x + torch.randn((B, M, N), generator=g, device=dev) * noise_std + mean
    frames = torch.clamp(torch.round(x), 0, 255).to(torch.int16)
    return frames.contiguous(), cells, tau


def full_range_frames(B: int, M: int, N: int, seed: int, device="cpu") -> torch.Tensor:
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    return torch.randint(-32768, 32768, (B, M, N), generator=g, device=dev,
                         dtype=torch.int32).to(torch.int16).contiguous()


def adc_stream(S: int, T: int, M: int, lut: np.ndarray, max_shift: int, seed: int,
               device: str | torch.device = "cpu", burst_len: int = 700,
               gap: tuple = (1500, 3500), src_std: float = 40.0, noise_std: float = 0.5,
               mean: float = 128.0) -> torch.Tensor:
    """Config 5 capture bytes u8 [S][T][M] (round-robin per sample, dma_sampler.c:17-23).

    Each stream has a stationary source at a random grid cell emitting
    broadband bursts of `burst_len` samples separated by random gaps; mic m
    hears it delayed by tau_m (the cell's LUT lags), over a quiet noise floor.
    The reference triggers as a burst leaves the newer half of the ring."""
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    P, G = lut.shape[0], lut.reshape(lut.shape[0], -1).shape[1]
    lut_t = torch.as_tensor(lut.reshape(P, -1).astype(np.int64), device=dev)
    cells = torch.randint(0, G, (S,), generator=g, device=dev)
    tau = torch.zeros((S, M), dtype=torch.int64, device=dev)
    for m in range(1, M):
        tau[:, m] = lut_t[m - 1][cells] - max_shift
    pad = max_shift + 1
    TT = T + 2 * pad
    nb = TT // gap[0] + 2
    gaps = torch.randint(gap[0], gap[1], (S, nb), generator=g, device=dev)
    starts = torch.cumsum(gaps, 1) - gaps[:, :1] + torch.randint(0, gap[0], (S, 1), generator=g,
                                                                 device=dev)
    edge = torch.zeros((S, TT + burst_len + 1), dtype=torch.int32, device=dev)
    ok = starts < TT
    st = torch.where(ok, starts, torch.full_like(starts, TT))
    edge.scatter_add_(1, st, ok.to(torch.int32))
    edge.scatter_add_(1, st + burst_len, -ok.to(torch.int32))
    env = (torch.cumsum(edge, 1)[:, :TT] > 0).to(torch.float32)
    y = torch.randn((S, TT), generator=g, device=dev) * src_std * env
    idx = torch.arange(T, device=dev).view(1, 1, T) + pad - tau.view(S, M, 1)
    x = torch.gather(y.view(S, 1, -1).expand(S, M, -1), 2, idx)
    x = x + torch.randn((S, M, T), generator=g, device=dev) * noise_std + mean
    b = torch.clamp(torch.round(x), 0, 255).to(torch.uint8)
    return b.permute(0, 2, 1).contiguous()


def square_mics(side: float = 0.15) -> np.ndarray:
    """Config 3: 4-mic square centred on the origin."""
    h = side / 2
    return np.array([[-h, -h], [h, -h], [h, h], [-h, h]], np.float32)


def circle_mics(M: int = 8, radius: float = 0.15) -> np.ndarray:
    """Config 4: M-mic circle centred on the origin."""
    a = 2 * np.pi * np.arange(M) / M
    return np.stack([radius * np.cos(a), radius * np.sin(a)], -1).astype(np.float32)
