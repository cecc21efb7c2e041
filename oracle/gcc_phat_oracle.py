"""Float64 GCC-PHAT restatement (TEST INFRASTRUCTURE ONLY).

The reference has no FFT/PHAT path: GCC_PHAT is the north-star
formulation layered on the reference's integer front end and back end.  This
oracle defines it:

  x      = prep(frame) / 2^15       prep = rolling_buffer.c:64-66 DC removal,
                                    buffer.c:13-16 <<8 wrap, buffer.c:4-11 window
  X_m    = rfft(x_m, L = 2N)        zero-padded: linear (not circular) lags
  R_ij   = conj(X_i) X_j / max(|conj(X_i) X_j|, eps)      (PHAT)
  r_ij   = irfft(R_ij, L)           r[s] peaks at s = d when mic j lags mic i by d,
                                    the sign of correlations.c:9-16
  scores = r[s mod L], s = -S..S;   best = first max (correlations.c:20-23)
  weighted = scores * scale[|s - best|]  (the float32 prior of correlations.c:30)
  gate, grid L = sum_p weighted_p[LUT_p] and its first argmax as DIRECT.

Parity of the fp32 GPU engine against this is tolerance-based (tests say
which tolerance); on clean integer-delay frames its lags equal DIRECT's.
"""
from __future__ import annotations

import numpy as np


def prep(frames: np.ndarray, window: np.ndarray) -> np.ndarray:
    """Integer front end, vectorised: int16 [B][M][N] raw -> windowed int16."""
    fr = np.asarray(frames, dtype=np.int16)
    N = fr.shape[-1]
    bits = int(np.log2(N))
    tot = fr.astype(np.int64).sum(-1, keepdims=True)
    off = (tot >> bits).astype(np.int64)
    x = ((fr.astype(np.int64) - off) & 0xFFFF).astype(np.uint16).view(np.int16)
    x = ((x.astype(np.int64) << 8) & 0xFFFF).astype(np.uint16).view(np.int16)
    t = x.astype(np.int64) * np.asarray(window, np.int64)
    return ((t >> 15) & 0xFFFF).astype(np.uint16).view(np.int16)


def prior_table(K: int) -> np.ndarray:
    d = np.arange(K)
    arg = (-(d * d)).astype(np.float32) / np.float32(36.0)
    return np.exp(arg.astype(np.float64)).astype(np.float32)


def gcc_phat_batch(frames, S, window, lut=None, eps=1e-12, half_w=50, half_h=50,
                   grid_scale=24.0):
    x = prep(frames, window).astype(np.float64) / 32768.0
    B, M, N = x.shape
    L = 2 * N
    X = np.fft.rfft(x, L, axis=-1)
    pairs = [(i, j) for i in range(M) for j in range(i + 1, M)]
    P, K = len(pairs), 2 * S + 1
    s_idx = np.arange(-S, S + 1) % L
    scores = np.zeros((B, P, K))
    for p, (i, j) in enumerate(pairs):
        R = np.conj(X[:, i]) * X[:, j]
        R = R / np.maximum(np.abs(R), eps)
        r = np.fft.irfft(R, L, axis=-1)
        scores[:, p] = r[:, s_idx]
    best = np.argmax(scores, axis=-1)  # first max
    lags = (best - S).astype(np.int32)
    pr = prior_table(K).astype(np.float64)
    d = np.abs(np.arange(K)[None, None, :] - best[..., None])
    weighted = scores * pr[d]
    res = {"scores_f": scores, "weighted_f": weighted, "lags": lags,
           "gate": ((lags.astype(np.int64) ** 2).sum(-1) > 4).astype(np.uint8)}
    if lut is not None:
        lut2 = np.asarray(lut).reshape(P, -1).astype(np.int64)
        Lg = np.zeros((B, lut2.shape[1]))
        for p in range(P):
            Lg += weighted[:, p][:, lut2[p]]
        cell = np.argmax(Lg, axis=-1)
        W = 2 * half_w + 1
        res["cell"] = cell.astype(np.int32)
        res["max_Lf"] = Lg.max(-1)
        res["L"] = Lg
        res["xy"] = np.stack([(cell % W - half_w).astype(np.float32) / np.float32(grid_scale),
                              (half_h - cell // W).astype(np.float32) / np.float32(grid_scale)], -1)
    return res
