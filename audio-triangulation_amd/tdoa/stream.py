"""Streaming pipeline: the Python face of tdoa_stream_* (include/tdoa.h).

The batched form of the reference's sample loop (sample_compute.h:53-146)
for S independent streams: every `step()` consumes one hop of H samples per
stream from a device capture ring of 8-bit ADC bytes [S][capture_len][M]
(dma_sampler.c:17-23), runs the trigger scan, the DIRECT path on the
triggered frames, the EMA (correlations.c:38-63) and the grid solve on the
EMA scores -- all libtdoa kernels, replayed as one hipGraph per step.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from ._lib import StreamOutputs, check, load
from .localizer import Localizer


class StreamPipeline:
    # use_graph: each hop replayed as a captured hipGraph of its two kernels.
    # Plain stream launches are the default: 67.0 vs 71.8 us per config-5 hop
    # (tools/diag_stream_launch.py, same box; the graph's launch adds ~5 us)
    def __init__(self, loc: Localizer, capture: torch.Tensor, hop: int = 512,
                 use_graph: bool = False):
        if loc.engine != "direct":
            raise ValueError("the streaming pipeline runs the DIRECT engine")
        if capture.dtype != torch.uint8 or capture.dim() != 3 or capture.shape[2] != loc.dims.M:
            raise ValueError(f"capture must be uint8 [S][T][{loc.dims.M}]")
        if capture.device != loc.torch_device or not capture.is_contiguous():
            raise ValueError("capture must be contiguous on the localizer's device")
        self.loc, self.capture, self.hop = loc, capture, hop
        self.S, self.capture_len = capture.shape[0], capture.shape[1]
        P = loc.dims.P
        dev = loc.torch_device
        S = self.S
        self.out = {
            "count": torch.zeros(1, dtype=torch.int32, device=dev),
            "stream_id": torch.zeros(S, dtype=torch.int32, device=dev),
            "end": torch.zeros(S, dtype=torch.int64, device=dev),
            "lags": torch.zeros((S, P), dtype=torch.int32, device=dev),
            "gate": torch.zeros(S, dtype=torch.uint8, device=dev),
            "ema_best": torch.zeros((S, P), dtype=torch.int32, device=dev),
            "cell": torch.zeros(S, dtype=torch.int32, device=dev),
            "xy": torch.zeros((S, 2), dtype=torch.float32, device=dev),
            "max_L": torch.zeros(S, dtype=torch.int64, device=dev),
        }
        self._s = StreamOutputs(*[self.out[n].data_ptr() for n, _ in StreamOutputs._fields_])
        # graph capture needs a real (non-default) stream
        self.stream = torch.cuda.Stream(device=dev)
        h = C.c_void_p()
        check(load().tdoa_stream_create(loc._ctx, S, hop, C.c_void_p(capture.data_ptr()),
                                        self.capture_len, int(use_graph), C.byref(h)),
              "tdoa_stream_create")
        self._h = h

    def step(self) -> dict:
        """One hop for every stream (asynchronous on self.stream)."""
        check(load().tdoa_stream_step(self._h, C.byref(self._s),
                                      C.c_void_p(self.stream.cuda_stream)), "tdoa_stream_step")
        return self.out

    def records(self) -> dict:
        """Synchronously fetch this step's triggered slots, sorted by stream."""
        self.stream.synchronize()
        n = int(self.out["count"].item())
        r = {k: v[:n].cpu().numpy() for k, v in self.out.items() if k != "count"}
        order = np.argsort(r["stream_id"], kind="stable")
        return {k: v[order] for k, v in r.items()}

    def reset(self) -> None:
        check(load().tdoa_stream_reset(self._h, C.c_void_p(self.stream.cuda_stream)),
              "tdoa_stream_reset")

    def state(self):
        P, K = self.loc.dims.P, self.loc.dims.K
        pos = np.zeros(1, np.int64)
        est = np.zeros((self.S, P, K), np.int64)
        last = np.zeros(self.S, np.uint64)
        check(load().tdoa_stream_state(self._h, pos.ctypes.data_as(C.c_void_p),
                                       est.ctypes.data_as(C.c_void_p),
                                       last.ctypes.data_as(C.c_void_p), None), "tdoa_stream_state")
        return int(pos[0]), est, last

    def totals(self):
        """(samples consumed per stream, triggered frames, gated frames) so far."""
        pos = np.zeros(1, np.int64)
        st = np.zeros(2, np.int64)
        check(load().tdoa_stream_state(self._h, pos.ctypes.data_as(C.c_void_p), None, None,
                                       st.ctypes.data_as(C.c_void_p)), "tdoa_stream_state")
        return int(pos[0]), int(st[0]), int(st[1])

    def close(self) -> None:
        if getattr(self, "_h", None):
            load().tdoa_stream_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
