"""Batched localizer: the Python face of include/tdoa.h.

`Localizer.localize(frames)` is the batched form of the reference's per-frame
hot path (sample_compute.h:105-134 -> vga_heatmap.h:99-108).  Inputs and
outputs are torch tensors on the context's GPU; torch only provides device
memory and the stream -- the work is libtdoa's kernels.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import Config, Outputs, check, load


def _ptr(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


@dataclass
class Geometry:
    """Derived sizes of a context: M mics, N samples, P pairs, K lags, G cells."""
    M: int
    N: int
    P: int
    K: int
    G: int
    S: int = field(init=False)

    def __post_init__(self):
        self.S = (self.K - 1) // 2


class Localizer:
    """One libtdoa context bound to one GPU (not thread-safe).

    engine: "direct" (exact int64, the reference's semantics bit-for-bit) or
    "gcc_phat" (fp32 FFT cross-spectrum with PHAT weighting).
    """

    def __init__(self, num_mics: int = 3, frame_len: int = 1024,
                 sample_rate_hz: int = 50000, max_shift: int = 0,
                 engine: str = "direct", mic_xy=None, grid_half_w: int = 50,
                 grid_half_h: int = 50, grid_scale: float = 24.0,
                 height_offset: float = 1.2, speed_of_sound: float = 343.0,
                 window_q15=None, phat_eps: float = 1e-12, device: int = 0):
        L = load()
        cfg = Config()
        L.tdoa_config_default(C.byref(cfg))
        cfg.num_mics = num_mics
        cfg.frame_len = frame_len
        cfg.sample_rate_hz = sample_rate_hz
        cfg.max_shift = max_shift
        cfg.speed_of_sound = speed_of_sound
        cfg.engine = _lib.ENGINES[engine]
        cfg.grid_half_w = grid_half_w
        cfg.grid_half_h = grid_half_h
        cfg.grid_scale = grid_scale
        cfg.height_offset = height_offset
        cfg.phat_eps = phat_eps
        self._keep = []
        if mic_xy is not None:
            a = np.ascontiguousarray(mic_xy, dtype=np.float32).reshape(-1)
            assert a.size == 2 * num_mics, "mic_xy must be [num_mics][2]"
            self._keep.append(a)
            cfg.mic_xy = a.ctypes.data_as(C.POINTER(C.c_float))
        if window_q15 is not None:
            w = np.ascontiguousarray(window_q15, dtype=np.int32)
            assert w.size == frame_len
            self._keep.append(w)
            cfg.window_q15 = w.ctypes.data_as(C.POINTER(C.c_int32))
        self.engine = engine
        self.device = device
        self.torch_device = torch.device("cuda", device)
        ctx = C.c_void_p()
        check(L.tdoa_create(C.byref(cfg), device, C.byref(ctx)), "tdoa_create")
        self._ctx = ctx
        d = [C.c_int32() for _ in range(5)]
        check(L.tdoa_get_dims(ctx, *[C.byref(x) for x in d]), "tdoa_get_dims")
        self.dims = Geometry(*[x.value for x in d])
        self.grid_W = 2 * grid_half_w + 1
        self.grid_half_w, self.grid_half_h, self.grid_scale = grid_half_w, grid_half_h, grid_scale

    # ---------------------------------------------------------- lifetime
    def close(self):
        if getattr(self, "_ctx", None):
            load().tdoa_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------- tables
    def batch_kernel(self) -> str:
        """Name of the kernel a batch of this context runs first (tdoa_batch_kernel)."""
        return (load().tdoa_batch_kernel(self._ctx) or b"").decode()

    def batch_grid_fused(self) -> bool:
        """A grid-requesting batch solves the grid inside its first kernel (tdoa_batch_grid_fused)."""
        return bool(load().tdoa_batch_grid_fused(self._ctx))

    def window(self) -> np.ndarray:
        w = np.zeros(self.dims.N, np.int32)
        check(load().tdoa_get_window(self._ctx, w.ctypes.data_as(C.c_void_p)), "tdoa_get_window")
        return w

    def mics(self) -> np.ndarray:
        m = np.zeros((self.dims.M, 2), np.float32)
        check(load().tdoa_get_mics(self._ctx, m.ctypes.data_as(C.c_void_p)), "tdoa_get_mics")
        return m

    def lut(self) -> np.ndarray:
        lut = np.zeros((self.dims.P, self.dims.G), np.uint8)
        check(load().tdoa_get_lut(self._ctx, lut.ctypes.data_as(C.c_void_p)), "tdoa_get_lut")
        return lut

    def prior(self) -> np.ndarray:
        p = np.zeros(self.dims.K, np.float32)
        check(load().tdoa_get_prior(self._ctx, p.ctypes.data_as(C.c_void_p)), "tdoa_get_prior")
        return p

    # ---------------------------------------------------------- compute
    def alloc_outputs(self, B: int, scores: bool = False, grid: bool = True,
                      ls: bool = False, engine: str | None = None) -> dict:
        """Output tensors for a batch of B frames; `engine` overrides the
        context's (the prepared path always fills the DIRECT int64 set)."""
        dev, P, K = self.torch_device, self.dims.P, self.dims.K
        direct = (engine or self.engine) == "direct"
        o = {"lags": torch.empty((B, P), dtype=torch.int32, device=dev),
             "gate": torch.empty(B, dtype=torch.uint8, device=dev)}
        if grid:
            o["cell"] = torch.empty(B, dtype=torch.int32, device=dev)
            o["xy"] = torch.empty((B, 2), dtype=torch.float32, device=dev)
            if direct:
                o["max_L"] = torch.empty(B, dtype=torch.int64, device=dev)
            else:
                o["max_Lf"] = torch.empty(B, dtype=torch.float32, device=dev)
        if ls:
            o["xy_ls"] = torch.empty((B, 2), dtype=torch.float32, device=dev)
            o["ls_rms"] = torch.empty(B, dtype=torch.float32, device=dev)
        if scores:
            if direct:
                o["scores"] = torch.empty((B, P, K), dtype=torch.int64, device=dev)
                o["weighted"] = torch.empty((B, P, K), dtype=torch.int64, device=dev)
            else:
                o["scores_f"] = torch.empty((B, P, K), dtype=torch.float32, device=dev)
                o["weighted_f"] = torch.empty((B, P, K), dtype=torch.float32, device=dev)
        return o

    @staticmethod
    def _outputs_struct(o: dict) -> Outputs:
        s = Outputs()
        for name, _ in Outputs._fields_:
            t = o.get(name)
            setattr(s, name, None if t is None else t.data_ptr())
        return s

    def _check_frames(self, frames: torch.Tensor) -> int:
        M, N = self.dims.M, self.dims.N
        if frames.dtype != torch.int16 or frames.dim() != 3 or tuple(frames.shape[1:]) != (M, N):
            raise ValueError(f"frames must be int16 [B][{M}][{N}], got {tuple(frames.shape)} {frames.dtype}")
        if frames.device != self.torch_device:
            raise ValueError(f"frames must live on {self.torch_device}")
        if not frames.is_contiguous():
            raise ValueError("frames must be contiguous")
        return frames.shape[0]

    def localize_into(self, frames: torch.Tensor, out: dict, stream=None) -> dict:
        """Asynchronous batched localization into preallocated outputs."""
        B = self._check_frames(frames)
        st = stream if stream is not None else torch.cuda.current_stream(self.torch_device)
        s = self._outputs_struct(out)
        check(load().tdoa_localize_batch(self._ctx, C.c_void_p(frames.data_ptr()), B,
                                         C.byref(s), C.c_void_p(st.cuda_stream)),
              "tdoa_localize_batch")
        return out

    def prepare(self, frames: torch.Tensor, out: dict, stream=None):
        """A prebuilt localize_into(frames, out, stream): the argument checks and
        the ctypes output struct are done once, and each call of the returned
        function enqueues the same tdoa_localize_batch (frames and outputs must
        stay allocated; they are kept referenced).  For launch loops whose
        host-side Python would otherwise be on the critical path."""
        B = self._check_frames(frames)
        st = stream if stream is not None else torch.cuda.current_stream(self.torch_device)
        s = self._outputs_struct(out)
        fn = load().tdoa_localize_batch
        args = (self._ctx, C.c_void_p(frames.data_ptr()), B, C.byref(s), C.c_void_p(st.cuda_stream))

        def launch():
            rc = fn(*args)
            if rc != 0:
                check(rc, "tdoa_localize_batch")
            return out

        launch.keep = (frames, out, s, st)
        return launch

    def localize(self, frames: torch.Tensor, scores: bool = False, grid: bool = True,
                 stream=None, ls: bool = False) -> dict:
        out = self.alloc_outputs(self._check_frames(frames), scores=scores, grid=grid, ls=ls)
        return self.localize_into(frames, out, stream)

    def correlate_prepared(self, prepared: torch.Tensor, scores: bool = True,
                           grid: bool = True) -> dict:
        """Frames already DC-removed, normalised and windowed (correlations_init
        inputs).  Runs the reference's integer path (DIRECT) on any context, so
        the int64 outputs are returned whatever the context's engine."""
        B = self._check_frames(prepared)
        out = self.alloc_outputs(B, scores=scores, grid=grid, engine="direct")
        s = self._outputs_struct(out)
        st = torch.cuda.current_stream(self.torch_device)
        check(load().tdoa_correlate_prepared(self._ctx, C.c_void_p(prepared.data_ptr()), B,
                                             C.byref(s), C.c_void_p(st.cuda_stream)),
              "tdoa_correlate_prepared")
        return out

    def average(self, est: torch.Tensor, fresh: torch.Tensor, decay: torch.Tensor,
                best: torch.Tensor, solve: dict | None = None) -> None:
        """EMA of correlations.c:38-63 over S streams, in place on `est`/`best`."""
        S = est.shape[0]
        P, K = self.dims.P, self.dims.K
        assert est.dtype == torch.int64 and tuple(est.shape) == (S, P, K) and est.is_contiguous()
        assert fresh.dtype == torch.int64 and tuple(fresh.shape) == (S, P, K) and fresh.is_contiguous()
        assert decay.dtype == torch.float32 and decay.numel() == S
        assert best.dtype == torch.int32 and tuple(best.shape) == (S, P)
        st = torch.cuda.current_stream(self.torch_device)
        sol = C.byref(self._outputs_struct(solve)) if solve is not None else None
        check(load().tdoa_average_batch(self._ctx, S, _ptr(est), _ptr(fresh), _ptr(decay),
                                        _ptr(best), sol, C.c_void_p(st.cuda_stream)),
              "tdoa_average_batch")

    def heatmap(self, weighted: torch.Tensor, max_L: torch.Tensor) -> torch.Tensor:
        """vga_heatmap.h:110-130 colour classes [B][H][W] (4 white .. 0 black)."""
        B = weighted.shape[0]
        is_float = weighted.dtype == torch.float32
        assert weighted.dtype in (torch.int64, torch.float32) and max_L.dtype == weighted.dtype
        assert tuple(weighted.shape[1:]) == (self.dims.P, self.dims.K) and weighted.is_contiguous()
        H = self.dims.G // self.grid_W
        out = torch.empty((B, H, self.grid_W), dtype=torch.uint8, device=self.torch_device)
        st = torch.cuda.current_stream(self.torch_device)
        check(load().tdoa_heatmap(self._ctx, _ptr(weighted), _ptr(max_L), int(is_float), B,
                                  _ptr(out), C.c_void_p(st.cuda_stream)), "tdoa_heatmap")
        return out

    def cell_xy(self, cell: np.ndarray) -> np.ndarray:
        """((x - half_w)/scale, (half_h - y)/scale) of row-major cells, float32 as on device."""
        cell = np.asarray(cell)
        x = (cell % self.grid_W - self.grid_half_w).astype(np.float32)
        y = (self.grid_half_h - cell // self.grid_W).astype(np.float32)
        return np.stack([x / np.float32(self.grid_scale), y / np.float32(self.grid_scale)], -1)
