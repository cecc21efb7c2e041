"""ctypes binding of libtdoa.so (include/tdoa.h, include/tdoa_reference_abi.h).

This is the Python host side of the product: it only marshals device
pointers (torch tensors on the GPU) into the C ABI.  Every computation runs in
libtdoa's gfx950 kernels; if the library or a gfx950 device is missing the
calls raise -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TDOA_LIB") or os.path.join(HERE, "libtdoa.so")

ENGINE_DIRECT = 0
ENGINE_GCC_PHAT = 1
ENGINES = {"direct": ENGINE_DIRECT, "gcc_phat": ENGINE_GCC_PHAT}

STATUS = {0: "TDOA_OK", -1: "TDOA_ERR_INVALID", -2: "TDOA_ERR_HIP",
          -3: "TDOA_ERR_NO_DEVICE", -4: "TDOA_ERR_NOMEM"}

# Every symbol include/*.h declares (tests check the library exports them).
EXPORTED_SYMBOLS = [
    # tdoa.h
    "tdoa_config_default", "tdoa_create", "tdoa_destroy", "tdoa_get_dims",
    "tdoa_localize_batch", "tdoa_correlate_prepared", "tdoa_average_batch",
    "tdoa_decay_us", "tdoa_get_window", "tdoa_get_mics", "tdoa_get_lut",
    "tdoa_get_prior", "tdoa_dpss_q15", "tdoa_last_error", "tdoa_abi_version", "tdoa_batch_kernel",
    "tdoa_batch_grid_fused", "tdoa_gpu_clock_mhz",
    "tdoa_heatmap", "tdoa_stream_create", "tdoa_stream_step", "tdoa_stream_reset", "tdoa_stream_state",
    "tdoa_stream_destroy",
    # tdoa_reference_abi.h
    "microphones_init", "rolling_buffer_init", "rolling_buffer_push",
    "rolling_buffer_write_out", "rolling_buffer_get_incoming_power",
    "rolling_buffer_get_outgoing_power", "buffer_window",
    "buffer_normalize_range", "correlations_init", "correlations_average",
    "tdoa_ref_set_clock", "tdoa_ref_set_device",
    "mic_a_location", "mic_b_location", "mic_c_location",
]


class TdoaError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: {STATUS.get(code, code)}: {msg}")
        self.code = code


class Config(C.Structure):
    """struct tdoa_config (include/tdoa.h)."""
    _fields_ = [
        ("num_mics", C.c_int32), ("frame_len", C.c_int32),
        ("sample_rate_hz", C.c_int32), ("max_shift", C.c_int32),
        ("speed_of_sound", C.c_float), ("engine", C.c_int32),
        ("mic_xy", C.POINTER(C.c_float)),
        ("grid_half_w", C.c_int32), ("grid_half_h", C.c_int32),
        ("grid_scale", C.c_float), ("height_offset", C.c_float),
        ("window_q15", C.POINTER(C.c_int32)), ("phat_eps", C.c_float),
    ]


class Outputs(C.Structure):
    """struct tdoa_outputs (include/tdoa.h): device pointers."""
    _fields_ = [(n, C.c_void_p) for n in (
        "lags", "gate", "cell", "xy", "max_L", "max_Lf", "scores", "weighted",
        "scores_f", "weighted_f", "xy_ls", "ls_rms")]


class StreamOutputs(C.Structure):
    """struct tdoa_stream_outputs (include/tdoa.h): device pointers."""
    _fields_ = [(n, C.c_void_p) for n in (
        "count", "stream_id", "end", "lags", "gate", "ema_best", "cell", "xy", "max_L")]


# reference structs (include/tdoa_reference_abi.h, reference buffer.h:8-12,
# rolling_buffer.h:13-25, correlations.h:10-16, point.h:3-6)
class Buffer(C.Structure):
    _fields_ = [("buffer", C.c_int16 * 1024), ("power", C.c_int64)]


class RollingBuffer(C.Structure):
    _fields_ = [("head", C.c_int), ("incoming_power", C.c_int64),
                ("incoming_total", C.c_int64), ("outgoing_power", C.c_int64),
                ("outgoing_total", C.c_int64), ("is_full", C.c_bool),
                ("buffer", C.c_int16 * 1024)]


class Correlations(C.Structure):
    _fields_ = [("correlations", C.c_int64 * 93), ("best_shift", C.c_int),
                ("last_update", C.c_uint64)]


class Point2d(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float)]


CLOCK_FN = C.CFUNCTYPE(C.c_uint64)

_lib = None


def load() -> C.CDLL:
    """Load libtdoa.so (built in-tree by __graft_entry__.build / make)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise TdoaError(-3, "load", f"{LIB_PATH} missing: run `make -C audio-triangulation_amd`")
    L = C.CDLL(LIB_PATH)
    P, I32, I64 = C.c_void_p, C.c_int32, C.c_int64
    L.tdoa_config_default.argtypes = [C.POINTER(Config)]
    L.tdoa_create.argtypes = [C.POINTER(Config), C.c_int, C.POINTER(P)]
    L.tdoa_destroy.argtypes = [P]
    L.tdoa_get_dims.argtypes = [P] + [C.POINTER(I32)] * 5
    L.tdoa_localize_batch.argtypes = [P, P, I64, C.POINTER(Outputs), P]
    L.tdoa_correlate_prepared.argtypes = [P, P, I64, C.POINTER(Outputs), P]
    L.tdoa_average_batch.argtypes = [P, I64, P, P, P, P, C.POINTER(Outputs), P]
    L.tdoa_decay_us.argtypes = [C.c_uint64, C.c_uint64]
    L.tdoa_decay_us.restype = C.c_float
    L.tdoa_get_window.argtypes = [P, P]
    L.tdoa_get_mics.argtypes = [P, P]
    L.tdoa_get_lut.argtypes = [P, P]
    L.tdoa_get_prior.argtypes = [P, P]
    L.tdoa_dpss_q15.argtypes = [I32, C.c_double, P]
    L.tdoa_last_error.restype = C.c_char_p
    L.tdoa_abi_version.restype = C.c_int
    L.tdoa_batch_kernel.argtypes = [P]
    L.tdoa_batch_kernel.restype = C.c_char_p
    L.tdoa_batch_grid_fused.argtypes = [P]
    L.tdoa_batch_grid_fused.restype = C.c_int
    L.tdoa_gpu_clock_mhz.argtypes = [C.c_int, P, C.c_double, C.POINTER(C.c_double)]
    L.tdoa_heatmap.argtypes = [P, P, P, C.c_int, I64, P, P]
    L.tdoa_stream_create.argtypes = [P, I32, I32, P, I64, C.c_int, C.POINTER(P)]
    L.tdoa_stream_step.argtypes = [P, C.POINTER(StreamOutputs), P]
    L.tdoa_stream_reset.argtypes = [P, P]
    L.tdoa_stream_state.argtypes = [P, P, P, P, P]
    L.tdoa_stream_destroy.argtypes = [P]
    # reference-named per-frame symbols
    L.microphones_init.argtypes = []
    L.rolling_buffer_init.argtypes = [C.POINTER(RollingBuffer)]
    L.rolling_buffer_push.argtypes = [C.POINTER(RollingBuffer), C.c_int16]
    L.rolling_buffer_write_out.argtypes = [C.POINTER(RollingBuffer), C.POINTER(Buffer)]
    L.rolling_buffer_get_incoming_power.argtypes = [C.POINTER(RollingBuffer)]
    L.rolling_buffer_get_incoming_power.restype = C.c_int64
    L.rolling_buffer_get_outgoing_power.argtypes = [C.POINTER(RollingBuffer)]
    L.rolling_buffer_get_outgoing_power.restype = C.c_int64
    L.buffer_window.argtypes = [C.POINTER(Buffer)]
    L.buffer_normalize_range.argtypes = [C.POINTER(Buffer)]
    L.correlations_init.argtypes = [C.POINTER(Correlations), C.POINTER(Buffer), C.POINTER(Buffer)]
    L.correlations_average.argtypes = [C.POINTER(Correlations), C.POINTER(Correlations)]
    L.tdoa_ref_set_clock.argtypes = [CLOCK_FN]
    L.tdoa_ref_set_device.argtypes = [C.c_int]
    _lib = L
    return L


def check(rc: int, where: str) -> None:
    if rc != 0:
        msg = load().tdoa_last_error()
        raise TdoaError(rc, where, msg.decode() if msg else "")


def dpss_q15(n: int, nw: float = 2.0):
    """DPSS(n, nw) Q15 window from libtdoa's host generator."""
    import numpy as np
    out = np.zeros(n, np.int32)
    check(load().tdoa_dpss_q15(n, nw, out.ctypes.data_as(C.c_void_p)), "tdoa_dpss_q15")
    return out


def decay_us(now_us: int, last_us: int) -> float:
    return float(load().tdoa_decay_us(int(now_us), int(last_us)))
