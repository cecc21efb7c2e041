"""MI355X TDOA localizer -- Python host side over libtdoa.so.

    from tdoa import Localizer
    loc = Localizer()                       # reference config: 3 mics, 1024, 50 kHz
    out = loc.localize(frames_int16_cuda)   # lags, gate, cell, xy, max_L

See include/tdoa.h for the C ABI and DESIGN.md for the kernels.
"""
from ._lib import (ENGINE_DIRECT, ENGINE_GCC_PHAT, EXPORTED_SYMBOLS, LIB_PATH,  # noqa: F401
                   TdoaError, decay_us, dpss_q15, load)

__all__ = ["Localizer", "TdoaError", "load", "dpss_q15", "decay_us"]


def __getattr__(name):
    # torch-dependent pieces load lazily so the ABI helpers work without torch
    if name == "Localizer":
        from .localizer import Localizer
        return Localizer
    if name in ("synth", "localizer", "stream", "shard"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
