#!/usr/bin/env python3
"""Per-phase cycle split of k_direct (diagnostic build libtdoa_diag.so with
s_memtime stamps).  Never used by tests or bench.py.

    TDOA_LIB=audio-triangulation_amd/tdoa/libtdoa_diag.so python tools/diag_phases.py
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("TDOA_LIB", os.path.join(ROOT, "audio-triangulation_amd", "tdoa", "libtdoa_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "audio-triangulation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tdoa  # noqa: E402
from tdoa import synth  # noqa: E402
from tdoa.localizer import Localizer  # noqa: E402


def main():
    engine = sys.argv[1] if len(sys.argv) > 1 else "direct"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    loc = Localizer(engine=engine)
    lut = loc.lut().reshape(3, 101, 101)
    fr, _, _ = synth.adc_frames(B, 3, 1024, lut, 46, 1, device="cuda")
    out = loc.alloc_outputs(B)
    for _ in range(5):
        loc.localize_into(fr, out)
    torch.cuda.synchronize()
    L = tdoa.load()
    L.tdoa_diag_fetch.argtypes = [C.c_void_p, C.c_int]
    n = 8 * 4096
    buf = np.zeros(n, np.uint64)
    assert L.tdoa_diag_fetch(buf.ctypes.data_as(C.c_void_p), n) == 0
    st = buf.reshape(-1, 8).astype(np.int64)
    nwg = int((st[:, 0] != 0).sum())
    st = st[:nwg]
    names = ["stage", "xcorr", "argmax+prior", "grid"]
    d = np.diff(st[:, :5], axis=1)
    tot = st[:, 4] - st[:, 0]
    print(f"engine={engine} B={B} workgroups={nwg}")
    for i, nm in enumerate(names):
        print(f"  {nm:14s} median {np.median(d[:, i]):9.0f} cyc  ({np.median(d[:, i]) / np.median(tot) * 100:5.1f}%)")
    print(f"  total          median {np.median(tot):9.0f} cyc")
    span = st[:, 4].max() - st[:, 0].min()
    print(f"  launch span {span} cyc")


if __name__ == "__main__":
    main()
