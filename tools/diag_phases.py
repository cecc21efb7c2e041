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
    n = 16 * 4096
    buf = np.zeros(n, np.uint64)
    assert L.tdoa_diag_fetch(buf.ctypes.data_as(C.c_void_p), n) == 0
    st = buf.reshape(-1, 16 if os.environ.get('TDOA_DIRECT_MFMA', '1') != '0' else 8).astype(np.int64)
    nwg = int((st[:, 0] != 0).sum())
    st = st[:nwg]
    mfma = os.environ.get("TDOA_DIRECT_MFMA", "1") != "0"
    names = (["stage", "sums+xor", "xcorr", "argmax+prior", "grid"] if mfma else
             ["stage", "xcorr", "argmax+prior", "grid"])
    ns = len(names)
    d = np.diff(st[:, :ns + 1], axis=1)
    tot = st[:, ns] - st[:, 0]
    print(f"engine={engine} B={B} workgroups={nwg}")
    for i, nm in enumerate(names):
        print(f"  {nm:14s} median {np.median(d[:, i]):9.0f} cyc  ({np.median(d[:, i]) / np.median(tot) * 100:5.1f}%)")
    print(f"  total          median {np.median(tot):9.0f} cyc")
    if mfma:
        print("  stage split: tables+pads %d, raw sums %d, prep+store %d cyc (median)" %
              (np.median(st[:, 6] - st[:, 0]), np.median(st[:, 7] - st[:, 6]), np.median(st[:, 1] - st[:, 7])))
        print("  grid split: scan %d, wave reductions + barrier %d, final %d cyc (median)" %
              (np.median(st[:, 8] - st[:, 4]), np.median(st[:, 9] - st[:, 8]), np.median(st[:, 5] - st[:, 9])))
    span = st[:, ns].max() - st[:, 0].min()
    print(f"  launch span {span} cyc")
    t0 = st[:, 0] - st[:, 0].min()
    print("  workgroup start (cyc from first): p25 %d p50 %d p75 %d p90 %d max %d" %
          tuple(np.percentile(t0, [25, 50, 75, 90, 100])))
    te = st[:, ns] - st[:, 0].min()
    print("  workgroup end:                    p25 %d p50 %d p75 %d p90 %d max %d" %
          tuple(np.percentile(te, [25, 50, 75, 90, 100])))


if __name__ == "__main__":
    main()
