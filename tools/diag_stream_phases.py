#!/usr/bin/env python3
"""Per-workgroup phase split of k_direct_mfma<.., EMA> in the config-5 hop
(libtdoa_diag.so stamps of the last hop).  Diagnostic only; never used by
tests or bench.py.

    python tools/diag_stream_phases.py [S]
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
from tdoa.stream import StreamPipeline  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
H = 512
loc = Localizer(sample_rate_hz=48000)
cap = synth.adc_stream(S, 64 * H, 3, loc.lut(), loc.dims.S, synth.SEEDS[5], device="cuda")
pipe = StreamPipeline(loc, cap, hop=H, use_graph=False)
L = tdoa.load()
L.tdoa_diag_fetch.argtypes = [C.c_void_p, C.c_int]
n = 16 * 4096
for _ in range(12):
    pipe.step()
pipe.stream.synchronize()
buf = np.zeros(n, np.uint64)
assert L.tdoa_diag_fetch(buf.ctypes.data_as(C.c_void_p), n) == 0
st = buf.reshape(-1, 16).astype(np.int64)
cnt = int(pipe.out["count"].item())
nwg = (cnt + 3) // 4
st = st[:nwg]
names = [("stage", 0, 1), ("sums+xor", 1, 2), ("xcorr", 2, 3), ("argmax+prior", 3, 4), ("ema+grid", 4, 5)]
tot = st[:, 5] - st[:, 0]
print(f"count={cnt} workgroups={nwg}")
for nm, a, b in names:
    d = st[:, b] - st[:, a]
    print(f"  {nm:14s} median {np.median(d):9.0f} cyc  ({np.median(d) / np.median(tot) * 100:5.1f}%)")
print(f"  total          median {np.median(tot):9.0f} cyc")
print("  before stage: count read %d cyc; stage split: issue+zero %d, frame data+row sums %d, prep+stores %d (median)" %
      (np.median(st[:, 0] - st[:, 10]), np.median(st[:, 6] - st[:, 0]), np.median(st[:, 7] - st[:, 6]),
       np.median(st[:, 1] - st[:, 7])))
print("  grid split: scan %d, reductions %d, final %d cyc (median)" %
      (np.median(st[:, 8] - st[:, 4]), np.median(st[:, 9] - st[:, 8]), np.median(st[:, 5] - st[:, 9])))
# s_memtime has no common base across CUs: start / end of every workgroup
# from the 100 MHz realtime stamps (slots 11, 12) relative to the first start
r0 = st[:, 11].min()
rs, re_ = (st[:, 11] - r0) * 10.0, (st[:, 12] - r0) * 10.0  # ns
print("  realtime (ns from the first workgroup's start): start p50 %.0f p90 %.0f max %.0f; end p10 %.0f p50 %.0f p90 %.0f max %.0f"
      % (np.median(rs), np.percentile(rs, 90), rs.max(), np.percentile(re_, 10), np.median(re_), np.percentile(re_, 90), re_.max()))
print("  workgroup duration (realtime) p50 %.0f ns max %.0f ns" % (np.median(re_ - rs), (re_ - rs).max()))
pipe.close()
