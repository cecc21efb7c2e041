"""The reference's OWN sample loop EXECUTED, unchanged, against libtdoa: the
protothread of src/sample_compute.h:45-150 (included as it stands, with
host/pico_host/ for the Pico SDK side), its rolling_buffer_* / buffer_* /
correlations_* calls resolved by libtdoa.so and run on libtdoa's host path
(tdoa_ref_set_device(-1): no HIP call, so it runs here without a GPU).
host/sample_compute_main.c feeds a synthetic 3-mic capture (injected delays
5 / 9 samples) and, at every VGA hand-off, logs the loop's own structs.  Each
hand-off is then checked against the oracle:

  rings      the reference's running totals / powers equal their sums over
             the two halves of the ring (rolling_buffer.c:16-41), and the
             trigger condition of sample_compute.h:75-90 holds
  buffers    write_out -> normalize -> window of the ring == the loop's
             buffer_a/b/c (rolling_buffer.c:43-71, buffer.c:4-18)
  new_corr   int64 xcorr + first max + lag prior == correlations_init's
             (correlations.c:4-33), for (a,b), (a,c), (b,c)
  corr       the EMA chain (correlations.c:38-63) with the loop's own clock

Skipped where the reference is absent (the GPU box).  Nothing built here is
shipped; the reference's component .c files are not compiled."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import PKG, golden
from tdoa import _lib

REF = "/root/reference/src"
RECORD = [("smp", C.c_int64), ("now", C.c_uint64)] + \
         [(f"rb{m}", _lib.RollingBuffer) for m in "abc"] + \
         [(f"buf{m}", _lib.Buffer) for m in "abc"] + \
         [(f"new_{p}", _lib.Correlations) for p in ("ab", "ac", "bc")] + \
         [(f"est_{p}", _lib.Correlations) for p in ("ab", "ac", "bc")]


class Record(C.Structure):
    _fields_ = RECORD


def _i16(a):
    return np.frombuffer(bytes(a), np.int16).copy()


def _i64(a):
    return np.frombuffer(bytes(a), np.int64).copy()


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "sample_compute.h")),
                    reason="reference sources not present (GPU box)")
def test_unchanged_reference_loop_runs_on_libtdoa(tmp_path, oracle):
    # TDOA_LIB: another build of the library (tests/test_sanitizers.py: the
    # ASan + UBSan build, whose runtime the process inherits via LD_PRELOAD; the
    # host program itself stays a gcc build -- the reference's protothread
    # header uses GCC's labels-as-values in a form clang rejects,
    # pt_cornell_rp2040_v1_3.h:800,860 -- so only libtdoa's side is instrumented)
    lib = os.environ.get("TDOA_LIB") or os.path.join(PKG, "tdoa", "libtdoa.so")
    if not os.path.exists(lib):
        pytest.skip("libtdoa.so not built")
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    exe = tmp_path / "sample_compute_host"
    cmd = ["gcc", "-std=gnu11", "-O2", "-w", "-I", os.path.join(PKG, "host", "pico_host"),
           "-I", REF, os.path.join(PKG, "host", "sample_compute_main.c"), lib,
           "-L/opt/rocm/lib", "-lamdhip64", "-lm",
           "-Wl,--no-undefined", "-Wl,-rpath," + os.path.dirname(lib), "-o", str(exe)]
    if os.environ.get("TDOA_SAN") == "1":  # the instrumented library's runtime (clang's, preloaded)
        cmd[-2:-2] = [os.environ["LD_PRELOAD"]]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    log = tmp_path / "handoffs.bin"
    n = 12
    env = dict(os.environ, TDOA_REF_HOST="1", TDOA_REF_LOG=str(log))
    r = subprocess.run([str(exe), str(n)], capture_output=True, text=True, env=env, timeout=300)
    # exit 0: the last hand-off's best shifts are the injected delays (5, 9, 4)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    raw = log.read_bytes()
    assert len(raw) == n * C.sizeof(Record)
    recs = [Record.from_buffer_copy(raw, i * C.sizeof(Record)) for i in range(n)]

    win = golden("window_q15.npz")["n1024"]
    S, K, H = 46, 93, 512
    thr = 2 << 18  # POWER_THRESHOLD, sample_compute.h:21
    est = {p: np.zeros(K, np.int64) for p in ("ab", "ac", "bc")}
    last = {p: 0 for p in ("ab", "ac", "bc")}
    prev_smp = -1
    for rec in recs:
        assert rec.smp > prev_smp
        prev_smp = rec.smp
        po = pi = 0
        w = {}
        for m in "abc":
            rb = getattr(rec, f"rb{m}")
            assert rb.is_full
            ring = _i16(rb.buffer).astype(np.int64)
            lin = np.concatenate([ring[rb.head:], ring[:rb.head]])  # oldest first
            out_h, in_h = lin[:H], lin[H:]
            assert rb.outgoing_total == out_h.sum() and rb.outgoing_power == (out_h * out_h).sum()
            assert rb.incoming_total == in_h.sum() and rb.incoming_power == (in_h * in_h).sum()
            po += (int(rb.outgoing_power) << 9) - int(rb.outgoing_total) ** 2
            pi += (int(rb.incoming_power) << 9) - int(rb.incoming_total) ** 2
            dc, pw = oracle.dc_remove(lin.astype(np.int16))
            w[m] = oracle.window(oracle.normalize(dc), win)
            buf = getattr(rec, f"buf{m}")
            assert (_i16(buf.buffer) == w[m]).all(), m
            assert buf.power == pw, m
        assert po > thr + pi  # the trigger fired on this frame (sample_compute.h:89)
        for p in ("ab", "ac", "bc"):
            sc, best = oracle.xcorr(w[p[0]], w[p[1]], S)
            new = getattr(rec, f"new_{p}")
            assert new.best_shift == best, p
            assert (_i64(new.correlations) == oracle.prior(sc, best)).all(), p
            cur = getattr(rec, f"est_{p}")
            est[p], b = oracle.average(est[p], _i64(new.correlations), oracle.decay(cur.last_update, last[p]))
            last[p] = cur.last_update
            assert (_i64(cur.correlations) == est[p]).all(), p
            assert cur.best_shift == b, p
    assert [recs[-1].new_ab.best_shift, recs[-1].new_ac.best_shift, recs[-1].new_bc.best_shift] == [5, 9, 4]
