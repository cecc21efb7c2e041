"""Host-code sanitizers (CPU suite): ASan + UBSan, every report fatal.

`make -C audio-triangulation_amd sanitize` builds tdoa/libtdoa_san.so -- the whole
library with its HOST code instrumented (tdoa_host_path.cpp's per-frame path,
tdoa_reference_abi.cpp's capture ring and geometry, the context setup and table
builders of tdoa_capi.cpp; device code is not, -fno-gpu-sanitize) -- and
`make -C oracle sanitize` the oracle restatement.  Then, in a child process with
clang's sanitizer runtime preloaded:
  * tests/test_ref_host_path.py, test_abi.py and test_reference_loop.py run
    against those builds (the reference's unchanged sample loop is compiled
    with the sanitizers too) and must pass with no report;
  * negative control: an output buffer 24 words short handed to
    tdoa_dpss_q15 must stop the process with a heap-buffer-overflow report;
  * positive control (where /root/reference exists): the reference's own
    buffer.c under UBSan reports its `buf->buffer[i] <<= 8` on a negative
    sample (buffer.c:16, a left shift of a negative value) -- the one expected
    UB site, in oracle/_ref only; the same buffer through libtdoa_san's
    buffer_normalize_range reports nothing (tdoa_host_path.cpp shifts the
    unsigned bit pattern).
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "audio-triangulation_amd")
SAN_LIB = os.path.join(PKG, "tdoa", "libtdoa_san.so")
ORC_SAN = os.path.join(ROOT, "oracle", "liboracle_san.so")
REF_SAN = os.path.join(ROOT, "oracle", "_ref", "libref_components_san.so")
RT = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))

pytestmark = pytest.mark.skipif(not RT or not os.path.exists("/opt/rocm/bin/hipcc"),
                                reason="ROCm clang sanitizer runtime / hipcc missing")


@pytest.fixture(scope="module")
def san_env():
    jobs = os.environ.get("MAX_JOBS", "8")
    for args in (["make", "-C", PKG, f"-j{jobs}", "sanitize"], ["make", "-C", os.path.join(ROOT, "oracle"), "sanitize"]):
        r = subprocess.run(args, capture_output=True, text=True, timeout=1200)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return dict(os.environ, LD_PRELOAD=RT[-1], TDOA_LIB=SAN_LIB, TDOA_ORACLE_LIB=ORC_SAN, TDOA_SAN="1",
                ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
                UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def _reports(text):
    return [ln for ln in text.splitlines() if "AddressSanitizer" in ln or "runtime error:" in ln]


def test_host_paths_clean_under_asan_ubsan(san_env):
    tests = [os.path.join(ROOT, "tests", t) for t in ("test_ref_host_path.py", "test_abi.py", "test_reference_loop.py")]
    r = subprocess.run([sys.executable, "-m", "pytest", *tests, "-m", "not gpu", "-q", "-p", "no:cacheprovider"],
                       env=san_env, capture_output=True, text=True, timeout=900, cwd=ROOT)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert not _reports(out), _reports(out)[:5]
    assert " passed" in r.stdout


CHILD_OVERFLOW = r"""
import ctypes as C, sys
sys.path.insert(0, {pkg!r})
import numpy as np
import tdoa
L = tdoa.load()
assert L._name == {lib!r}, L._name
short = np.zeros(1000, np.int32)
L.tdoa_dpss_q15(1024, 2.0, short.ctypes.data_as(C.c_void_p))
print("no report")
"""


def test_asan_catches_an_overflow(san_env):
    code = CHILD_OVERFLOW.format(pkg=PKG, lib=SAN_LIB)
    r = subprocess.run([sys.executable, "-c", code], env=san_env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "no report" not in r.stdout, r.stdout[-2000:]
    assert "heap-buffer-overflow" in r.stderr, r.stderr[-3000:]


CHILD_SHIFT = r"""
import ctypes as C, sys
sys.path.insert(0, {pkg!r})
import numpy as np
from tdoa import _lib
lib = C.CDLL({lib!r})
b = _lib.Buffer()
x = np.full(1024, -3, np.int16)
C.memmove(b.buffer, x.ctypes.data, 2048)
lib.buffer_normalize_range(C.byref(b))
print("normalized", np.frombuffer(bytes(b.buffer), np.int16)[0])
"""


@pytest.mark.skipif(not os.path.isdir("/root/reference/src/components"), reason="reference sources absent")
def test_ubsan_flags_the_reference_buffer_c16_only(san_env):
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref_san"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and os.path.exists(REF_SAN), r.stdout[-2000:] + r.stderr[-2000:]
    ref = subprocess.run([sys.executable, "-c", CHILD_SHIFT.format(pkg=PKG, lib=REF_SAN)], env=san_env,
                         capture_output=True, text=True, timeout=300)
    assert ref.returncode != 0, ref.stdout
    assert "buffer.c:16" in ref.stderr and "left shift of negative value" in ref.stderr, ref.stderr[-3000:]
    env = dict(san_env)
    ours = subprocess.run([sys.executable, "-c", "import ctypes; ctypes.CDLL(%r).tdoa_ref_set_device(-1)\n" % SAN_LIB
                           + CHILD_SHIFT.format(pkg=PKG, lib=SAN_LIB)], env=env, capture_output=True, text=True,
                          timeout=300)
    assert ours.returncode == 0, ours.stderr[-3000:]
    assert "normalized -768" in ours.stdout and not _reports(ours.stderr)
