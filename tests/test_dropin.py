"""Drop-in check of the north star's boundary: the reference's OWN sample
loop -- src/sample_compute.h, unchanged, with the reference's component
headers -- compiles against include/'s ABI and links against libtdoa.so
alone for every component symbol (rolling_buffer_*, buffer_*, correlations_*),
with host/pico_host/ replacing the Pico SDK side (capture, clock, protothread
primitives).  Link check; tests/test_reference_loop.py RUNS the same program on
libtdoa's host path and checks every hand-off against the oracle.  Skipped where
the reference is absent (the GPU box); nothing built here is shipped.
The reference's component .c files are NOT compiled: libtdoa provides them."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG

REF = "/root/reference/src"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "sample_compute.h")),
                    reason="reference sources not present (GPU box)")
def test_unchanged_sample_compute_links_against_libtdoa(tmp_path):
    lib = os.path.join(PKG, "tdoa", "libtdoa.so")
    if not os.path.exists(lib):
        pytest.skip("libtdoa.so not built")
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    exe = tmp_path / "sample_compute_host"
    cmd = ["gcc", "-std=gnu11", "-O2", "-w", "-I", os.path.join(PKG, "host", "pico_host"),
           "-I", REF, os.path.join(PKG, "host", "sample_compute_main.c"),
           "-L", os.path.join(PKG, "tdoa"), "-ltdoa", "-L/opt/rocm/lib", "-lamdhip64", "-lm",
           "-Wl,--no-undefined", "-Wl,-rpath," + os.path.join(PKG, "tdoa"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    # every reference component symbol the loop calls is undefined in the
    # executable and resolved by libtdoa.so (not by a copy of the reference)
    und = subprocess.run(["nm", "-u", str(exe)], capture_output=True, text=True).stdout
    need = ["rolling_buffer_init", "rolling_buffer_push", "rolling_buffer_write_out",
            "rolling_buffer_get_incoming_power", "rolling_buffer_get_outgoing_power",
            "buffer_normalize_range", "buffer_window", "correlations_init",
            "correlations_average"]
    for s in need:
        assert s in und, f"{s} is not imported from libtdoa"
    exports = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True,
                             text=True).stdout
    for s in need:
        assert f" T {s}" in exports, s
