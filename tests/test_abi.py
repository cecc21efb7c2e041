"""CPU-side checks of libtdoa.so: it loads, exports every symbol include/*.h
declares, and its host-only pieces (DPSS window generator, decay, capture
ring, microphone geometry) match the oracle / reference fixtures.  No kernel
runs here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden

import tdoa
from tdoa import _lib


def _declared_symbols():
    names = set()
    for h in ("tdoa.h", "tdoa_reference_abi.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        txt = re.sub(r"//[^\n]*", "", txt)
        txt = re.sub(r"#[^\n]*", "", txt)
        for m in re.finditer(r"\b([A-Za-z_]\w*)\s*\(([^;{}]*)\)\s*;", txt):
            name = m.group(1)
            if name in ("sizeof",):
                continue
            # skip function-pointer parameters like (*now_us)(void)
            names.add(name)
        for m in re.finditer(r"extern\s+\w+\s+(\w+)\s*;", txt):
            names.add(m.group(1))
    names.discard("now_us")
    return names


def test_library_loads_and_exports_all_declared_symbols():
    L = tdoa.load()
    declared = _declared_symbols()
    assert len(declared) >= 25
    missing = [n for n in sorted(declared) if not hasattr(L, n)]
    assert not missing, f"libtdoa.so lacks {missing}"
    assert declared <= set(_lib.EXPORTED_SYMBOLS) | {"now_us"}
    assert L.tdoa_abi_version() == 1


def test_config_defaults_match_reference_constants():
    cfg = _lib.Config()
    tdoa.load().tdoa_config_default(C.byref(cfg))
    assert (cfg.num_mics, cfg.frame_len, cfg.sample_rate_hz) == (3, 1024, 50000)
    assert (cfg.grid_half_w, cfg.grid_half_h) == (50, 50)
    assert cfg.grid_scale == np.float32(24.0) and cfg.height_offset == np.float32(1.2)
    assert cfg.speed_of_sound == np.float32(343.0)


@pytest.mark.parametrize("n", [256, 512, 1024, 2048, 4096])
def test_dpss_generator_matches_notebook_procedure(n):
    assert (tdoa.dpss_q15(n) == golden("window_q15.npz")[f"n{n}"]).all()


def test_decay_matches_oracle(oracle):
    rng = np.random.default_rng(1)
    for _ in range(500):
        last = int(rng.integers(0, 1 << 40))
        now = last + int(rng.integers(0, 5_000_000))
        assert np.float32(tdoa.decay_us(now, last)) == np.float32(oracle.decay(now, last))
    assert tdoa.decay_us(123, 0) == np.float32(oracle.decay(123, 0))


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    cfg = _lib.Config()
    L = tdoa.load()
    L.tdoa_config_default(C.byref(cfg))
    ctx = C.c_void_p()
    rc = L.tdoa_create(C.byref(cfg), 0, C.byref(ctx))
    assert rc == -3 and not ctx.value
    assert b"no HIP device" in L.tdoa_last_error()
    with pytest.raises(tdoa.TdoaError):
        tdoa.Localizer()


def test_create_rejects_bad_config():
    L = tdoa.load()
    cfg = _lib.Config()
    L.tdoa_config_default(C.byref(cfg))
    cfg.frame_len = 1000
    ctx = C.c_void_p()
    assert L.tdoa_create(C.byref(cfg), 0, C.byref(ctx)) == -1
    assert b"power of two" in L.tdoa_last_error()
    L.tdoa_config_default(C.byref(cfg))
    cfg.num_mics = 4  # needs mic_xy
    assert L.tdoa_create(C.byref(cfg), 0, C.byref(ctx)) == -1


def test_host_microphones_init_matches_reference_fixture():
    L = tdoa.load()
    L.microphones_init()
    got = np.array([[_lib.Point2d.in_dll(L, n).x, _lib.Point2d.in_dll(L, n).y]
                    for n in ("mic_a_location", "mic_b_location", "mic_c_location")], np.float32)
    assert (got == golden("ref_components.npz")["mics"]).all()


def test_host_capture_ring_matches_reference_fixture():
    g = golden("ref_components.npz")
    L = tdoa.load()
    rb = _lib.RollingBuffer()
    L.rolling_buffer_init(C.byref(rb))
    for i, v in enumerate(g["pushes"]):
        L.rolling_buffer_push(C.byref(rb), int(v))
        assert L.rolling_buffer_get_incoming_power(C.byref(rb)) == g["incoming_power"][i]
        assert L.rolling_buffer_get_outgoing_power(C.byref(rb)) == g["outgoing_power"][i]
        assert rb.head == g["heads"][i]
    assert C.sizeof(_lib.RollingBuffer) == 2096
    assert C.sizeof(_lib.Buffer) == 2056 and C.sizeof(_lib.Correlations) == 760
