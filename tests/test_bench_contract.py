"""bench.py's contract pieces that need no GPU: the BASELINE configs it
measures, its defaults (config 2 GCC-PHAT, N = 1, K / W that finish in
minutes), and the `roofline.traffic` wiring -- PMC bytes are attached only for
the kernels a run dispatches, configs 3 / 4 sum their two kernels, config 5
sums the hop's three."""
import json
import os
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _args(*argv):
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


def test_configs_are_baseline_shapes():
    c = bench.CONFIGS
    assert (c[1]["M"], c[1]["N"]) == (2, 1024)
    assert (c[2]["M"], c[2]["N"], c[2]["batch"]) == (3, 1024, 4096)
    assert (c[3]["M"], c[3]["N"], c[3]["batch"]) == (4, 4096, 65536)
    assert (c[4]["M"], c[4]["N"], c[4]["batch"], c[4]["scaling"]) == (8, 2048, 1_000_000, "strong")
    assert (c[5]["hop"], c[5]["fs"], c[5]["batch"]) == (512, 48000, 16384)


def test_defaults_are_the_headline_run():
    a = _args()
    assert (a.config, a.engine, a.gpus, a.batch) == (2, "gcc_phat", 1, 4096)
    assert a.steps >= 100 and a.warmup >= 1
    assert _args("--config", "5").engine == "direct"
    assert _args("--config", "1").engine == "direct"
    # the untimed preflight is on by default and can be switched off
    assert a.preflight_s > 0 and _args("--preflight-s", "0").preflight_s == 0


def test_traffic_only_for_dispatched_kernels():
    tj = json.load(open(os.path.join(ROOT, "profiles", "hbm_traffic.json")))
    t2, src = bench.traffic_entry(_args())
    assert t2 == tj["c2_gcc_phat"]["hbm_bytes_per_launch"] and "k_p1k_lean" in src
    # a kernel the committed passes were not taken on: no traffic figure
    real = bench.dominant_kernel
    bench.dominant_kernel = lambda config, engine, first="", fused=True: "k_not_profiled"
    try:
        assert bench.traffic_entry(_args()) == (None, None)
    finally:
        bench.dominant_kernel = real
    for cfg in (3, 4):
        ks = tj[f"c{cfg}_gcc_phat"]["kernels"]
        with_grid = any(k.startswith("k_grid") for k in ks)
        for fused in (False, True):
            t, src = bench.traffic_entry(_args("--config", str(cfg)), "", fused)
            if fused and with_grid:  # a pass with the separate grid kernel is not a fused launch's traffic
                assert (t, src) == (None, None)
            elif not fused and not with_grid:  # (and the reverse)
                assert t is None
            elif fused:
                want = sum(v["hbm_bytes"] for k, v in ks.items() if k.split("<")[0] == "k_frame16")
                assert t == want and "k_frame16" in src and "k_grid_bb" not in src
            else:
                want = sum(v["hbm_bytes"] for k, v in ks.items() if k.split("<")[0] in ("k_frame16", "k_grid_bb"))
                assert t == want and "k_frame16 + k_grid_bb" in src
    t5, src5 = bench.stream_traffic(_args("--config", "5"))
    ks = tj["c5_direct"]["kernels"]
    assert t5 == sum(v["hbm_bytes"] for k, v in ks.items()
                     if k.split("<")[0] in ("k_stream_trigger_p", "k_direct_mfma", "k_stream_update"))
    assert "k_stream_trigger_p + k_direct_mfma" in src5
    # algorithmic bytes: traffic within a small factor (no silent re-reads on config 2)
    assert t2 < 1.1 * 4096 * (3 * 1024 * 2 + 4 * 3 + 8)
