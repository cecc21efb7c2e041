"""Code-object guard (CPU suite): the gfx950 kernels inside the built libtdoa.so.

The hand-scheduled kernels depend on properties no numerical test sees until
they fail at run time (DESIGN.md "Code-object guard"; tools/co_audit.py reads
the code objects out of the library's offload bundles):
  * no private segment, no spills, no calls -- the round-5 k_frame16 build
    whose lagged-epilogue lambda fell out of line (688 B of scratch, calls, flat
    accesses) stalled; the lambdas are forced inline since;
  * no flat memory instructions (a flat access waits on both vmcnt and lgkmcnt);
  * one wait state between a transcendental's result and the VALU reading it:
    the compiler does not pad ahead of inline asm, and k_frame16's c_unit
    (tdoa_cplx.h) carries its own s_nop 0 -- without it the results are wrong;
  * no scalar load with SBASE = X + R and SOFFSET = R: gfx950 drops the SGPR
    base's low two address bits (tools/probe/smem_sbase_align.hip), and hipcc
    splits a 2-byte kernel-argument element's address that way -- the round-5
    k_frame16 build with wrong compact offsets (F16_RNG_SCALAR=1).
The last test rebuilds k_frame16's translation unit with the known bad forms
(no s_nop, lambdas left to the inliner; the scalar range pick) and checks the
guard flags each, so a green run means the checks look at real code.
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import co_audit as A  # noqa: E402

PKG = os.path.join(ROOT, "audio-triangulation_amd")
LIB = os.path.join(PKG, "tdoa", "libtdoa.so")
AB_LIB = os.path.join(PKG, "tdoa", "libtdoa_ab.so")
HIPCC = "/opt/rocm/bin/hipcc"

# the kernels bench.py times and the GPU parity tests hold to the oracle
HOT = ("k_p1k_lean", "k_frame16I", "k_grid_bbI", "k_direct_mfmaI", "k_stream_trigger_pI", "k_lsI")

pytestmark = pytest.mark.skipif(not os.path.exists(f"{A.LLVM}/llvm-objdump"), reason="ROCm LLVM tools missing")


def _clean(r):
    return {k: r[k] for k in ("private_segment", "dynamic_stack", "vgpr_spill", "calls", "flat", "scratch")
            if r[k]} | {k: r[k][:2] for k in ("trans_use", "smem_split") if r[k]}


@pytest.fixture(scope="module")
def prod():
    assert os.path.exists(LIB), "build libtdoa.so first (__graft_entry__.build)"
    return A.audit(LIB)


def test_every_hot_kernel_is_clean(prod):
    for pat in HOT:
        names = [n for n in prod if pat in n]
        assert names, f"no {pat} kernel in libtdoa.so"
        for n in names:
            assert not _clean(prod[n]), (n, _clean(prod[n]))
            assert prod[n]["instructions"] > 100, n


def test_no_product_kernel_needs_scratch_calls_or_flat(prod):
    bad = {n: _clean(r) for n, r in prod.items() if _clean(r)}
    assert not bad, bad


def test_product_holds_only_dispatched_kernels(prod):
    """The A/B kernels that measured slower live in tdoa/libtdoa_ab.so only."""
    assert not [n for n in prod if "k_p1k_w64" in n or "k_frame16w" in n]
    # k_frame16<C, M, DM, XS, FG>: no fused-grid (FG = true) instantiation
    assert not [n for n in prod if "k_frame16I" in n and re.search(r"ELb1ELb1EEEv", n)]
    if os.path.exists(AB_LIB):
        ab = A.audit(AB_LIB)
        assert [n for n in ab if "k_p1k_w64" in n] and [n for n in ab if "k_frame16w" in n]
        assert [n for n in ab if "k_frame16I" in n and re.search(r"ELb1ELb1EEEv", n)]
        # the A/B library's copies of the product kernels are as clean
        for pat in HOT:
            for n in ab:
                if pat in n and not re.search(r"ELb1ELb1EEEv", n):
                    assert not _clean(ab[n]), (n, _clean(ab[n]))


def test_trans_use_check_on_known_sequences():
    rsq = "v_rsq_f32_e32 v14, v15"
    assert A.trans_use_violations([rsq, "v_pk_mul_f32 v[16:17], v[12:13], v[14:15] op_sel_hi:[1,0]"])
    assert A.trans_use_violations([rsq, "v_fmac_f32_e32 v14, v1, v2"])  # reads its destination
    assert A.trans_use_violations([rsq, "v_mul_f32_e32 v3, v14, v2"])
    assert not A.trans_use_violations([rsq, "s_nop 0", "v_mul_f32_e32 v3, v14, v2"])
    assert not A.trans_use_violations([rsq, "v_mul_f32_e32 v3, v1, v2", "v_mul_f32_e32 v4, v14, v2"])
    assert not A.trans_use_violations([rsq, "v_mov_b32_e32 v14, 0"])  # overwrites, reads nothing
    assert not A.trans_use_violations([rsq, "v_rsq_f32_e32 v16, v14"])  # trans -> trans


BAD_BUILDS = {
    # the asm multiply's s_nop removed and the epilogue lambdas left to the inliner
    "nop_and_inline": ['-DTDOA_UNIT_NOP=""', "-DF16_LAMBDA_AI=0"],
    # the compact ranges picked from the wave's scalar loads
    "scalar_pick": ["-DF16_RNG_SCALAR=1"],
}


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc missing")
@pytest.mark.parametrize("build", sorted(BAD_BUILDS))
def test_guard_catches_the_known_bad_builds(tmp_path, build):
    """k_frame16's translation unit rebuilt with a known bad form: the guard
    must see the trans-use hazard, the calls, the scratch and the flat
    accesses (nop_and_inline), or the split-index scalar loads (scalar_pick),
    in config 4's k_frame16."""
    obj = tmp_path / "r16_bad.o"
    cmd = [HIPCC, "-O3", "-std=c++17", "-ffp-contract=fast", "--offload-arch=gfx950", "--cuda-device-only",
           f"-I{ROOT}/include", f"-I{PKG}/csrc", *BAD_BUILDS[build], "-c",
           os.path.join(PKG, "csrc", "tdoa_phat_r16.hip"), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    bad = A.audit(str(obj))
    k4 = [n for n in bad if "k_frame16ILi2048ELi8ELi1E" in n]
    assert k4
    for n in k4:
        if build == "nop_and_inline":
            assert bad[n]["trans_use"], n
            assert bad[n]["calls"] and bad[n]["private_segment"] > 0 and bad[n]["flat"] > 0, (n, _clean(bad[n]))
        else:
            assert bad[n]["smem_split"], n
            assert not bad[n]["trans_use"] and not bad[n]["calls"], (n, _clean(bad[n]))
    shutil.rmtree(tmp_path, ignore_errors=True)
