#!/usr/bin/env python3
"""Code-object audit of libtdoa.so's gfx950 kernels (tests/test_code_objects.py).

    python3 tools/co_audit.py [path/to/libtdoa.so]

The hand-scheduled kernels rest on properties no functional test sees until
they break at run time (DESIGN.md "Code-object guard"):
  * no private segment (scratch) and no register spills -- a spill or a
    byval argument copied to scratch turns LDS / kernarg accesses into flat
    ones and puts 16-wave barrier workgroups behind a scratch allocation;
  * no calls (s_swappc / s_setpc): an out-of-line lambda (the round-5
    k_frame16 variant that stalled) copies the kernel arguments it captures by
    reference into scratch;
  * no flat memory instructions: a flat access counts in both vmcnt and
    lgkmcnt, so every wait for it drains both queues;
  * no scalar load whose SGPR base was formed as X + R with the same R as its
    SGPR offset: gfx950 drops the base's low two address bits (tools/probe/
    smem_sbase_align.hip), so hipcc's split of a 2-byte element address
    kernarg + 2 p into SBASE = kernarg + p, SOFFSET = p reads the wrong dword
    whenever p is not a multiple of 4 -- the round-5 k_frame16 build whose
    compact ranges were wrong (F16_RNG_SCALAR=1 rebuilds it);
  * the trans-use wait state: a VALU instruction reading the VGPR a
    transcendental (v_rsq / v_rcp / v_sqrt / v_exp / v_log / v_sin / v_cos)
    wrote needs one wait state between them on gfx950.  The compiler pads its
    own code, not a consumer inside inline asm (k_frame16's c_unit opens its asm
    multiply with s_nop 0, tdoa_cplx.h), so the disassembly is checked.

The code objects are read straight out of the library's .hip_fatbin bundles
(clang offload bundle format) and examined with the ROCm LLVM tools.
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

import yaml

LLVM = "/opt/rocm/lib/llvm/bin"
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# transcendental VALU ops (gfx950's TRANS unit)
TRANS = re.compile(r"^v_(rsq|rcp|sqrt|exp|log|sin|cos)_(f32|f16|legacy_f32)")
REG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def code_objects(so_path: str) -> list[bytes]:
    """Every gfx950 code object of the offload bundles embedded in a host ELF."""
    data = open(so_path, "rb").read()
    out, i = [], 0
    while True:
        j = data.find(BUNDLE_MAGIC, i)
        if j < 0:
            return out
        n = struct.unpack_from("<Q", data, j + 24)[0]
        p = j + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if "gfx950" in triple and size:
                out.append(data[j + off:j + off + size])
        i = j + len(BUNDLE_MAGIC)


def _tool(args: list[str]) -> str:
    return subprocess.run(args, check=True, capture_output=True, text=True).stdout


def kernel_metadata(co_path: str) -> dict[str, dict]:
    """name -> the kernel's AMDGPU metadata (private segment, spills, VGPRs ...)."""
    txt = _tool([f"{LLVM}/llvm-readelf", "--notes", co_path])
    start = txt.index("---")
    start = txt.index("\n", start) + 1
    end = txt.index("\n...", start)
    meta = yaml.safe_load(txt[start:end])
    return {k[".name"]: k for k in meta.get("amdhsa.kernels", [])}


def disassembly(co_path: str) -> dict[str, list[str]]:
    """symbol -> its instructions (mnemonic + operands), in address order."""
    txt = _tool([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "--no-leading-addr", co_path])
    funcs, cur = {}, None
    for line in txt.splitlines():
        m = re.match(r"^<(.+)>:$", line.strip())
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        s = line.split("//")[0].strip()
        if cur is not None and s and not s.endswith(":"):
            cur.append(s)
    return funcs


def _regs(operand: str) -> set[int]:
    r = set()
    for m in REG.finditer(operand):
        if m.group(1) is not None:
            r.add(int(m.group(1)))
        else:
            r.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return r


def trans_use_violations(insts: list[str]) -> list[str]:
    """Trans results read by the very next VALU instruction (no wait state)."""
    bad = []
    for a, b in zip(insts, insts[1:]):
        op_a = a.split()[0]
        if not TRANS.match(op_a):
            continue
        ops_a = a[len(op_a):].split(",")
        dst = _regs(ops_a[0])
        op_b = b.split()[0]
        if not op_b.startswith("v_") or TRANS.match(op_b):
            continue
        ops_b = [o.strip() for o in b[len(op_b):].split(",")]
        # sources; accumulate forms (mac / fmac) and DPP moves also read the destination
        srcs = ops_b if ("mac" in op_b or "dpp" in op_b) else ops_b[1:]
        if any(dst & _regs(o) for o in srcs):
            bad.append(f"{a}  ->  {b}")
    return bad


SMEM_SOE = re.compile(r"^s_(?:load|buffer_load)_dword\w*\s+\S+,\s*s\[(\d+):\d+\],\s*s(\d+)\s+offset:")


def smem_split_index(insts: list[str], window: int = 48) -> list[str]:
    """Scalar loads whose base SGPR pair was last written by s_add_u32 of the
    same SGPR that serves as the load's offset (SBASE = X + R, SOFFSET = R)."""
    bad = []
    for i, s in enumerate(insts):
        m = SMEM_SOE.match(s)
        if not m:
            continue
        base, off = int(m.group(1)), int(m.group(2))
        for t in reversed(insts[max(0, i - window):i]):
            mt = re.match(r"^s_\w+\s+s(\d+)\b(.*)", t)
            if not mt or int(mt.group(1)) != base:
                continue
            ma = re.match(r"^s_add_u32\s+s\d+,\s*(\S+),\s*(\S+)", t)
            if ma and f"s{off}" in (ma.group(1), ma.group(2)):
                bad.append(f"{t}  ->  {s}")
            break
    return bad


def audit(so_path: str) -> dict[str, dict]:
    """Per kernel: metadata and the ISA findings."""
    res = {}
    with tempfile.TemporaryDirectory() as td:
        for n, co in enumerate(code_objects(so_path)):
            path = os.path.join(td, f"co{n}.elf")
            open(path, "wb").write(co)
            meta = kernel_metadata(path)
            dis = disassembly(path)
            for name, md in meta.items():
                insts = dis.get(name, [])
                res[name] = {
                    "private_segment": int(md.get(".private_segment_fixed_size", 0)),
                    "dynamic_stack": bool(md.get(".uses_dynamic_stack", False)),
                    "vgpr_spill": int(md.get(".vgpr_spill_count", 0)),
                    "sgpr_spill": int(md.get(".sgpr_spill_count", 0)),
                    "vgprs": int(md.get(".vgpr_count", 0)),
                    "instructions": len(insts),
                    "calls": sum(1 for s in insts if s.startswith(("s_swappc", "s_setpc", "s_call"))),
                    "flat": sum(1 for s in insts if s.startswith("flat_")),
                    "scratch": sum(1 for s in insts if s.startswith("scratch_")),
                    "trans_use": trans_use_violations(insts),
                    "smem_split": smem_split_index(insts),
                    "functions": len(dis) - len(meta),
                }
    return res


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-triangulation_amd", "tdoa", "libtdoa.so")
    for name, r in sorted(audit(so).items()):
        flag = "" if not (r["private_segment"] or r["calls"] or r["flat"] or r["trans_use"] or r["smem_split"]) \
            else "  <--"
        print(f"{name[:90]:90s} priv {r['private_segment']:4d} spill {r['vgpr_spill']:2d}/{r['sgpr_spill']:3d} "
              f"vgpr {r['vgprs']:3d} calls {r['calls']} flat {r['flat']:3d} trans-use {len(r['trans_use'])} "
              f"smem-split {len(r['smem_split'])}{flag}")
        for v in (r["trans_use"] + r["smem_split"])[:4]:
            print("    ", v)


if __name__ == "__main__":
    main()
