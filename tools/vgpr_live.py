#!/usr/bin/env python3
"""Approximate VGPR/AGPR liveness profile of one kernel in a hipcc -S file.

    python3 tools/vgpr_live.py kernel.s <mangled-kernel-name> [--top N]

Backward scan over the kernel's instruction stream treated as straight-line
code (branches ignored, so loop-carried values show up only where they are
used): live = (live - defs) | uses.  Prints the pressure peaks with the
nearest preceding source-line comment and a running count of DS / VMEM
instructions, which is enough to tell which phase of an unrolled FFT kernel
holds the most registers.  Diagnostic only.
"""
import re
import sys

REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)\b)")


def regs(tok):
    out = []
    for m in REG.finditer(tok):
        k = m.group(1)
        if m.group(4) is not None:
            out.append((k, int(m.group(4))))
        else:
            out += [(k, r) for r in range(int(m.group(2)), int(m.group(3)) + 1)]
    return out


def main():
    path, name = sys.argv[1], sys.argv[2]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 12
    txt = open(path).read()
    a = txt.index(name + ":")
    b = txt.index(".Lfunc_end", a)
    lines = txt[a:b].splitlines()
    insts = []
    loc = ""
    nds = nvm = 0
    for l in lines:
        s = l.strip()
        if s.startswith(";") and ".hip:" in s:
            loc = s
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        s = s.split(";")[0].strip()
        op = s.split()[0]
        if op.startswith("ds_"):
            nds += 1
        if op.startswith(("global_", "buffer_", "scratch_")):
            nvm += 1
        ops = s[len(op):].split(",")
        ops = [o.strip() for o in ops]
        stores = op.startswith(("ds_write", "global_store", "buffer_store", "scratch_store",
                                "s_", "ds_store")) or op in ("s_nop",)
        if op.startswith("v_cmp") and not op.startswith("v_cmpx"):
            # VOPC: first operand is an SGPR/vcc destination
            defs, uses = [], sum((regs(o) for o in ops[1:]), [])
        elif stores or not ops or not ops[0]:
            defs, uses = [], sum((regs(o) for o in ops), [])
        else:
            defs, uses = regs(ops[0]), sum((regs(o) for o in ops[1:]), [])
            if op.startswith(("v_mac", "v_fmac", "v_dot2c")) or "_dpp" in op:
                uses += defs  # read-modify-write
        insts.append((op, defs, uses, loc, nds, nvm, s))
    live = set()
    prof = [0] * len(insts)
    for i in range(len(insts) - 1, -1, -1):
        op, defs, uses, *_ = insts[i]
        live -= set(defs)
        live |= set(uses)
        prof[i] = len(live)
    order = sorted(range(len(prof)), key=lambda i: -prof[i])
    shown = []
    for i in order:
        if any(abs(i - j) < 40 for j in shown):
            continue
        shown.append(i)
        op, _, _, loc, nds, nvm, s = insts[i]
        print(f"{prof[i]:4d} live @ inst {i:5d} ds#{nds:4d} vmem#{nvm:3d}  {s[:48]:48s} {loc[-60:]}")
        if len(shown) >= top:
            break
    print("max", max(prof), "instructions", len(insts))


if __name__ == "__main__":
    main()


def explain(path, name, at):
    """Registers live at instruction `at`, grouped by the instruction that
    defined them (the last def before `at`) and their next use."""
    txt = open(path).read()
    a = txt.index(name + ":")
    b = txt.index(".Lfunc_end", a)
    insts = []
    for l in txt[a:b].splitlines():
        s = l.strip()
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        s = s.split(";")[0].strip()
        insts.append(s)
    return insts
