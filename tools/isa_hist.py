#!/usr/bin/env python3
"""Static opcode-class histogram of one kernel, per phase.  Diagnostic only.

    python3 tools/isa_hist.py kernel.s <mangled-name> [--split s_memtime]

Phases are the stretches between consecutive occurrences of the split
instruction (the diagnostic build's phase stamps), so the same source built
with -DTDOA_DIAG gives the per-phase view; without stamps the whole kernel is
one phase.  Loop bodies count once (static), so a phase with a loop reports
its body -- say which in the profile that quotes it.
"""
import collections
import re
import sys

CLASSES = [
    ("pk_fma", r"^v_pk_fma_f32"),
    ("pk_mul", r"^v_pk_mul_f32"),
    ("pk_add", r"^v_pk_add_f32"),
    ("pk_mov", r"^v_pk_mov_b32"),
    ("dpp_mov", r"^v_mov_b32_dpp|^v_mov_b64_dpp"),
    ("dpp_alu", r"_dpp$|_dpp "),
    ("mov", r"^v_mov_b32|^v_mov_b64"),
    ("cndmask", r"^v_cndmask"),
    ("cmp", r"^v_cmp"),
    ("transc", r"^v_(rsq|rcp|sqrt|exp|log|sin|cos)_f32"),
    ("f32_fma", r"^v_(fma|fmac|mac|mad)_f32"),
    ("f32_mul", r"^v_mul_f32"),
    ("f32_add", r"^v_(add|sub|subrev)_f32"),
    ("f32_minmax", r"^v_(max|min|max3|min3)_f32"),
    ("floor_cvt", r"^v_(floor|cvt|trunc|rndne)"),
    ("int", r"^v_(add|sub|lshl|lshr|ashr|and|or|xor|bfe|bfi|mul_lo|mul_hi|mad|perm|alignbit|"
            r"alignbyte|not|min_i|max_i|min_u|max_u|sad|lshl_add|add_lshl|or3|and_or|xad|"
            r"add3|dot|sdot|udot|med3_i|med3_u|bcnt|ffbh|ffbl|readlane|readfirstlane|writelane)"),
    ("valu_other", r"^v_"),
    ("ds_read", r"^ds_read|^ds_load"),
    ("ds_write", r"^ds_write|^ds_store"),
    ("ds_other", r"^ds_"),
    ("global_load", r"^(global|buffer|flat)_load"),
    ("global_store", r"^(global|buffer|flat)_store"),
    ("s_nop", r"^s_nop"),
    ("s_waitcnt", r"^s_waitcnt"),
    ("salu", r"^s_"),
]


def cls(op):
    for name, pat in CLASSES:
        if re.search(pat, op):
            return name
    return "other"


def kernel_lines(path, name):
    out, on = [], False
    for line in open(path):
        if line.startswith(name + ":"):
            on = True
            continue
        if on:
            if line.startswith(".Lfunc_end") or line.strip().startswith(".end_amdhsa_kernel") \
                    or line.startswith("\t.size"):
                break
            s = line.strip()
            if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
                continue
            out.append(s.split(";")[0].strip())
    return out


def main():
    path, name = sys.argv[1], sys.argv[2]
    split = "s_memtime"
    if "--split" in sys.argv:
        split = sys.argv[sys.argv.index("--split") + 1]
    insts = kernel_lines(path, name)
    phases, cur = [], collections.Counter()
    for s in insts:
        op = s.split()[0]
        if op == split:
            phases.append(cur)
            cur = collections.Counter()
            continue
        cur[cls(op)] += 1
    phases.append(cur)
    keys = [c for c, _ in CLASSES] + ["other"]
    used = [k for k in keys if any(p[k] for p in phases)]
    hdr = "phase " + " ".join(f"{k[:9]:>9s}" for k in used) + "      VALU"
    print(hdr)
    tot = collections.Counter()
    valu_keys = [k for k in used if k not in ("ds_read", "ds_write", "ds_other", "global_load",
                                               "global_store", "s_nop", "s_waitcnt", "salu", "other")]
    for i, p in enumerate(phases):
        tot.update(p)
        print(f"{i:5d} " + " ".join(f"{p[k]:9d}" for k in used) + f" {sum(p[k] for k in valu_keys):9d}")
    print("total " + " ".join(f"{tot[k]:9d}" for k in used) + f" {sum(tot[k] for k in valu_keys):9d}")


if __name__ == "__main__":
    main()
