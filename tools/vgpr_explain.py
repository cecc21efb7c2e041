#!/usr/bin/env python3
"""Live VGPR/AGPR set at one instruction of a kernel (see vgpr_live.py),
bucketed by where each value was defined and next used.  Diagnostic only.

    python3 tools/vgpr_explain.py kernel.s <mangled-name> <inst-index> [bucket]
"""
import collections
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
import vgpr_live as V  # noqa: E402


def parse(path, name):
    insts = V.explain(path, name, 0)
    parsed = []
    for s in insts:
        op = s.split()[0]
        ops = [o.strip() for o in s[len(op):].split(",")]
        stores = op.startswith(("ds_write", "global_store", "buffer_store", "scratch_store", "s_"))
        if op.startswith("v_cmp") and not op.startswith("v_cmpx"):
            d, u = [], sum((V.regs(o) for o in ops[1:]), [])
        elif stores or not ops or not ops[0]:
            d, u = [], sum((V.regs(o) for o in ops), [])
        else:
            d, u = V.regs(ops[0]), sum((V.regs(o) for o in ops[1:]), [])
            if op.startswith(("v_mac", "v_fmac", "v_dot2c")) or "_dpp" in op:
                u += d
        parsed.append((d, u))
    return insts, parsed


def main():
    path, name, at = sys.argv[1], sys.argv[2], int(sys.argv[3])
    bk = int(sys.argv[4]) if len(sys.argv) > 4 else 250
    insts, parsed = parse(path, name)
    live = set()
    for i in range(len(parsed) - 1, at - 1, -1):
        d, u = parsed[i]
        live -= set(d)
        live |= set(u)
    groups = collections.defaultdict(list)
    for r in live:
        ld = max([i for i in range(at) if r in parsed[i][0]], default=-1)
        nu = min([i for i in range(at, len(parsed)) if r in parsed[i][1]], default=-1)
        groups[(ld // bk * bk, nu // bk * bk)].append((ld, nu, r))
    for k in sorted(groups):
        g = groups[k]
        ld, nu, r = g[0]
        print(f"def~{k[0]:5d} use~{k[1]:5d}: {len(g):3d} regs  e.g. {insts[ld][:44]!r} -> {insts[nu][:44]!r}")
    print("total", len(live))


if __name__ == "__main__":
    main()
