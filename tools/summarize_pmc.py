#!/usr/bin/env python3
"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/gpu/run.sh pmc:C:E)
into profiles/hbm_traffic.json: per-launch HBM bytes of each kernel a config
/ engine launch dispatches, keyed "c<config>_<engine>".

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports
half the bytes of a wide (16 B/lane) coalesced streaming read, so read bytes
= 2 * FETCH_SIZE KiB; WRITE_SIZE is exact for 16-B stores (4-8 B stores:
uncalibrated, small).  FETCH_SIZE and WRITE_SIZE come from separate passes.

    python tools/summarize_pmc.py <pmc-dir> <config> <engine> <dominant-kernel> \
        <algorithmic-bytes-per-launch> [profiles/hbm_traffic.json]
"""
import csv
import datetime
import json
import os
import sys
from collections import defaultdict


def per_kernel(path, counter):
    """{kernel name: [value per dispatch]} (warm-up quarter dropped)."""
    vals = defaultdict(list)
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            name = (r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
                    .split("(")[0])
            vals[name].append(float(r["Counter_Value"]))
    return {k: v[len(v) // 4:] for k, v in vals.items() if v[len(v) // 4:]}


def main():
    src, cfg, eng, dom, algo = sys.argv[1:6]
    dst = sys.argv[6] if len(sys.argv) > 6 else "profiles/hbm_traffic.json"
    f = per_kernel(os.path.join(src, f"fetch_c{cfg}_{eng}", "run_counter_collection.csv"), "FETCH_SIZE")
    w = per_kernel(os.path.join(src, f"write_c{cfg}_{eng}", "run_counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        if k.startswith("at::") or "native" in k:
            continue  # torch's own kernels (synthetic data generation)
        rd = 2.0 * 1024.0 * (sum(f.get(k, [0])) / max(1, len(f.get(k, []))))
        wr = 1024.0 * (sum(w.get(k, [0])) / max(1, len(w.get(k, []))))
        kernels[k] = {"hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes": rd + wr,
                      "dispatches": len(f.get(k, []))}
    # the launch's kernels: dispatched once per bench step (a kernel dispatched far
    # fewer times -- the parity report's DIRECT run -- is not part of the launch)
    top = max((v["dispatches"] for v in kernels.values()), default=0)
    total = sum(v["hbm_bytes"] for k, v in kernels.items() if v["dispatches"] and v["dispatches"] * 2 >= top)
    dk = next((v for k, v in kernels.items() if dom in k), None)
    out = json.load(open(dst)) if os.path.exists(dst) else {}
    out["note"] = ("per launch; read = 2 x FETCH_SIZE KiB (gfx950 wide-load correction), write = "
                   "WRITE_SIZE KiB; separate --pmc passes; algorithmic = frames x (M N 2 + 4P + 8)")
    out[f"c{cfg}_{eng}"] = {
        "kernel": dom,
        "date": datetime.date.today().isoformat(),
        "hbm_bytes_per_launch": dk["hbm_bytes"] if dk else None,
        "hbm_bytes_all_kernels_per_launch": total,
        "algorithmic_bytes_per_launch": float(algo),
        "ratio_to_algorithmic": (dk["hbm_bytes"] / float(algo)) if dk else None,
        "kernels": kernels,
    }
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out[f"c{cfg}_{eng}"], indent=1))


if __name__ == "__main__":
    main()
