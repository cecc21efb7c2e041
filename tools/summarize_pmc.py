#!/usr/bin/env python3
"""Turn rocprofv3 PMC CSVs into profiles/hbm_traffic.json (per-launch HBM
bytes of the dominant kernel of each engine).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports
half the bytes of a wide (16 B/lane) coalesced streaming read, so read bytes
= 2 * FETCH_SIZE KiB; WRITE_SIZE is exact for 16-B stores (our outputs are
4-8 B/lane stores: uncalibrated, small).  FETCH_SIZE and WRITE_SIZE come from
separate --pmc passes.

    python tools/summarize_pmc.py gpurun_out/pmc profiles/hbm_traffic.json
"""
import csv
import json
import os
import sys

KERNELS = {"gcc_phat": "k_phat1024", "direct": "k_direct"}


def per_dispatch(path, counter, kname):
    vals = []
    if not os.path.exists(path):
        return vals
    for r in csv.DictReader(open(path)):
        if kname in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    src, dst = sys.argv[1], sys.argv[2]
    out = {"note": "per launch of 4096 cfg2 frames; read = 2 x FETCH_SIZE KiB (gfx950 wide-load "
                   "correction), write = WRITE_SIZE KiB; algorithmic bytes = 4096 x 6164"}
    for eng, kn in KERNELS.items():
        f = per_dispatch(os.path.join(src, f"fetch_{eng}", "run_counter_collection.csv"), "FETCH_SIZE", kn)
        w = per_dispatch(os.path.join(src, f"write_{eng}", "run_counter_collection.csv"), "WRITE_SIZE", kn)
        if not f:
            continue
        f = f[len(f) // 4:]  # drop warm-up dispatches
        w = w[len(w) // 4:] if w else [0.0]
        rd = 2.0 * 1024.0 * sum(f) / len(f)
        wr = 1024.0 * sum(w) / len(w)
        out[eng] = {"fetch_size_kib": sum(f) / len(f), "write_size_kib": sum(w) / len(w),
                    "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                    "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes_per_launch": 4096 * 6164,
                    "dispatches": len(f)}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
