#!/usr/bin/env python3
"""Fold a `tools/gpu/run.sh calib` run (tools/hbm_copy: event-timed JSON line and
the rocprofv3 --kernel-trace --stats summary of the same run) into
profiles/r05_hbm_calibration.json, the achievable-HBM denominators bench.py uses.

    python tools/summarize_calib.py gpurun_out/<TAG> [profiles/r05_hbm_calibration.json]
"""
import csv
import json
import os
import sys


def main():
    src = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else "profiles/r05_hbm_calibration.json"
    ev = json.loads(open(os.path.join(src, "calib.json")).read().strip().splitlines()[-1])
    avg = {}
    for r in csv.DictReader(open(os.path.join(src, "calib_kt", "run_kernel_stats.csv"))):
        name = r["Name"].split("(")[0].replace("void ", "").strip()
        avg[name] = float(r["AverageNs"])
    cb, rb = ev["copy_bytes_per_launch"], ev["read_bytes_per_launch"]
    out = {
        "tool": "tools/hbm_copy.hip (make -C audio-triangulation_amd calib), 1 GiB buffers, 20 launches each; "
                "k_copy16: nontemporal 16-B loads/stores, 8 x 256-thread workgroups per CU; k_copy16p: "
                "default-policy 16-B loads/stores, 4 per CU; k_read16: nontemporal 16-B read sweep",
        "events": ev,
        "rocprof_avg_ns": avg,
        "copy_gbs_rocprof": cb / avg["k_copy16"] if "k_copy16" in avg else None,
        "copy_plain_gbs_rocprof": cb / avg["k_copy16p"] if "k_copy16p" in avg else None,
        "read_gbs_rocprof": rb / avg["k_read16"],
        "note": "copy counts read + write bytes; the config-2..4 kernels are read-dominated, so bench.py "
                "prices them against the read sweep (frac_achievable); MI355X_MICROARCH.md quotes "
                "~6.3 TB/s achievable for a float4 copy",
        "date": "round 5",
    }
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
