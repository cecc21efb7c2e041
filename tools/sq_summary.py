#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per dispatch of one kernel (diagnostic).

    python tools/sq_summary.py <pmc_dir> <kernel-substring> [out.json]
Every run_counter_collection.csv under <pmc_dir> is read; the first quarter of
the dispatches (warm-up) is dropped."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    src, kname = sys.argv[1], sys.argv[2]
    vals = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    for path in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if kname in r["Kernel_Name"]:
                vals[r["Counter_Name"]][(path, r["Dispatch_Id"])] += float(r["Counter_Value"])
    out = {}
    for c, d in sorted(vals.items()):
        v = [d[k] for k in sorted(d, key=lambda k: (k[0], int(k[1])))]
        v = v[len(v) // 4:]
        out[c] = sum(v) / len(v)
    if "SQ_INSTS_VALU" in out and "SQ_WAVES" in out:
        out["valu_insts_per_wave"] = out["SQ_INSTS_VALU"] / out["SQ_WAVES"]
    if "SQ_INSTS_LDS" in out and "SQ_WAVES" in out:
        out["lds_insts_per_wave"] = out["SQ_INSTS_LDS"] / out["SQ_WAVES"]
    if "SQ_WAVE_CYCLES" in out:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in out:
                out[k + "_frac"] = out[k] / out["SQ_WAVE_CYCLES"]
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")


if __name__ == "__main__":
    main()
