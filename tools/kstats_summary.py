#!/usr/bin/env python3
"""Print libtdoa kernels' call counts and average durations from rocprofv3
--stats directories (run_kernel_stats.csv)."""
import csv
import os
import sys

for d in sys.argv[1:]:
    print("==", os.path.basename(d))
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
        n = r["Name"]
        if "at::native" in n or "rocclr" in n:
            continue
        short = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        print(f"  {short[:48]:48s} calls={int(r['Calls']):6d} avg_us={float(r['AverageNs'])/1e3:9.2f}"
              f" total_ms={float(r['TotalDurationNs'])/1e6:9.2f}")
