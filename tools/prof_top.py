#!/usr/bin/env python3
"""Per-step kernel time table from a rocprofv3 --stats kernel_stats.csv: python tools/prof_top.py CSV [steps] [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 7.0
n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = sum(float(x["TotalDurationNs"]) for x in rows)
print(f"total {tot / steps / 1e6:.3f} ms/step")
for x in rows[:n]:
    print(f"{float(x['TotalDurationNs']) / steps / 1e6:7.3f} ms {int(x['Calls']) / steps:5.1f} x {float(x['AverageNs']) / 1e3:8.1f} us  "
          f"{x['Name'][:95]}")
