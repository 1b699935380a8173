#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per kernel."""
import csv
import sys
from collections import defaultdict

def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:48]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}   (n={len(v)})")

if __name__ == "__main__":
    main(sys.argv[1:])
