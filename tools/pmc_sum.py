#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 counter CSVs under a directory (development tool).
usage: tools/pmc_sum.py DIR [kernel-substring] [units-per-launch]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
units = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
agg = collections.defaultdict(list)
for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(agg):
    v = agg[k]
    avg = sum(v) / len(v)
    extra = f"  per unit {avg / units:10.2f}" if units else ""
    print(f"{k:24s} n={len(v):3d} avg={avg:16.1f}{extra}")
for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
        print(f'{int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:10.1f} us  {r["Name"][:100]}')
