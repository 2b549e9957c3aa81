#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 counter CSVs under one or more directories,
grouped by kernel name (development tool).
usage: tools/pmc_by_kernel.py DIR [DIR ...] [--sub SUBSTRING]"""
import collections
import csv
import glob
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--sub=")]
sub = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--sub=")), "")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in args:
    for f in sorted(glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items()):
    print(k[:150])
    for c in sorted(cs):
        v = cs[c]
        print(f"    {c:24s} n={len(v):3d} avg={sum(v) / len(v):16.1f}")
