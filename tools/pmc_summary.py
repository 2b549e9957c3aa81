#!/usr/bin/env python3
"""Per-dispatch summary of rocprofv3 counter CSVs (development tool).
usage: tools/pmc_summary.py DIR [kernel-substring]  -- every *_counter_collection.csv under DIR"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "tally"
for f in sorted(glob.glob(f"{d}/**/*_counter_collection.csv", recursive=True)):
    per = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if sub not in r["Kernel_Name"]:
            continue
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0][-60:])
        per.setdefault(k, {"grid": r["Grid_Size"], "vgpr": r["VGPR_Count"], "sgpr": r["SGPR_Count"],
                           "lds": r["LDS_Block_Size"]})[r["Counter_Name"]] = float(r["Counter_Value"])
    print("#", f)
    for (did, name), v in per.items():
        extra = {k: v[k] for k in ("grid", "vgpr", "sgpr", "lds")}
        cnt = {k: v[k] for k in v if k not in extra}
        print(did, name, extra, " ".join(f"{k}={cnt[k]:.4g}" for k in sorted(cnt)))
