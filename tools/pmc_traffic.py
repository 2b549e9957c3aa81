#!/usr/bin/env python3
"""HBM traffic per launch of the dominant tally kernel from two rocprofv3 PMC
passes (FETCH_SIZE, WRITE_SIZE; separate runs of the same bench command).

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of wide coalesced streaming reads -> x2; WRITE_SIZE is taken as is.
Both counters are in KB.

usage: tools/pmc_traffic.py FETCH.csv WRITE.csv CONFIG OUT.json [kernel-substring]
"""
import csv
import json
import statistics
import sys


def per_launch(path, counter, sub):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and sub in r["Kernel_Name"]]
    return statistics.median(vals), len(vals)


def main():
    fetch_csv, write_csv, config, out = sys.argv[1:5]
    sub = sys.argv[5] if len(sys.argv) > 5 else "tally_kernel<false"
    f_kb, nf = per_launch(fetch_csv, "FETCH_SIZE", sub)
    w_kb, nw = per_launch(write_csv, "WRITE_SIZE", sub)
    rec = {"config": config, "kernel_match": sub, "launches": [nf, nw],
           "fetch_bytes": 2.0 * f_kb * 1024.0, "write_bytes": w_kb * 1024.0,
           "traffic_bytes": 2.0 * f_kb * 1024.0 + w_kb * 1024.0,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read halving), WRITE_SIZE x1, KB->B x1024",
           "sources": [fetch_csv, write_csv]}
    try:
        data = json.load(open(out))
    except (OSError, ValueError):
        data = {}
    data[config] = rec
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
