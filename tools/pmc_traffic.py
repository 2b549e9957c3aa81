#!/usr/bin/env python3
"""HBM traffic per launch of every engine kernel of a bench workload, from two
rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs of the same bench
command), into profiles/traffic.json under the workload's name.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of wide coalesced streaming reads -> x2; WRITE_SIZE is taken as is.
Both counters are in KB.  (The u8 columns are read 4 B per lane: an access width
the guide leaves uncalibrated; the x2 is applied to the whole FETCH_SIZE.)

usage: tools/pmc_traffic.py FETCH.csv WRITE.csv CONFIG OUT.json
"""
import csv
import json
import re
import statistics
import sys

# engine kernel name (agnes_kernel_times) -> regex on the demangled symbol
KERNELS = {
    # template <PC, SM, R1, EVC, W64, REC, EDG, RG>: the step's flow, and the record / edge
    # variants agnes_tally_records / agnes_tally_edges launch (round 5); RG = true: the
    # kernel that also holds the unaligned-stream loop (round 6, "flow_ragged"), which
    # runs instead of the aligned one when some instance offset is not a multiple of 4
    "flow": r"agnes::flow::flow<\w+, \w+, \w+, false, \w+, false, false, false>",
    "flow_counts": r"agnes::flow::flow<\w+, \w+, \w+, true, \w+, false, false, false>",
    "flow_records": r"agnes::flow::flow<\w+, \w+, \w+, true, \w+, true, false, false>",
    "flow_edges": r"agnes::flow::flow<\w+, \w+, \w+, true, \w+, false, true, false>",
    "flow_ragged": r"agnes::flow::flow<\w+, \w+, \w+, false, \w+, false, false, true>",
    "flow_ragged_counts": r"agnes::flow::flow<\w+, \w+, \w+, true, \w+, false, false, true>",
    "flow_ragged_records": r"agnes::flow::flow<\w+, \w+, \w+, true, \w+, true, false, true>",
    "flow_ragged_edges": r"agnes::flow::flow<\w+, \w+, \w+, true, \w+, false, true, true>",
    "flow_prep": r"agnes::flow::flow_prep",
    "sweep_walk": r"agnes::sweep::sweep<",
    "tally_fast": r"agnes::fast::tally_fast<",
    "apply_codes": r"agnes::apply::apply_codes<",
    "tally_list": r"agnes::tally_kernel<true, \w+, \w+, \w+, true,",
    "tally_wide": r"agnes::tally_kernel<true, \w+, \w+, \w+, false,",
    "partials": r"agnes::partials::partials_kernel",
    "fold": r"agnes::fold::fold_",
    "dedup_first": r"agnes::dedup::(first_kernel|bucket_)",
    "dedup_first_mask": r"agnes::dedup::bucket_",
    "dedup_mask": r"agnes::dedup::mask_kernel",
    "dedup_reject": r"agnes::dedup::reject_kernel",
    "edge_count": r"agnes::edges::edge_walk<false,",
    "edge_emit": r"agnes::edges::edge_walk<true,",
    "event_count": r"agnes::events::event_walk<false,",
    "event_count_list": r"agnes::events::event_count_list<",
    "event_emit": r"agnes::events::(event_emit_stream<\w+, \w+, false>|event_emit_wave|event_walk<true,)",
    # agnes_tally_records off the flow route (round 5): the emit writing the segments
    "seg_emit": r"agnes::events::event_emit_stream<\w+, \w+, true>",
    "seg_walk": r"agnes::events::seg_walk<",
    "seg_compact": r"agnes::events::seg_compact",
    "edge_seg_walk": r"agnes::edges::edge_seg_walk<",
    "edge_compact": r"agnes::edges::edge_compact",
}


MULTI = {"dedup_first", "dedup_first_mask"}  # engine steps made of several kernels


def per_launch(path, counter):
    """{engine kernel: (median KB per launch, launches)}"""
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for k, pat in KERNELS.items():
            if re.search(pat, r["Kernel_Name"]):
                vals.setdefault(k, {}).setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    # an engine step of several kernels (dedup_first: count, prefix, scatter, min): the
    # sum of each kernel's median per launch; any other entry: the median over its
    # launches (instantiations of one kernel, e.g. flow with and without record counts)
    out = {}
    for k, by in vals.items():
        if k in MULTI:
            out[k] = (sum(statistics.median(v) for v in by.values()), max(len(v) for v in by.values()))
        else:
            allv = [x for v in by.values() for x in v]
            out[k] = (statistics.median(allv), len(allv))
    return out


def main():
    fetch_csv, write_csv, config, out = sys.argv[1:5]
    f = per_launch(fetch_csv, "FETCH_SIZE")
    w = per_launch(write_csv, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(f) | set(w)):
        fb = 2.0 * f[k][0] * 1024.0 if k in f else None
        wb = w[k][0] * 1024.0 if k in w else None
        kernels[k] = {"launches": [f.get(k, (0, 0))[1], w.get(k, (0, 0))[1]],
                      "fetch_bytes": fb, "write_bytes": wb,
                      "traffic_bytes": (fb or 0.0) + (wb or 0.0),
                      "sources": [fetch_csv, write_csv]}
    rec = {"config": config, "kernels": kernels,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read halving), WRITE_SIZE x1, KB->B x1024"}
    try:
        data = json.load(open(out))
    except (OSError, ValueError):
        data = {}
    data[config] = rec
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
