#!/usr/bin/env python3
"""C5 pass-B probe (development tool): bench.py's one-instance step on variants of
the c5 / c5d workloads (DEDUP without duplicates, REFERENCE with them), to see
which input property sets pass B's time.  usage: tools/c5probe.py VARIANT [bench args]"""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from agnes_amd import abi  # noqa: E402

W = bench.WORKLOADS
v = {}
v["dedup_nodup"] = copy.deepcopy(W["c5d"])
v["dedup_nodup"]["gen"].update(dup_permille=0, equiv_permille=0)
v["ref_dups"] = copy.deepcopy(W["c5d"])
v["ref_dups"]["mode"] = abi.MODE_REFERENCE
v["dedup_dup"] = copy.deepcopy(W["c5d"])
v["dedup_dup"]["gen"].update(equiv_permille=0, dup_permille=200)
v["dedup_equiv"] = copy.deepcopy(W["c5d"])
v["dedup_equiv"]["gen"].update(equiv_permille=200, dup_permille=0)
W.update(v)
sys.argv = [sys.argv[0], "--config"] + sys.argv[1:]
bench.main()
