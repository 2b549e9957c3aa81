#!/usr/bin/env python3
"""Development probe: state mismatches on the wide (i64) path."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as ol  # noqa: E402
from agnes_amd import abi  # noqa: E402
from agnes_amd.engine import DeviceBatch, Engine, states_to_device, states_to_host  # noqa: E402

eng = Engine(0)
for name, lo, hi in [("wide_huge", 1 << 61, 1 << 62), ("fast_same_shape", 1, 1000)]:
    p = abi.gen_params(seed=0xA6E5, n_instances=500, n_vals=40, rounds_min=1, rounds_max=2,
                       nil_permille=400, dup_permille=300)
    hb = ol.gen_batch(p)
    power = ol.gen_power(0xA6E5, 3, 40, abi.POWER_UNIFORM, lo, hi)
    eng.upload_power(power)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 2)
    st0 = abi.new_states(500, 1, abi.STEP_PREVOTE)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.zeros(hb.n_votes, dtype=torch.uint8, device=eng.device)
    dst = states_to_device(st0, eng.device)
    eng.tally(cfg, db, codes, dst)
    torch.cuda.synchronize()
    gs = states_to_host(dst)
    oc, os_, _ = ol.tally(cfg, hb, power, None, st0)
    print(name, "codes equal:", np.array_equal(codes.cpu().numpy(), oc))
    nd = 0
    for i in range(500):
        if gs[i].tobytes() != os_[i].tobytes():
            nd += 1
            if nd <= 5:
                diffs = {f: (gs[i][f].tolist(), os_[i][f].tolist()) for f in abi.STATE_DTYPE.names
                         if gs[i][f].tolist() != os_[i][f].tolist()}
                print("  inst", i, "len", int(hb.offsets[i + 1] - hb.offsets[i]), diffs)
    print("  differing states:", nd)
