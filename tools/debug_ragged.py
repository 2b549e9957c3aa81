#!/usr/bin/env python3
"""Development probe: characterise GPU/oracle mismatches on ragged batches."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as ol  # noqa: E402
from agnes_amd import abi  # noqa: E402
from agnes_amd.engine import DeviceBatch, Engine  # noqa: E402


def ragged(seed, n_inst, n_vals, R, lengths):
    rng = np.random.default_rng(seed)
    lens = rng.choice(lengths, n_inst)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    n = int(off[-1])
    inst = np.repeat(np.arange(n_inst, dtype=np.uint32), lens)
    rnd = rng.integers(0, R, n).astype(np.uint8)
    typ = rng.integers(0, 2, n).astype(np.uint8)
    val = np.where(rng.random(n) < 0.3, abi.NIL, rng.integers(0, 3, n)).astype(np.uint32)
    vid = rng.integers(0, n_vals, n).astype(np.uint32)
    return ol.batch_from_lists(inst, rnd, typ, val, vid, off)


eng = Engine(0)
for name, lengths, mode, flags, n_sets in [
    ("skip_only_tiny", [1, 2, 3], abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP, 1),
    ("skip_only_tiny_sets", [1, 2, 3], abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP, 13),
    ("skip_only_mixed", [0, 5, 70], abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP, 1),
    ("dedup_only_tiny", [1, 2, 3, 8], abi.MODE_DEDUP, 0, 1),
    ("skip_single_len64", [64], abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP, 1),
    ("skip_single_len100", [100], abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP, 1),
    ("sm_tiny", [1, 2, 3], abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1),
    ("skip_sm_tiny", [1, 2, 3], abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 1),
    ("skip_sm_len100", [100], abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 1),
    ("skip_sm_mixed", [0, 5, 70], abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 1),
    ("skip_sm_len200", [200], abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 1),
]:
    hb = ragged(3, int(os.environ.get("NI", "40000")), 9, 3, lengths)
    power = ol.gen_power(3, n_sets, 9, abi.POWER_UNIFORM, 1, 20)
    eng.upload_power(power)
    cfg = abi.config(mode, flags, 3)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.zeros(hb.n_votes, dtype=torch.uint8, device=eng.device)
    st0 = None
    dst = None
    if flags & abi.FLAG_STATE_MACHINE:
        from agnes_amd.engine import states_to_device
        st0 = abi.new_states(hb.n_instances, 1, abi.STEP_PREVOTE)
        dst = states_to_device(st0, eng.device)
    eng.tally(cfg, db, codes, dst)
    torch.cuda.synchronize()
    g = codes.cpu().numpy()
    o, _, _ = ol.tally(cfg, hb, power, None, st0)
    bad = np.nonzero(g != o)[0]
    print(f"{name}: votes={hb.n_votes} mismatches={len(bad)}")
    for k in bad[:6]:
        i = int(hb.instance[k])
        s = int(hb.offsets[i])
        print(f"   vote {k} inst {i} pos {k - s} len {int(hb.offsets[i + 1]) - s} r {hb.round[k]} "
              f"t {hb.type[k]} val {hb.validator[k]} gpu {g[k]:#x} orc {o[k]:#x} "
              f"chunk_lane {k % 64}")
