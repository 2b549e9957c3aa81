#!/usr/bin/env python3
"""Development check: one generated config through agnes_tally (AUTO route), synchronise,
and compare codes / States with the checker; prints the first mismatches."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
import oracle_lib as ol  # noqa: E402
from agnes_amd import abi  # noqa: E402
from agnes_amd.engine import DeviceBatch, Engine, states_to_device  # noqa: E402
from test_gpu_parity import _make, _start_states  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c4_small"
eng = Engine(0)
p, hb, power, cfg = _make(name)
states = _start_states(p.n_instances) if cfg.flags & abi.FLAG_STATE_MACHINE else None
eng.upload_power(power)
db = DeviceBatch.from_host(hb, eng.device)
codes = torch.zeros(max(hb.n_votes, 1), dtype=torch.uint8, device=eng.device)
dst = None if states is None else states_to_device(states, eng.device)
eng.tally(cfg, db, codes, dst)
try:
    torch.cuda.synchronize()
    print("sync ok", flush=True)
except Exception as ex:  # noqa: BLE001
    print("sync error:", ex, flush=True)
    raise SystemExit(1)
g = codes[:hb.n_votes].cpu().numpy()
o_codes, _, o_states = ol.tally(cfg, hb, power, None, states, threads=8)
bad = np.nonzero(g != o_codes)[0]
print(name, "votes", hb.n_votes, "code mismatches", len(bad), flush=True)
if len(bad):
    inst = np.searchsorted(hb.offsets.astype(np.int64), bad, side="right") - 1
    for k in bad[:12]:
        i = int(np.searchsorted(hb.offsets.astype(np.int64), k, side="right") - 1)
        print(f"  vote {k} inst {i} (start {hb.offsets[i]}) gpu {g[k]:#x} oracle {o_codes[k]:#x}")
    print("  instances with mismatches:", len(np.unique(inst)))
if len(bad):
    raise SystemExit(1)
