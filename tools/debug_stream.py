#!/usr/bin/env python3
"""Debug a GPU/oracle code mismatch on a generated config (development tool).
Prints, for the first mismatching instance, per vote: position, key, weight,
running value/nil sums of its bucket, the set's q2, oracle and GPU codes.
usage: tools/debug_stream.py [config-name]   (configs of tests/test_gpu_parity.py)"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as ol  # noqa: E402
from agnes_amd import abi  # noqa: E402
from agnes_amd.engine import DeviceBatch, Engine, states_to_device  # noqa: E402
import test_gpu_parity as T  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3_small"
p, hb, power, cfg = T._make(name)
states = T._start_states(p.n_instances) if cfg.flags & abi.FLAG_STATE_MACHINE else None
eng = Engine(0)
eng.upload_power(power)
db = DeviceBatch.from_host(hb, eng.device)
codes = torch.zeros(hb.n_votes, dtype=torch.uint8, device=eng.device)
dst = None if states is None else states_to_device(states, eng.device)
eng.tally(cfg, db, codes, dst)
torch.cuda.synchronize()
g = codes.cpu().numpy()
o, _, _ = ol.tally(cfg, hb, power, None, states)
bad = np.nonzero(g != o)[0]
print(f"{name}: {len(bad)} mismatches")
if len(bad) == 0:
    sys.exit(0)
off = hb.offsets.astype(np.int64)
i = int(np.searchsorted(off, bad[0], side="right") - 1)
n_sets = power.shape[0]
set_ = int(hb.instance_set[i]) if getattr(hb, "instance_set", None) is not None else i % n_sets
tot = int(power[set_].sum())
q2 = (2 * tot) // 3
print(f"instance {i} votes [{off[i]}, {off[i+1]}) set {set_} total {tot} q2 {q2}; "
      f"mismatching votes in it: {np.count_nonzero((bad >= off[i]) & (bad < off[i+1]))}")
sums = {}
for j in range(off[i], off[i + 1]):
    r, t, v, x = int(hb.round[j]), int(hb.type[j]), int(hb.value[j]), int(hb.validator[j])
    w = int(power[set_][x]) if x < power.shape[1] else 0
    k = (r, t)
    sv, sn = sums.get(k, (0, 0))
    if v == abi.NIL:
        sn += w
    else:
        sv += w
    sums[k] = (sv, sn)
    mark = " <<<" if g[j] != o[j] else ""
    if abs(j - bad[0]) < 40 or mark:
        print(f"{j:9d} loc {j-off[i]:5d} chunkpos {(j - off[i]) % 256:3d} r{r} t{t} nil{int(v == abi.NIL)} "
              f"w {w:5d} sv {sv:7d} sn {sn:7d} sum {sv+sn:7d}  oracle {o[j]:#04x} gpu {g[j]:#04x}{mark}")
