"""Python handle on the native multi-GPU driver (include/agnes.h agnes_multi_*):
host batch in, host codes / States out, one device context + stream + host thread
per listed device, contiguous instance ranges balanced by votes; the split-instance
C5 path (agnes_multi_tally_one: slices per device, the exchanges over RCCL or pinned
host memory) and the gathered edge summary.  The same entries a non-Python consumer
binds; agnes_amd/dist.py is the one-process-per-GPU path."""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import abi
from .lib import check, load


class MultiEngine:
    def __init__(self, devices: Sequence[int]):
        self.lib = load()
        self.devices = list(devices)
        arr = (C.c_int * len(self.devices))(*self.devices)
        h = C.c_void_p()
        check(self.lib.agnes_multi_create(arr, len(self.devices), C.byref(h)), "agnes_multi_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.agnes_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def upload_power(self, power: np.ndarray, totals: Optional[np.ndarray] = None):
        power = np.ascontiguousarray(power, dtype=np.int64)
        tot = None if totals is None else np.ascontiguousarray(totals, dtype=np.int64)
        check(self.lib.agnes_multi_upload_power(self.h, power.ctypes.data, power.shape[0], power.shape[1],
                                                None if tot is None else tot.ctypes.data), "agnes_multi_upload_power")

    def tally(self, cfg: abi.Config, hb, states: Optional[np.ndarray] = None):
        """hb: host batch (numpy columns instance/round/type/value/validator/offsets,
        optional instance_set / weight).  Returns (codes u8, states or None, stats
        abi.MULTI_STATS_DTYPE per device)."""
        def p(a):
            return None if a is None else a.ctypes.data
        cols = {k: np.ascontiguousarray(getattr(hb, k)) for k in ("instance", "round", "type", "value",
                                                                   "validator", "offsets")}
        iset = getattr(hb, "instance_set", None)
        w = getattr(hb, "weight", None)
        n_votes = int(cols["offsets"][-1])
        b = abi.VoteBatch(p(cols["instance"]), p(cols["round"]), p(cols["type"]), p(cols["value"]),
                          p(cols["validator"]), p(cols["offsets"]), p(iset), p(w), n_votes,
                          len(cols["offsets"]) - 1, 0)
        codes = np.zeros(max(n_votes, 1), np.uint8)
        st = None if states is None else np.array(states, dtype=abi.STATE_DTYPE, copy=True)
        stats = np.zeros(len(self.devices), abi.MULTI_STATS_DTYPE)
        check(self.lib.agnes_multi_tally(self.h, C.byref(cfg), C.byref(b), codes.ctypes.data, p(st),
                                         stats.ctypes.data), "agnes_multi_tally")
        return codes[:n_votes], st, stats

    def exchange(self, mode: int):
        """abi.MULTI_EXCHANGE_AUTO / _HOST / _RCCL for tally_one's exchanges."""
        check(self.lib.agnes_multi_exchange(self.h, mode), "agnes_multi_exchange")

    def test_corrupt(self, ops: int):
        """Test hook: bit k re-arms the self-check of kind k (0 MIN u64, 1 MIN i64, 2 MAX
        i64, 3 all-gather) and flips the first received byte of its next RCCL collective;
        bit 4 + k flips it in every RCCL collective of kind k (a broken RCCL), so the
        self-check's fallback (stats['exchange'] & abi.MULTI_X_FALLBACK) can be tested."""
        check(self.lib.agnes_multi_test_corrupt(self.h, ops), "agnes_multi_test_corrupt")

    def tally_one(self, cfg: abi.Config, hb, state: Optional[np.ndarray] = None, segments: int = 0):
        """C5: hb holds ONE instance (host columns).  Returns (codes u8, state (1
        record) or None, counts abi.VOTE_COUNT_DTYPE [2 * max_rounds], stats)."""
        def p(a):
            return None if a is None else a.ctypes.data
        cols = {k: np.ascontiguousarray(getattr(hb, k)) for k in ("instance", "round", "type", "value",
                                                                   "validator", "offsets")}
        n_votes = int(cols["offsets"][-1])
        b = abi.VoteBatch(p(cols["instance"]), p(cols["round"]), p(cols["type"]), p(cols["value"]),
                          p(cols["validator"]), p(cols["offsets"]), None, None, n_votes, 1, 0)
        codes = np.zeros(max(n_votes, 1), np.uint8)
        st = None if state is None else np.array(state, dtype=abi.STATE_DTYPE, copy=True).reshape(1)
        counts = np.zeros(2 * cfg.max_rounds, abi.VOTE_COUNT_DTYPE)
        stats = np.zeros(len(self.devices), abi.MULTI_STATS_DTYPE)
        check(self.lib.agnes_multi_tally_one(self.h, C.byref(cfg), C.byref(b), codes.ctypes.data, p(st),
                                             counts.ctypes.data, segments, stats.ctypes.data),
              "agnes_multi_tally_one")
        return codes[:n_votes], st, counts, stats

    def edges(self, cfg: abi.Config, n_instances: int):
        """The edge summary of the last tally()'s batch, gathered from every device:
        (offsets u64 [n + 1], records abi.EDGE_DTYPE)."""
        offs = np.zeros(n_instances + 1, np.uint64)
        check(self.lib.agnes_multi_edge_offsets(self.h, C.byref(cfg), offs.ctypes.data), "agnes_multi_edge_offsets")
        out = np.zeros(max(int(offs[-1]), 1), abi.EDGE_DTYPE)
        check(self.lib.agnes_multi_edges(self.h, C.byref(cfg), offs.ctypes.data, out.ctypes.data), "agnes_multi_edges")
        return offs, out[:int(offs[-1])]
