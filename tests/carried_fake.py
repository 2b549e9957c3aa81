"""CPU stand-in for agnes_tally_carried (TEST INFRASTRUCTURE ONLY: the checker's
side of the split-instance tests; never part of the engine).

Restates, for REFERENCE mode without RoundSkip / State machine, the contract of
include/agnes.h `agnes_tally_carried`: each segment of the batch continues the
RoundVotes state in `counts[segment][round * 2 + type]` (VoteCount,
round_votes.rs:15-19; add_vote :48-67; is_quorum :31-33 in wrapping i64; to_event
vote_executor.rs:26-36) and leaves its state there.  With AGNES_FLAG_ONE_INSTANCE
every segment is a slice of one instance whose votes carry id cfg.reserved.
"""
from __future__ import annotations

import numpy as np

from agnes_amd import abi

M64 = (1 << 64) - 1


def _s64(x: int) -> int:
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def _quorum(v: int, total: int) -> bool:
    return _s64(3 * v) > _s64(2 * total)


class CarriedFake:
    def __init__(self, power: np.ndarray, totals=None):
        self.power = np.ascontiguousarray(power, dtype=np.int64)
        self.totals = (np.array([_s64(int(x)) for x in self.power.sum(axis=1, dtype=np.int64)])
                       if totals is None else np.asarray(totals, dtype=np.int64))

    def tally_carried(self, cfg: abi.Config, b, codes: np.ndarray, counts: np.ndarray):
        """b: HostBatch-like (instance, round, type, value, validator, offsets,
        instance_set); counts: VOTE_COUNT_DTYPE [n_segments, 2 * max_rounds]."""
        R = cfg.max_rounds
        one = bool(cfg.flags & abi.FLAG_ONE_INSTANCE)
        n_sets, nv = self.power.shape
        off = np.asarray(b.offsets, dtype=np.int64)
        for k in range(len(off) - 1):
            want = cfg.reserved if one else k
            s = int(b.instance_set[k]) if b.instance_set is not None else (want % n_sets)
            total = int(self.totals[s]) if s < n_sets else 0
            vw = [int(x) for x in counts[k]["value_w"]]
            vn = [int(x) for x in counts[k]["nil_w"]]
            lab = [int(x) for x in counts[k]["value"]]
            for j in range(int(off[k]), int(off[k + 1])):
                r, t, val, x = int(b.round[j]), int(b.type[j]), int(b.value[j]), int(b.validator[j])
                if int(b.instance[j]) != want or r >= R or t > 1 or s >= n_sets or x >= nv:
                    codes[j] = abi.CODE_INVALID
                    continue
                w = int(self.power[s, x])
                q = r * 2 + t
                if val != abi.NIL:
                    vw[q] = _s64(vw[q] + w)
                    lab[q] = val
                else:
                    vn[q] = _s64(vn[q] + w)
                if _quorum(vw[q], total):
                    ev = abi.CODE_POLKA_VALUE if t == 0 else abi.CODE_PRECOMMIT_VALUE
                elif _quorum(vn[q], total):
                    ev = abi.CODE_POLKA_NIL if t == 0 else abi.CODE_NONE
                elif _quorum(_s64(vw[q] + vn[q]), total):
                    ev = abi.CODE_POLKA_ANY if t == 0 else abi.CODE_PRECOMMIT_ANY
                else:
                    ev = abi.CODE_NONE
                codes[j] = ev
            counts[k]["value_w"] = vw
            counts[k]["nil_w"] = vn
            counts[k]["value"] = lab


class DedupFake:
    """CPU stand-in for agnes_dedup_first / _mask / _reject (include/agnes.h): the
    first vote of each (round, type, validator) of one instance found across
    slices, the later ones masked out of the tally and coded REJECTED."""

    MASKED = 0xFE

    def __init__(self, n_sets: int, n_vals: int):
        self.n_sets, self.n_vals = n_sets, n_vals

    def _keys(self, cfg, b):
        r = np.asarray(b.round, np.int64)
        t = np.asarray(b.type, np.int64)
        x = np.asarray(b.validator, np.int64)
        ok = ((np.asarray(b.instance, np.int64) == cfg.reserved) & (r < cfg.max_rounds) & (t <= 1)
              & (x < self.n_vals) & (cfg.reserved % self.n_sets < self.n_sets))
        return ok, (r * 2 + t) * self.n_vals + x

    def first(self, cfg, b, base: int, first: np.ndarray):
        ok, key = self._keys(cfg, b)
        idx = base + np.arange(len(key), dtype=np.int64)
        np.minimum.at(first, key[ok], idx[ok])

    def mask(self, cfg, b, base: int, first: np.ndarray) -> np.ndarray:
        ok, key = self._keys(cfg, b)
        t = np.asarray(b.type, np.uint8).copy()
        idx = base + np.arange(len(key), dtype=np.int64)
        dup = ok.copy()
        dup[ok] = first[key[ok]] != idx[ok]
        t[~ok] = 0xFF  # invalid in the one-stream DEDUP tally: rejected by the carried tally too
        t[dup] = self.MASKED
        return t

    def reject(self, type_masked: np.ndarray, codes: np.ndarray):
        codes[type_masked == self.MASKED] = abi.CODE_REJECTED
