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
        mrej = bool(cfg.flags & abi.FLAG_MASKED_REJECTED)
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
                    codes[j] = abi.CODE_REJECTED if mrej and t == abi.TYPE_MASKED else abi.CODE_INVALID
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

    MASKED = abi.TYPE_MASKED

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


class OneSmFake:
    """CPU stand-in for agnes_one_sm_scan / _apply / _finish (include/agnes.h; TEST
    INFRASTRUCTURE): the State machine of one instance split into slices, from the
    slice codes of the carried tally.  Restates state_machine.rs:196-211 for vote
    events without RoundSkip: P1 = first PolkaNil / PolkaValue at State.round in
    Prevote, C = first PrecommitValue; messages by position relative to them."""

    MAXM = (1 << 63) - 1

    def __init__(self, state):
        self.state = state  # abi.STATE_DTYPE record (numpy void), read and written

    def scan(self, codes, round_, value, base, marks):
        s = self.state
        if int(s["step"]) == abi.STEP_COMMIT:
            return
        e = codes & abi.CODE_EVENT_MASK
        eqr = round_.astype(np.int64) == int(s["round"])
        pos = base + np.arange(len(codes), dtype=np.int64)
        p1 = (int(s["step"]) == abi.STEP_PREVOTE) & eqr & ((e == abi.CODE_POLKA_NIL) | (e == abi.CODE_POLKA_VALUE))
        if p1.any():
            j = int(np.argmax(p1))
            lv = int(value[j]) if e[j] == abi.CODE_POLKA_VALUE else abi.NIL
            marks[0] = min(int(marks[0]), (int(pos[j]) << 32) | lv)
        cc = e == abi.CODE_PRECOMMIT_VALUE
        if cc.any():
            j = int(np.argmax(cc))
            marks[1] = min(int(marks[1]), (int(pos[j]) << 32) | int(value[j]))

    def apply(self, codes, round_, value, base, marks):
        s = self.state
        if int(s["step"]) == abi.STEP_COMMIT:
            return
        C = self.MAXM if int(marks[1]) == self.MAXM else int(marks[1]) >> 32
        P1 = self.MAXM if int(marks[0]) == self.MAXM else int(marks[0]) >> 32
        if P1 >= C:
            P1 = self.MAXM
        step = int(s["step"])
        for j in range(len(codes)):
            e = int(codes[j]) & abi.CODE_EVENT_MASK
            eqr = int(round_[j]) == int(s["round"])
            pos = base + j
            msg = 0
            if pos < C:
                if e == abi.CODE_PRECOMMIT_ANY and eqr:
                    msg = abi.VMSG_TIMEOUT_PRECOMMIT
                if e == abi.CODE_POLKA_ANY and eqr and step == abi.STEP_PREVOTE and pos < P1:
                    msg = abi.VMSG_TIMEOUT_PREVOTE
                if pos == P1:
                    msg = abi.VMSG_PRECOMMIT_VALUE if e == abi.CODE_POLKA_VALUE else abi.VMSG_PRECOMMIT_NIL
            elif pos == C:
                msg = abi.VMSG_DECISION
                marks[3] = max(int(marks[3]), int(round_[j]) + 1)
            codes[j] |= msg << abi.CODE_MSG_SHIFT
            if (e == abi.CODE_POLKA_VALUE and eqr and int(value[j]) != abi.NIL and pos < C
                    and ((step == abi.STEP_PREVOTE and pos >= P1) or step == abi.STEP_PRECOMMIT)):
                marks[2] = max(int(marks[2]), ((pos + 1) << 32) | int(value[j]))

    def finish(self, marks):
        s = self.state
        if int(s["step"]) == abi.STEP_COMMIT:
            return
        m0, m1, m2, m3 = (int(x) for x in marks)
        C = self.MAXM if m1 == self.MAXM else m1 >> 32
        P1 = self.MAXM if m0 == self.MAXM else m0 >> 32
        if P1 < C:
            s["step"] = abi.STEP_PRECOMMIT
            if (m0 & 0xFFFFFFFF) != abi.NIL:
                s["locked_present"], s["locked_round"], s["locked_value"] = 1, s["round"], m0 & 0xFFFFFFFF
        if m2:
            s["valid_present"], s["valid_round"], s["valid_value"] = 1, s["round"], m2 & 0xFFFFFFFF
        if C != self.MAXM:
            s["step"], s["decided"] = abi.STEP_COMMIT, 1
            s["decision_round"], s["decision_value"] = m3 - 1, m1 & 0xFFFFFFFF
