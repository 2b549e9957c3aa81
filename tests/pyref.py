"""Independent pure-Python restatement of the Agnes vote path (test infrastructure).

Written separately from oracle/agnes_oracle.c (object-per-executor, dict-keyed,
Python ints masked to i64) so that agreement between the two is evidence, not
an echo.  Follows:

  round_votes.rs:31-33   is_quorum            vote_executor.rs:20-36  VoteExecutor
  round_votes.rs:48-67   VoteCount::add_vote  state_machine.rs:183-322 apply
  consensus_executor.rs:61-69  apply_msg (Vote arm: event applied at the vote's round)

Small inputs only (pure-Python loops).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Dict, List, Optional, Tuple

NIL = 0xFFFFFFFF
MASK = (1 << 64) - 1

PREVOTE, PRECOMMIT = 0, 1
T_INIT, T_ANY, T_NIL, T_VALUE = 0, 1, 2, 3
S_NEW_ROUND, S_PROPOSE, S_PREVOTE, S_PRECOMMIT, S_COMMIT = range(5)
(EV_NEW_ROUND, EV_NEW_ROUND_PROPOSER, EV_PROPOSAL, EV_PROPOSAL_INVALID, EV_POLKA_ANY,
 EV_POLKA_NIL, EV_POLKA_VALUE, EV_PRECOMMIT_ANY, EV_PRECOMMIT_VALUE, EV_ROUND_SKIP,
 EV_TIMEOUT_PROPOSE, EV_TIMEOUT_PREVOTE, EV_TIMEOUT_PRECOMMIT) = range(13)
EV_NONE = 0xFF
M_NONE, M_NEW_ROUND, M_PROPOSAL, M_VOTE, M_TIMEOUT, M_DECISION = range(6)
TO_PROPOSE, TO_PREVOTE, TO_PRECOMMIT = range(3)

CODE_INVALID, CODE_REJECTED, CODE_SKIP = 6, 7, 8
MODE_REFERENCE, MODE_DEDUP = 0, 1
FLAG_ROUND_SKIP, FLAG_STATE_MACHINE, FLAG_DISTINCT_VALUES = 1, 2, 4


def i64(x: int) -> int:
    """Two's-complement wrap to i64 (Rust release-mode arithmetic)."""
    x &= MASK
    return x - (1 << 64) if x >> 63 else x


def quorum(value: int, total: int) -> bool:
    return i64(3 * value) > i64(2 * total)


def one_third(value: int, total: int) -> bool:
    return i64(3 * value) > total


class Count:
    """VoteCount (round_votes.rs:15-19)."""

    def __init__(self, total: int):
        self.total, self.nil, self.vw, self.label = total, 0, 0, 0

    def add(self, value: int, w: int) -> Tuple[int, int]:
        if value == NIL:
            self.nil = i64(self.nil + w)
        else:
            self.vw = i64(self.vw + w)
            self.label = value
        if quorum(self.vw, self.total):
            return T_VALUE, self.label
        if quorum(self.nil, self.total):
            return T_NIL, 0
        if quorum(self.vw + self.nil, self.total):
            return T_ANY, 0
        return T_INIT, 0


_EVENT_OF = {
    (PREVOTE, T_ANY): EV_POLKA_ANY, (PREVOTE, T_NIL): EV_POLKA_NIL,
    (PREVOTE, T_VALUE): EV_POLKA_VALUE, (PRECOMMIT, T_ANY): EV_PRECOMMIT_ANY,
    (PRECOMMIT, T_NIL): EV_NONE, (PRECOMMIT, T_VALUE): EV_PRECOMMIT_VALUE,
}


def to_event(typ: int, thresh: int) -> int:
    return EV_NONE if thresh == T_INIT else _EVENT_OF[(typ, thresh)]


class VoteExecutor:
    """VoteExecutor with one RoundVotes (vote_executor.rs:8-23)."""

    def __init__(self, height: int, total: int):
        self.height = height
        self.counts = {PREVOTE: Count(total), PRECOMMIT: Count(total)}

    def apply(self, typ: int, value: int, weight: int) -> Tuple[int, int]:
        th, label = self.counts[typ].add(value, weight)
        return to_event(typ, th), label


@dataclass(frozen=True)
class State:
    height: int = 0
    round: int = 0
    step: int = S_NEW_ROUND
    locked: Optional[Tuple[int, int]] = None
    valid: Optional[Tuple[int, int]] = None
    decision: Optional[Tuple[int, int]] = None  # extension: recorded Decision


@dataclass(frozen=True)
class Msg:
    kind: int
    round: int = 0
    value: int = 0
    pol_round: int = 0
    vote_type: int = 0
    timeout_step: int = 0


def _next(s: State) -> State:
    nxt = {S_NEW_ROUND: S_PROPOSE, S_PROPOSE: S_PREVOTE, S_PREVOTE: S_PRECOMMIT}
    return replace(s, step=nxt.get(s.step, s.step))


def apply(s: State, rnd: int, ev: int, value: int = 0, pol_round: int = 0,
          distinct_values: bool = False) -> Tuple[State, Optional[Msg]]:
    """fn apply, state_machine.rs:183-214."""
    eqr = s.round == rnd
    st = s.step
    if st == S_NEW_ROUND and ev == EV_NEW_ROUND_PROPOSER and eqr:
        s = _next(s)
        v, pol = (s.valid[1], s.valid[0]) if s.valid else (value, -1)
        return s, Msg(M_PROPOSAL, s.round, v, pol)
    if st == S_NEW_ROUND and ev == EV_NEW_ROUND and eqr:
        s = _next(s)
        return s, Msg(M_TIMEOUT, s.round, timeout_step=TO_PROPOSE)
    if st == S_PROPOSE and ev == EV_PROPOSAL and eqr and -1 <= pol_round < s.round:
        s = _next(s)
        if s.locked is None:
            out = value
        elif s.locked[0] <= pol_round:
            out = value
        elif (not distinct_values) or s.locked[1] == value:
            out = value
        else:
            out = NIL
        return s, Msg(M_VOTE, s.round, out, vote_type=PREVOTE)
    if st == S_PROPOSE and ev in (EV_PROPOSAL_INVALID, EV_TIMEOUT_PROPOSE) and eqr:
        s = _next(s)
        return s, Msg(M_VOTE, s.round, NIL, vote_type=PREVOTE)
    if st == S_PREVOTE and ev == EV_POLKA_ANY and eqr:
        return s, Msg(M_TIMEOUT, s.round, timeout_step=TO_PREVOTE)
    if st == S_PREVOTE and ev in (EV_POLKA_NIL, EV_TIMEOUT_PREVOTE) and eqr:
        s = _next(s)
        return s, Msg(M_VOTE, s.round, NIL, vote_type=PRECOMMIT)
    if st == S_PREVOTE and ev == EV_POLKA_VALUE and eqr:
        s = _next(replace(s, locked=(s.round, value), valid=(s.round, value)))
        return s, Msg(M_VOTE, s.round, value, vote_type=PRECOMMIT)
    if st == S_PRECOMMIT and ev == EV_POLKA_VALUE and eqr:
        return replace(s, valid=(s.round, value)), None
    if st == S_COMMIT:
        return s, None
    if ev == EV_PRECOMMIT_ANY and eqr:
        return s, Msg(M_TIMEOUT, s.round, timeout_step=TO_PRECOMMIT)
    if ev == EV_TIMEOUT_PRECOMMIT and eqr:
        r = i64(rnd + 1)
        return replace(s, round=r, step=S_NEW_ROUND), Msg(M_NEW_ROUND, r)
    if ev == EV_ROUND_SKIP and s.round < rnd:
        return replace(s, round=rnd, step=S_NEW_ROUND), Msg(M_NEW_ROUND, rnd)
    if ev == EV_PRECOMMIT_VALUE:
        return replace(s, step=S_COMMIT, decision=(rnd, value)), Msg(M_DECISION, rnd, value)
    return s, None


_CODE_OF_EV = {EV_NONE: 0, EV_POLKA_ANY: 1, EV_POLKA_NIL: 2, EV_POLKA_VALUE: 3,
               EV_PRECOMMIT_ANY: 4, EV_PRECOMMIT_VALUE: 5}


def _vmsg(m_skip: Optional[Msg], m_ev: Optional[Msg]) -> int:
    base = 0
    if m_ev is not None:
        if m_ev.kind == M_TIMEOUT:
            base = 1 if m_ev.timeout_step == TO_PREVOTE else 2
        elif m_ev.kind == M_VOTE:
            base = 3 if m_ev.value == NIL else 4
        elif m_ev.kind == M_DECISION:
            base = 5
        else:
            raise AssertionError(m_ev)
    if m_skip is not None:
        return {0: 6, 2: 7, 5: 8}[base]
    return base


@dataclass
class Batch:
    instance: List[int]
    round: List[int]
    type: List[int]
    value: List[int]
    validator: List[int]
    offsets: List[int]
    weight: Optional[List[int]] = None
    instance_set: Optional[List[int]] = None


def tally(batch: Batch, power: List[List[int]], totals: List[int], mode: int, flags: int,
          max_rounds: int, states: Optional[List[State]] = None):
    """Batch contract: returns (codes, states)."""
    codes = [0] * len(batch.round)
    states = list(states) if states is not None else None
    n_inst = len(batch.offsets) - 1
    skip_on = bool(flags & FLAG_ROUND_SKIP)
    sm = bool(flags & FLAG_STATE_MACHINE) and states is not None
    distinct = bool(flags & FLAG_DISTINCT_VALUES)
    need_val = batch.weight is None or mode == MODE_DEDUP or skip_on
    for i in range(n_inst):
        set_idx = batch.instance_set[i] if batch.instance_set else (i % len(power) if power else 0)
        set_ok = set_idx < len(power)
        total = totals[set_idx] if set_ok else 0
        n_vals = len(power[set_idx]) if set_ok else 0
        execs: Dict[int, VoteExecutor] = {}
        seen_vote = set()
        seen_skip = set()
        skip_w: Dict[int, int] = {}
        for j in range(batch.offsets[i], batch.offsets[i + 1]):
            r, t, val, value = batch.round[j], batch.type[j], batch.validator[j], batch.value[j]
            if (batch.instance[j] != i or r >= max_rounds or t > 1
                    or (need_val and (not set_ok or val >= n_vals))
                    or (batch.weight is None and not set_ok)):
                codes[j] = CODE_INVALID
                continue
            w = batch.weight[j] if batch.weight is not None else power[set_idx][val]
            if skip_on and (r, val) not in seen_skip:
                seen_skip.add((r, val))
                skip_w[r] = i64(skip_w.get(r, 0) + w)
            if mode == MODE_DEDUP:
                if (r, t, val) in seen_vote:
                    codes[j] = CODE_REJECTED
                    continue
                seen_vote.add((r, t, val))
            ex = execs.setdefault(r, VoteExecutor(0, total))
            ev, label = ex.apply(t, value, w)
            skip = skip_on and one_third(skip_w.get(r, 0), total)
            code = _CODE_OF_EV[ev] | (CODE_SKIP if skip else 0)
            if sm:
                s = states[i]
                m1 = m2 = None
                if skip:
                    s, m1 = apply(s, r, EV_ROUND_SKIP, distinct_values=distinct)
                if ev != EV_NONE:
                    s, m2 = apply(s, r, ev, label, distinct_values=distinct)
                states[i] = s
                code |= _vmsg(m1, m2) << 4
            codes[j] = code
    return codes, states


IN_VOTE, IN_PROPOSAL, IN_TIMEOUT, IN_NEW_ROUND = range(4)
_TIMEOUT_EV = {TO_PROPOSE: EV_TIMEOUT_PROPOSE, TO_PREVOTE: EV_TIMEOUT_PREVOTE,
               TO_PRECOMMIT: EV_TIMEOUT_PRECOMMIT}


def apply_msgs(batch: Batch, kinds: List[int], pol_round: Optional[List[int]], power: List[List[int]],
               totals: List[int], flags: int, max_rounds: int, states: List[State]):
    """ConsensusExecutor::apply_msg over per-instance message streams
    (consensus_executor.rs:54-86): one executor per (round, type) per instance,
    Proposal -> Event::Proposal(pol_round, value) (:56-60), Vote -> VoteExecutor
    then its event (:61-69), Timeout -> TimeoutX (:70-77), each at the message's
    round; NewRound input -> NewRound / NewRoundProposer(value).
    Returns (codes, states, msgs: list of Optional[Msg])."""
    n = len(batch.round)
    codes, msgs = [0] * n, [None] * n
    states = list(states)
    distinct = bool(flags & FLAG_DISTINCT_VALUES)
    for i in range(len(batch.offsets) - 1):
        set_idx = batch.instance_set[i] if batch.instance_set else (i % len(power) if power else 0)
        set_ok = set_idx < len(power)
        total = totals[set_idx] if set_ok else 0
        n_vals = len(power[set_idx]) if set_ok else 0
        counts: Dict[Tuple[int, int], Count] = {}
        s = states[i]
        for j in range(batch.offsets[i], batch.offsets[i + 1]):
            k, r, t, v = kinds[j], batch.round[j], batch.type[j], batch.value[j]
            ev, ev_val, pol = EV_NONE, 0, 0
            if k == IN_VOTE:
                val = batch.validator[j]
                if (batch.instance[j] != i or r >= max_rounds or t > 1
                        or (batch.weight is None and (not set_ok or val >= n_vals))):
                    codes[j] = CODE_INVALID
                    continue
                w = batch.weight[j] if batch.weight is not None else power[set_idx][val]
                th, ev_val = counts.setdefault((r, t), Count(total)).add(v, w)
                ev = to_event(t, th)
                codes[j] = _CODE_OF_EV[ev]
            elif k == IN_PROPOSAL:
                ev, ev_val, pol = EV_PROPOSAL, v, (pol_round[j] if pol_round is not None else -1)
            elif k == IN_TIMEOUT and t in _TIMEOUT_EV:
                ev = _TIMEOUT_EV[t]
            elif k == IN_NEW_ROUND:
                ev, ev_val = (EV_NEW_ROUND_PROPOSER, v) if v != NIL else (EV_NEW_ROUND, 0)
            else:
                codes[j] = CODE_INVALID
                continue
            if ev != EV_NONE:
                s, msgs[j] = apply(s, r, ev, ev_val, pol, distinct_values=distinct)
        states[i] = s
    return codes, states, msgs
