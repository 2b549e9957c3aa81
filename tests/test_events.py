"""The event stream's checker (oracle/agnes_oracle.c orc_tally_labels + orc_events)
against a pure-Python restatement of the reference, on small batches.

Restatement: per instance, per (round, type), a VoteCount (round_votes.rs:15-19)
with one value slot (add_vote :48-67, last writer wins), is_quorum :31-33 in
wrapping i64, to_event vote_executor.rs:26-36; every vote's Some(Event) in order,
PolkaValue / PrecommitValue carrying the slot's Value after the vote.  The
per-vote codes come from the checker's tally (REFERENCE, no RoundSkip: the
restatement re-derives the events alone, and must agree with them too).
"""
import numpy as np
import pytest

import oracle_lib as ol
from agnes_amd import abi

M64 = (1 << 64) - 1


def _s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def _q(v, total):
    return _s64(3 * v) > _s64(2 * total)


def restate(hb, power, R):
    """[(vote, instance, value, round, kind)] of a REFERENCE batch (fresh executors)."""
    totals = [_s64(int(x)) for x in power.sum(axis=1)]
    n_sets, nv = power.shape
    out = []
    off = hb.offsets.astype(np.int64)
    for i in range(len(off) - 1):
        s = int(hb.instance_set[i]) if hb.instance_set is not None else i % n_sets
        total = totals[s] if s < n_sets else 0
        cnt = {}
        for j in range(off[i], off[i + 1]):
            r, t, v, x = int(hb.round[j]), int(hb.type[j]), int(hb.value[j]), int(hb.validator[j])
            if int(hb.instance[j]) != i or r >= R or t > 1 or s >= n_sets or x >= nv:
                continue
            w = int(power[s, x])
            c = cnt.setdefault((r, t), [0, 0, 0])  # value weight, nil weight, value slot
            if v != abi.NIL:
                c[0] = _s64(c[0] + w)
                c[2] = v
            else:
                c[1] = _s64(c[1] + w)
            if _q(c[0], total):
                kind, val = (abi.EV_POLKA_VALUE if t == 0 else abi.EV_PRECOMMIT_VALUE), c[2]
            elif _q(c[1], total):
                kind, val = (abi.EV_POLKA_NIL if t == 0 else None), abi.NIL
            elif _q(_s64(c[0] + c[1]), total):
                kind, val = (abi.EV_POLKA_ANY if t == 0 else abi.EV_PRECOMMIT_ANY), abi.NIL
            else:
                kind = None
            if kind is not None:
                out.append((j, i, val, r, kind))
    return out


@pytest.mark.parametrize("seed,n_inst,nv,R,kind", [(1, 40, 7, 1, abi.POWER_UNIFORM), (2, 30, 25, 3, abi.POWER_ZIPF),
                                                   (3, 20, 4, 2, abi.POWER_EQUAL)])
def test_events_equal_restatement(seed, n_inst, nv, R, kind):
    p = abi.gen_params(seed=seed, n_instances=n_inst, n_vals=nv, rounds_min=1, rounds_max=R, nil_permille=300)
    hb = ol.gen_batch(p)
    power = ol.gen_power(seed, 3, nv, kind, 1, 100)
    hb.instance_set = (np.arange(n_inst) % 3).astype(np.uint32)
    cfg = abi.config(abi.MODE_REFERENCE, 0, R)
    codes, _, _, offs, ev = ol.events(cfg, hb, power, threads=2)
    want = restate(hb, power, R)
    got = [(int(e["vote"]), int(e["instance"]), int(e["value"]), int(e["round"]), int(e["kind"])) for e in ev]
    assert got == want
    assert (ev["message"] == 0).all()
    # offsets: per instance, the records of its votes
    for i in range(n_inst):
        seg = ev[int(offs[i]):int(offs[i + 1])]
        assert (seg["instance"] == i).all()
    # the codes the checker's tally left say the same events
    c = codes & abi.CODE_EVENT_MASK
    assert int(((c >= 1) & (c <= 5)).sum()) == len(ev)
    assert any(e[4] in (abi.EV_POLKA_VALUE, abi.EV_PRECOMMIT_VALUE) for e in want)


def test_events_round_skip_and_messages():
    """DEDUP + RoundSkip + State machine: a RoundSkip record before the vote's own
    event, both with the vote's message nibble; REJECTED / INVALID votes give none"""
    p = abi.gen_params(seed=9, n_instances=60, n_vals=30, rounds_min=1, rounds_max=4, nil_permille=300,
                       dup_permille=100, equiv_permille=100, higher_permille=50)
    hb = ol.gen_batch(p)
    power = ol.gen_power(9, 2, 30, abi.POWER_ZIPF, 1, 1000)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE | abi.FLAG_DISTINCT_VALUES, 5)
    codes, st, bad, offs, ev = ol.events(cfg, hb, power, None, abi.new_states(60, 1, abi.STEP_PREVOTE), threads=2)
    c2, s2, b2 = ol.tally(cfg, hb, power, None, abi.new_states(60, 1, abi.STEP_PREVOTE))
    assert np.array_equal(codes, c2) and st.tobytes() == s2.tobytes() and bad == b2
    skips = ev[ev["kind"] == abi.EV_ROUND_SKIP]
    assert len(skips) == int(((codes & abi.CODE_SKIP) != 0).sum()) > 0
    for e in skips:
        assert e["value"] == abi.NIL and e["message"] == codes[e["vote"]] >> 4
    votes = ev["vote"]
    assert np.all(np.diff(votes.astype(np.int64)) >= 0)  # vote order within the stream
    ce = codes[votes] & abi.CODE_EVENT_MASK
    assert not np.isin(ce, [abi.CODE_INVALID, abi.CODE_REJECTED]).any()
    assert (ev["message"] != 0).any()
