"""Pins the CPU checker (oracle/) to the reference's own test vectors, then
cross-checks it against the independent Python restatement (tests/pyref.py).

CPU only.  The reference's golden vectors are its two unit tests
(round_votes.rs:107-132, state_machine.rs:331-345); see tests/golden/.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

import oracle_lib as ol
import pyref
from agnes_amd import abi

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF = json.load(open(os.path.join(GOLD, "reference_tests.json")))
REGRESS = json.load(open(os.path.join(GOLD, "regress_small.json")))

EV_BY_NAME = {n: i for i, n in enumerate(abi.EVENT_NAMES)}
CODE_OF_EVENT = {None: 0, "PolkaAny": 1, "PolkaNil": 2, "PolkaValue": 3, "PrecommitAny": 4,
                 "PrecommitValue": 5}


def nil_or(v):
    return abi.NIL if v is None else v


def test_add_votes_golden_oracle():
    g = REF["add_votes"]
    rv = ol.RoundVotes(1, 0, g["total"])  # RoundVotes::new(1, 0, total) :115
    got = [abi.THRESH_NAMES[rv.add_vote(t, nil_or(v), g["weight"])[0]] for t, v in g["votes"]]
    assert got == g["thresh"]


def test_add_votes_golden_pyref():
    g = REF["add_votes"]
    c = pyref.Count(g["total"])
    got = [abi.THRESH_NAMES[c.add(nil_or(v), g["weight"])[0]] for _, v in g["votes"]]
    assert got == g["thresh"]


def _event(d):
    e = abi.Event()
    e.kind = EV_BY_NAME[d["kind"]]
    e.round = d["round"]
    e.value = d.get("value", 0)
    e.pol_round = d.get("pol_round", 0)
    return e


def _msg_matches(m, want):
    if want is None:
        return m is None
    if m is None:
        return False
    if abi.MSG_NAMES[m.kind] != want["kind"] or m.round != want["round"]:
        return False
    if "value" in want and m.value != want["value"]:
        return False
    if "pol_round" in want and m.pol_round != want["pol_round"]:
        return False
    if "vote_type" in want and m.vote_type != ["Prevote", "Precommit"].index(want["vote_type"]):
        return False
    return True


def test_happy_case_golden_oracle():
    g = REF["happy_case"]
    s = ol.state_new(g["height"])
    for ev, want in zip(g["events"], g["messages"]):
        s, m = ol.state_apply(s, ev["round"], _event(ev))
        assert _msg_matches(m, want), (ev, want)
    assert abi.STEP_NAMES[s.step] == g["final_step"]


def test_happy_case_golden_pyref():
    g = REF["happy_case"]
    s = pyref.State(height=g["height"])
    for ev, want in zip(g["events"], g["messages"]):
        s, m = pyref.apply(s, ev["round"], EV_BY_NAME[ev["kind"]], ev.get("value", 0),
                           ev.get("pol_round", 0))
        assert m is not None and abi.MSG_NAMES[m.kind] == want["kind"]
        assert m.round == want["round"] and m.value == want["value"]
    assert abi.STEP_NAMES[s.step] == g["final_step"]


@pytest.mark.parametrize("name", ["c1_value", "c1_nil", "c1_mixed"])
def test_c1_vote_executor_traces(name):
    g = REF[name]
    rv = ol.RoundVotes(1, 0, g["total"])  # VoteExecutor::new(1, 4)
    got = []
    for t, v in g["votes"]:
        e, _ = rv.ve_apply(t, nil_or(v), g["weight"])
        got.append(None if e == abi.EV_NONE else abi.EVENT_NAMES[e])
    assert got == g["events"]


def _c1_state_after_proposal():
    s = ol.state_new(1)
    s, _ = ol.state_apply(s, 0, _event({"kind": "NewRoundProposer", "round": 0, "value": 7}))
    s, _ = ol.state_apply(s, 0, _event({"kind": "Proposal", "round": 0, "value": 7,
                                        "pol_round": -1}))
    assert s.step == abi.STEP_PREVOTE
    return s


def test_c1_batch_composed_with_state_machine():
    """Config C1 through the batch contract: weights = power table of 4 x 1."""
    g = REF["c1_value"]
    n = len(g["votes"])
    b = ol.batch_from_lists([0] * n, [0] * n, [t for t, _ in g["votes"]],
                            [nil_or(v) for _, v in g["votes"]], [k % 4 for k in range(n)], [0, n])
    st0 = np.frombuffer(bytes(_c1_state_after_proposal()), dtype=abi.STATE_DTYPE).copy()
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)
    codes, st, nbad = ol.tally(cfg, b, np.ones((1, 4), np.int64), states=st0)
    assert nbad == 0
    ev = [int(c) & abi.CODE_EVENT_MASK for c in codes]
    assert ev == [CODE_OF_EVENT[e] for e in g["events"]]
    msgs = [int(c) >> abi.CODE_MSG_SHIFT for c in codes]
    want = [0, 0, abi.VMSG_PRECOMMIT_VALUE, 0, 0, 0, abi.VMSG_DECISION, 0]
    assert msgs == want
    assert st["step"][0] == abi.STEP_COMMIT and st["decided"][0] == 1


def _states_from_json(lst):
    arr = abi.new_states(len(lst))
    for k, s in enumerate(lst):
        arr[k]["height"], arr[k]["round"], arr[k]["step"] = s["height"], s["round"], s["step"]
        if s["locked"]:
            arr[k]["locked_present"] = 1
            arr[k]["locked_round"], arr[k]["locked_value"] = s["locked"]
        if s["valid"]:
            arr[k]["valid_present"] = 1
            arr[k]["valid_round"], arr[k]["valid_value"] = s["valid"]
        if s.get("decision"):
            arr[k]["decided"] = 1
            arr[k]["decision_round"], arr[k]["decision_value"] = s["decision"]
    return arr


def _cmp_states(a, b):
    for f in ["height", "round", "step", "locked_present", "valid_present", "decided"]:
        np.testing.assert_array_equal(a[f], b[f], err_msg=f)
    for pres, fields in [("locked_present", ["locked_round", "locked_value"]),
                         ("valid_present", ["valid_round", "valid_value"]),
                         ("decided", ["decision_round", "decision_value"])]:
        m = a[pres] == 1
        for f in fields:
            np.testing.assert_array_equal(a[f][m], b[f][m], err_msg=f)


@pytest.mark.parametrize("case", REGRESS, ids=[c["name"] for c in REGRESS])
def test_regress_fixtures_oracle(case):
    b = ol.batch_from_lists(case["instance"], case["round"], case["type"], case["value"],
                            case["validator"], case["offsets"])
    cfg = abi.config(case["mode"], case["flags"], case["max_rounds"])
    st_in = _states_from_json(case["states_in"]) if "states_in" in case else None
    codes, st, _ = ol.tally(cfg, b, np.array(case["power"], np.int64),
                            np.array(case["totals"], np.int64), st_in)
    assert codes.tolist() == case["codes"]
    if st_in is not None:
        _cmp_states(st, _states_from_json(case["states_out"]))


# --------------------------------------------------------------- cross-check


def _to_pyref_states(arr):
    out = []
    for s in arr:
        out.append(pyref.State(
            height=int(s["height"]), round=int(s["round"]), step=int(s["step"]),
            locked=(int(s["locked_round"]), int(s["locked_value"])) if s["locked_present"] else None,
            valid=(int(s["valid_round"]), int(s["valid_value"])) if s["valid_present"] else None,
            decision=(int(s["decision_round"]), int(s["decision_value"])) if s["decided"] else None))
    return out


def _from_pyref_states(lst):
    return _states_from_json([{
        "height": s.height, "round": s.round, "step": s.step,
        "locked": list(s.locked) if s.locked else None,
        "valid": list(s.valid) if s.valid else None,
        "decision": list(s.decision) if s.decision else None} for s in lst])


I64 = st.integers(min_value=-(1 << 63), max_value=(1 << 63) - 1)


@st.composite
def small_batches(draw):
    n_inst = draw(st.integers(1, 4))
    n_vals = draw(st.integers(1, 6))
    n_sets = draw(st.integers(1, 3))
    max_rounds = draw(st.integers(1, 4))
    huge = draw(st.booleans())
    wgen = I64 if huge else st.integers(-3, 20)
    power = [[draw(wgen) for _ in range(n_vals)] for _ in range(n_sets)]
    totals = [draw(wgen) if draw(st.booleans()) else sum(p) for p in power]
    totals = [pyref.i64(t) for t in totals]
    inst, rnd, typ, val, vid, offs = [], [], [], [], [], [0]
    for i in range(n_inst):
        k = draw(st.integers(0, 24))
        for _ in range(k):
            bad = draw(st.integers(0, 30)) == 0
            inst.append(i if not bad else i + 1)
            rnd.append(draw(st.integers(0, max_rounds)))  # == max_rounds -> invalid
            typ.append(draw(st.integers(0, 1)))
            val.append(draw(st.sampled_from([abi.NIL, 5, 6, 5])))
            vid.append(draw(st.integers(0, n_vals)))  # == n_vals -> invalid
        offs.append(len(rnd))
    mode = draw(st.sampled_from([abi.MODE_REFERENCE, abi.MODE_DEDUP]))
    flags = draw(st.integers(0, 7))
    step = draw(st.integers(0, 4))
    r0 = draw(st.integers(0, 2))
    return dict(inst=inst, rnd=rnd, typ=typ, val=val, vid=vid, offs=offs, power=power,
                totals=totals, mode=mode, flags=flags, max_rounds=max_rounds, step=step, r0=r0)


@settings(max_examples=300, deadline=None)
@given(small_batches())
def test_oracle_matches_pyref(d):
    b = ol.batch_from_lists(d["inst"], d["rnd"], d["typ"], d["val"], d["vid"], d["offs"])
    n_inst = len(d["offs"]) - 1
    st0 = abi.new_states(n_inst, 1, d["step"], d["r0"])
    cfg = abi.config(d["mode"], d["flags"], d["max_rounds"])
    codes, st_out, _ = ol.tally(cfg, b, np.array(d["power"], np.int64),
                                np.array(d["totals"], np.int64), st0)
    pb = pyref.Batch(d["inst"], d["rnd"], d["typ"], d["val"], d["vid"], d["offs"])
    pcodes, pst = pyref.tally(pb, d["power"], d["totals"], d["mode"], d["flags"],
                              d["max_rounds"], _to_pyref_states(st0))
    assert codes.tolist() == pcodes
    if d["flags"] & abi.FLAG_STATE_MACHINE:
        _cmp_states(st_out, _from_pyref_states(pst))


@settings(max_examples=300, deadline=None)
@given(st.integers(0, 4), st.integers(-1, 3), st.integers(0, 12), st.integers(-2, 3),
       st.integers(-2, 3), st.sampled_from([3, 4]), st.booleans(), st.booleans(), st.booleans())
def test_state_apply_matches_pyref(step, r0, kind, rnd, pol, value, locked, valid, distinct):
    s = ol.state_new(1)
    s.step, s.round = step, r0
    if locked:
        s.locked_present, s.locked_round, s.locked_value = 1, r0 - 1, 3
    if valid:
        s.valid_present, s.valid_round, s.valid_value = 1, r0, 4
    ev = abi.Event(rnd, pol, value, kind)
    flags = abi.FLAG_DISTINCT_VALUES if distinct else 0
    s2, m = ol.state_apply(s, rnd, ev, flags)
    ps = pyref.State(1, r0, step, (r0 - 1, 3) if locked else None, (r0, 4) if valid else None)
    ps2, pm = pyref.apply(ps, rnd, kind, value, pol, distinct)
    assert (m is None) == (pm is None)
    if m is not None:
        assert (m.kind, m.round, m.value) == (pm.kind, pm.round, pm.value)
        if m.kind == abi.MSG_PROPOSAL:
            assert m.pol_round == pm.pol_round
        if m.kind == abi.MSG_VOTE:
            assert m.vote_type == pm.vote_type
        if m.kind == abi.MSG_TIMEOUT:
            assert m.timeout_step == pm.timeout_step
    assert (s2.step, s2.round) == (ps2.step, ps2.round)
    assert bool(s2.locked_present) == (ps2.locked is not None)
    assert bool(s2.valid_present) == (ps2.valid is not None)
    if ps2.valid:
        assert (s2.valid_round, s2.valid_value) == ps2.valid


def test_wrapping_quorum():
    L = ol.lib()
    big = (1 << 63) - 1
    # 3 * i64::MAX wraps to i64::MAX - 2*2^63 ... compare with Python model
    for v, t in [(big, 4), (big // 3 + 1, 1), (-5, -8), (1 << 62, 1 << 62), (0, -1)]:
        assert bool(L.orc_is_quorum(v, t)) == pyref.quorum(v, t), (v, t)
        assert bool(L.orc_is_one_third(v, t)) == pyref.one_third(v, t), (v, t)


def test_mt_equals_single_thread():
    p = abi.gen_params(seed=11, n_instances=300, n_vals=21, rounds_min=1, rounds_max=3,
                       nil_permille=300, dup_permille=100, equiv_permille=100,
                       higher_permille=50)
    b = ol.gen_batch(p)
    power = ol.gen_power(11, 16, 21, abi.POWER_ZIPF, 1, 10000)
    st0 = abi.new_states(300, 1, abi.STEP_PREVOTE)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 5)
    c1, s1, n1 = ol.tally(cfg, b, power, states=st0)
    c2, s2, n2 = ol.tally(cfg, b, power, states=st0, threads=7)
    assert (c1 == c2).all() and n1 == n2 == 0
    assert s1.tobytes() == s2.tobytes()


def test_generator_shape():
    p = abi.gen_params(seed=3, n_instances=50, n_vals=13, rounds_min=1, rounds_max=4)
    b = ol.gen_batch(p)
    off = b.offsets
    for i in range(50):
        seg = slice(int(off[i]), int(off[i + 1]))
        assert (b.instance[seg] == i).all()
        R = (off[i + 1] - off[i]) // 26
        # every (round, type, validator) exactly once: the Feistel walk is a bijection
        keys = set(zip(b.round[seg].tolist(), b.type[seg].tolist(), b.validator[seg].tolist()))
        assert len(keys) == int(off[i + 1] - off[i]) == R * 26
        # rounds are sequential blocks
        assert (np.diff(b.round[seg].astype(int)) >= 0).all()


def test_generator_abstention():
    """absent_permille (round 6): each round keeps a prefix of its permuted order, so
    instance lengths take any value (offsets off multiples of 4, the ragged streams a
    real validator set produces when some validators do not vote); every kept vote is a
    distinct (round, type, validator) of the full round, rounds stay in order, and the
    instance's length is the sum of its rounds' kept counts."""
    full = abi.gen_params(seed=5, n_instances=400, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300)
    p = abi.gen_params(seed=5, n_instances=400, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                       absent_permille=50)
    b, bf = ol.gen_batch(p), ol.gen_batch(full)
    lens, lf = np.diff(b.offsets.astype(np.int64)), np.diff(bf.offsets.astype(np.int64))
    assert (lens <= lf).all() and (lens < lf).mean() > 0.9
    assert 0.9 < lens.sum() / lf.sum() < 0.99
    assert len(set((b.offsets % 4).tolist())) == 4  # every residue: no 4-aligned stream
    for i in range(0, 400, 7):
        seg = slice(int(b.offsets[i]), int(b.offsets[i + 1]))
        keys = list(zip(b.round[seg].tolist(), b.type[seg].tolist(), b.validator[seg].tolist()))
        assert len(set(keys)) == len(keys)
        assert (np.diff(b.round[seg].astype(int)) >= 0).all()
        assert (b.instance[seg] == i).all()
    L = ol.lib()
    assert [int(L.orc_gen_instance_votes(C.byref(p), i)) for i in range(5)] == lens[:5].tolist()
