"""Batched ConsensusExecutor::apply_msg (agnes_apply_msgs) on the CPU: the checker
(orc_apply_msgs) pinned to the reference's happy-case test driven as messages
(state_machine.rs:331-345 through consensus_executor.rs:54-86), then against the
independent Python restatement (tests/pyref.py apply_msgs) over generated
multi-round scripts (agnes_amd/script.py).  CPU only."""
import json
import os

import numpy as np
import pytest

import oracle_lib as ol
import pyref
from agnes_amd import abi
from agnes_amd.script import gen_script

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF = json.load(open(os.path.join(GOLD, "reference_tests.json")))
NIL = abi.NIL


def _states(n, height=1):
    return abi.new_states(n, height, abi.STEP_NEW_ROUND)


def _happy_script():
    """The happy case as messages: the executor's NewRound (proposer, value 7), the
    Proposal(7, pol -1), three prevotes for 7 of four validators, three precommits."""
    kinds = [abi.IN_NEW_ROUND, abi.IN_PROPOSAL] + [abi.IN_VOTE] * 6
    typ = [0, 0, 0, 0, 0, 1, 1, 1]
    val = [7] * 8
    validator = [0, 0, 0, 1, 2, 0, 1, 2]
    n = len(kinds)
    b = ol.batch_from_lists([0] * n, [0] * n, typ, val, validator, [0, n])
    return b, np.array(kinds, np.uint8), np.array([0, -1] + [0] * 6, np.int32)


def _msg_tuple(m):
    return (int(m["kind"]), int(m["round"]), int(m["value"]), int(m["pol_round"]), int(m["vote_type"]),
            int(m["timeout_step"]))


def _py_msg_tuple(m):
    if m is None:
        return (0, 0, 0, 0, 0, 0)
    return (m.kind, m.round & ((1 << 64) - 1) if m.round < 0 else m.round, m.value,
            m.pol_round, m.vote_type, m.timeout_step)


def test_happy_case_as_messages():
    g = REF["happy_case"]
    b, kinds, pol = _happy_script()
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)
    codes, st, msgs, bad = ol.apply_msgs(cfg, b, kinds, pol, np.ones((1, 4), np.int64), _states(1, g["height"]))
    assert bad == 0
    produced = [m for m in msgs if m["kind"] != abi.MSG_NONE]
    assert len(produced) == len(g["messages"])
    for m, want in zip(produced, g["messages"]):
        assert abi.MSG_NAMES[m["kind"]] == want["kind"] and m["round"] == want["round"]
        assert m["value"] == want["value"]
        if "pol_round" in want:
            assert m["pol_round"] == want["pol_round"]
        if "vote_type" in want:
            assert m["vote_type"] == ["Prevote", "Precommit"].index(want["vote_type"])
    # the messages come from the NewRound, the Proposal, the third prevote and the third precommit
    assert [int(k) for k in np.nonzero(msgs["kind"])[0]] == [0, 1, 4, 7]
    assert list(codes) == [0, 0, 0, 0, abi.CODE_POLKA_VALUE, 0, 0, abi.CODE_PRECOMMIT_VALUE]
    assert abi.STEP_NAMES[st["step"][0]] == g["final_step"]
    assert st["decided"][0] == 1 and st["decision_value"][0] == 7


def _pyref_run(sc, kinds, pol, power, flags, R, states):
    b = pyref.Batch([int(x) for x in sc.instance], [int(x) for x in sc.round], [int(x) for x in sc.type],
                    [int(x) for x in sc.value], [int(x) for x in sc.validator], [int(x) for x in sc.offsets],
                    None if getattr(sc, "weight", None) is None else [int(x) for x in sc.weight])
    pw = [[int(x) for x in row] for row in power]
    totals = [int(x) for x in ol.set_totals(power)]
    st0 = [pyref.State(height=int(s["height"])) for s in states]
    return pyref.apply_msgs(b, [int(k) for k in kinds], None if pol is None else [int(p) for p in pol], pw,
                            totals, flags, R, st0)


@pytest.mark.parametrize("seed,flags,rounds,weights", [(1, 0, 3, False), (2, abi.FLAG_DISTINCT_VALUES, 4, False),
                                                       (3, 0, 1, False), (4, abi.FLAG_DISTINCT_VALUES, 2, True)])
def test_oracle_matches_pyref_on_scripts(seed, flags, rounds, weights):
    sc = gen_script(seed, 24, 7, rounds)
    rng = np.random.default_rng(seed)
    power = rng.integers(1, 50, size=(3, 7)).astype(np.int64)
    if weights:
        sc.weight = rng.integers(-2, 40, size=sc.n_votes).astype(np.int64)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE | flags, rounds)
    states = _states(sc.n_instances)
    codes, st, msgs, bad = ol.apply_msgs(cfg, sc, sc.kinds, sc.pol_round, power, states)
    pcodes, pst, pmsgs = _pyref_run(sc, sc.kinds, sc.pol_round, power, flags, rounds, states)
    assert list(codes) == pcodes
    assert bad == sum(1 for c in pcodes if c == abi.CODE_INVALID)
    for j, (m, pm) in enumerate(zip(msgs, pmsgs)):
        assert _msg_tuple(m)[:1] == _py_msg_tuple(pm)[:1], j
        if pm is not None:
            assert (int(m["round"]), int(m["value"]), int(m["vote_type"]), int(m["timeout_step"])) == \
                (pm.round, pm.value, pm.vote_type, pm.timeout_step), j
            if pm.kind == pyref.M_PROPOSAL:
                assert int(m["pol_round"]) == pm.pol_round
    for s, ps in zip(st, pst):
        assert (int(s["round"]), int(s["step"])) == (ps.round, ps.step)
        assert bool(s["locked_present"]) == (ps.locked is not None)
        if ps.locked is not None:
            assert (int(s["locked_round"]), int(s["locked_value"])) == ps.locked
        assert bool(s["valid_present"]) == (ps.valid is not None)
        if ps.valid is not None:
            assert (int(s["valid_round"]), int(s["valid_value"])) == ps.valid
        assert bool(s["decided"]) == (ps.decision is not None)
        if ps.decision is not None:
            assert (int(s["decision_round"]), int(s["decision_value"])) == ps.decision


def test_script_shape():
    """Scripts move instances over rounds and decide: multi-round coverage."""
    sc = gen_script(11, 200, 10, 4)
    assert sc.n_votes == 200 * 4 * (5 + 2 * 10)
    assert (np.diff(sc.offsets.astype(np.int64)) == 4 * 25).all()
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4)
    power = np.ones((1, 10), np.int64)
    codes, st, msgs, bad = ol.apply_msgs(cfg, sc, sc.kinds, sc.pol_round, power, _states(200))
    assert st["decided"].sum() > 100
    assert (st["round"] == 3).sum() > 100  # the rounds before the last end in round_skip
    kinds = set(int(k) for k in msgs["kind"])
    assert {abi.MSG_NEW_ROUND, abi.MSG_PROPOSAL, abi.MSG_VOTE, abi.MSG_TIMEOUT, abi.MSG_DECISION} <= kinds
    assert bad > 0 and (codes == abi.CODE_INVALID).sum() == bad
    # votes of an earlier round arrive after the next round's NewRound
    r = sc.round.astype(np.int64).reshape(200, -1)
    assert (np.diff(r, axis=1) < 0).any()


def test_script_empty_and_unknown_kinds():
    sc = gen_script(5, 0, 3, 2)
    assert sc.n_votes == 0 and sc.n_instances == 0
    b, kinds, pol = _happy_script()
    kinds = kinds.copy()
    kinds[2] = 9  # not a message kind: INVALID, no State change
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)
    codes, st, msgs, bad = ol.apply_msgs(cfg, b, kinds, pol, np.ones((1, 4), np.int64), _states(1))
    assert codes[2] == abi.CODE_INVALID and bad == 1 and msgs["kind"][2] == abi.MSG_NONE
