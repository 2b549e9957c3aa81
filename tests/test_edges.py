"""Edge-triggered summary (include/agnes.h agnes_edge) — CPU side.

The checker's orc_edges is pinned here by (1) the reference's own level-triggered
traces (C1, vote_executor.rs:20-36 as in tests/golden/reference_tests.json: prevote
v x4 gives None, None, PolkaValue, PolkaValue, so ONE edge at the third vote), (2)
an independent pure-Python restatement on generated streams, and (3) the
round-trip property: expanding the edges back reproduces every valid vote's level.
"""
import numpy as np
import pytest

import oracle_lib as ol
from agnes_amd import abi

CODE_INVALID, CODE_REJECTED = 6, 7


def py_edges(cfg, hb, codes):
    """Pure-Python restatement of the edge rule (agnes.h): per (round, type) executor
    its level (code bits 0..3, 0 initially) and its last message; edge on a level
    change or a message other than the last; INVALID / REJECTED votes and keys >=
    2*max_rounds skipped.  `prev` = level | last message << 4 before the vote."""
    out, offs = [], [0]
    for i in range(hb.n_instances):
        level = {}
        for j in range(int(hb.offsets[i]), int(hb.offsets[i + 1])):
            c = int(codes[j])
            ev = c & 7
            r, t = int(hb.round[j]), int(hb.type[j])
            if ev in (CODE_INVALID, CODE_REJECTED) or t > 1 or r >= cfg.max_rounds:
                continue
            lv, lm = level.get((r, t), (0, 0))
            m = c >> 4
            nlm = m if m else lm
            if (c & 15) != lv or nlm != lm:
                out.append((j, i, r, t, c, lv | (lm << 4)))
            level[(r, t)] = (c & 15, nlm)
        offs.append(len(out))
    return np.array(offs, dtype=np.uint64), np.array(out, dtype=abi.EDGE_DTYPE)


def expand_levels(cfg, hb, codes, recs):
    """Round trip: each valid vote's level from the edges alone (the latest edge of
    its executor at or before it; 0 if none)."""
    lv = np.zeros(hb.n_votes, dtype=np.int64) - 1
    by_inst = {}
    for e in recs:
        by_inst.setdefault(int(e["instance"]), []).append(e)
    for i in range(hb.n_instances):
        cur = {}
        es = by_inst.get(i, [])
        k = 0
        for j in range(int(hb.offsets[i]), int(hb.offsets[i + 1])):
            while k < len(es) and int(es[k]["vote"]) <= j:
                cur[(int(es[k]["round"]), int(es[k]["type"]))] = int(es[k]["code"]) & 15
                k += 1
            c = int(codes[j])
            r, t = int(hb.round[j]), int(hb.type[j])
            if (c & 7) in (CODE_INVALID, CODE_REJECTED) or t > 1 or r >= cfg.max_rounds:
                continue
            lv[j] = cur.get((r, t), 0)
    return lv


def _c1_batch(kinds):
    n = len(kinds)
    typ = [t for t, _ in kinds]
    val = [v for _, v in kinds]
    return ol.batch_from_lists([0] * n, [0] * n, typ, val, list(range(n)), [0, n])


def test_c1_prevote_value_single_edge():
    # vote_executor.rs:20-36 with VoteExecutor::new(1, 4), weight 1
    hb = _c1_batch([(0, 1)] * 4)
    hb.validator[:] = [0, 1, 2, 3]
    power = np.ones((1, 4), dtype=np.int64)
    cfg = abi.config(abi.MODE_REFERENCE, 0, 1)
    codes, _, _ = ol.tally(cfg, hb, power)
    assert list(codes) == [0, 0, abi.CODE_POLKA_VALUE, abi.CODE_POLKA_VALUE]
    offs, recs = ol.edges(cfg, hb, codes)
    assert list(offs) == [0, 1]
    assert int(recs[0]["vote"]) == 2 and int(recs[0]["code"]) == abi.CODE_POLKA_VALUE
    assert int(recs[0]["prev"]) == 0


def test_c1_mixed_and_precommit_nil():
    # prevote v, nil, v, nil -> None, None, PolkaAny, PolkaAny: one edge;
    # precommit nil x4 -> all None (vote_executor.rs:33): no edge
    power = np.ones((1, 4), dtype=np.int64)
    cfg = abi.config(abi.MODE_REFERENCE, 0, 1)
    NIL = abi.NIL
    hb = ol.batch_from_lists([0] * 8, [0] * 8, [0, 0, 0, 0, 1, 1, 1, 1],
                             [1, NIL, 1, NIL, NIL, NIL, NIL, NIL], [0, 1, 2, 3, 0, 1, 2, 3], [0, 8])
    codes, _, _ = ol.tally(cfg, hb, power)
    assert list(codes[:4]) == [0, 0, abi.CODE_POLKA_ANY, abi.CODE_POLKA_ANY]
    assert list(codes[4:]) == [0, 0, 0, 0]
    offs, recs = ol.edges(cfg, hb, codes)
    assert list(offs) == [0, 1] and int(recs[0]["vote"]) == 2


def test_state_machine_messages_are_edges():
    # C1 composed with the State machine: the first PolkaValue emits precommit(0, v)
    # (state_machine.rs:198), the first PrecommitValue the Decision (:211) — both
    # edges; the repeats are neither level changes nor messages.
    power = np.ones((1, 4), dtype=np.int64)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)
    hb = ol.batch_from_lists([0] * 8, [0] * 8, [0] * 4 + [1] * 4, [1] * 8, [0, 1, 2, 3] * 2, [0, 8])
    st = abi.new_states(1, 1, abi.STEP_PREVOTE, 0)
    codes, _, _ = ol.tally(cfg, hb, power, None, st)
    offs, recs = ol.edges(cfg, hb, codes)
    assert [int(e["vote"]) for e in recs] == [2, 6]
    assert (int(recs[0]["code"]) >> 4) == abi.VMSG_PRECOMMIT_VALUE
    assert (int(recs[1]["code"]) >> 4) == abi.VMSG_DECISION


GEN = {
    "ref_sm": (dict(n_instances=120, n_vals=30, rounds_min=1, rounds_max=3, nil_permille=300),
               abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 3),
    "dedup_skip_sm": (dict(n_instances=120, n_vals=25, rounds_min=1, rounds_max=4, nil_permille=300,
                           dup_permille=150, equiv_permille=100, higher_permille=80),
                      abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 5),
    "ref_plain": (dict(n_instances=90, n_vals=17, rounds_min=2, rounds_max=6, nil_permille=500),
                  abi.MODE_REFERENCE, 0, 6),
}


@pytest.mark.parametrize("name", list(GEN))
def test_oracle_edges_equal_python_restatement(name):
    gp, mode, flags, R = GEN[name]
    p = abi.gen_params(seed=0xE0E, **gp)
    hb = ol.gen_batch(p)
    power = ol.gen_power(0xE0E, 4, gp["n_vals"], abi.POWER_ZIPF, 1, 10000)
    cfg = abi.config(mode, flags, R)
    st = abi.new_states(p.n_instances, 1, abi.STEP_PREVOTE, 0) if flags & abi.FLAG_STATE_MACHINE else None
    codes, _, _ = ol.tally(cfg, hb, power, None, st)
    # a few invalid votes and an out-of-range round: never edges
    hb.type[5] = 2
    codes[7] = CODE_INVALID
    offs, recs = ol.edges(cfg, hb, codes)
    poffs, precs = py_edges(cfg, hb, codes)
    assert np.array_equal(offs, poffs)
    assert recs.tobytes() == precs.tobytes()
    assert len(recs) > p.n_instances  # the stream exercises the rule
    assert len(recs) < hb.n_votes // 2  # and the summary compresses it
    lv = expand_levels(cfg, hb, codes, recs)
    valid = lv >= 0
    assert np.array_equal(lv[valid], (codes[valid] & 15).astype(np.int64))


def test_empty_and_ragged_instances():
    cfg = abi.config(abi.MODE_REFERENCE, 0, 2)
    hb = ol.batch_from_lists([1, 1, 3], [0, 1, 0], [0, 0, 1], [1, 1, 1], [0, 0, 0], [0, 0, 2, 2, 3])
    codes = np.array([abi.CODE_POLKA_ANY, abi.CODE_POLKA_ANY, abi.CODE_PRECOMMIT_ANY], dtype=np.uint8)
    offs, recs = ol.edges(cfg, hb, codes)
    assert list(offs) == [0, 0, 2, 2, 3]  # rounds 0 and 1 are separate executors
    assert [int(e["instance"]) for e in recs] == [1, 1, 3]


def test_repeated_timeout_message_is_one_edge():
    # prevote v, nil, v, nil in Prevote step: PolkaAny twice, and State::apply
    # schedules timeout_prevote on each (state_machine.rs:196 repeats) — one edge.
    power = np.ones((1, 4), dtype=np.int64)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)
    NIL = abi.NIL
    hb = ol.batch_from_lists([0] * 4, [0] * 4, [0] * 4, [1, NIL, 1, NIL], [0, 1, 2, 3], [0, 4])
    st = abi.new_states(1, 1, abi.STEP_PREVOTE, 0)
    codes, _, _ = ol.tally(cfg, hb, power, None, st)
    assert [int(c) >> 4 for c in codes[2:]] == [abi.VMSG_TIMEOUT_PREVOTE] * 2
    offs, recs = ol.edges(cfg, hb, codes)
    assert list(offs) == [0, 1] and int(recs[0]["vote"]) == 2
    assert int(recs[0]["prev"]) == 0


def test_edges_arbitrary_code_streams_hypothesis():
    """Any code bytes (events, RoundSkip, messages, invalid / rejected), rounds and
    types: the checker's orc_edges equals the Python restatement."""
    from hypothesis import given, settings, strategies as st

    @settings(max_examples=150, deadline=None)
    @given(st.lists(st.integers(0, 12), min_size=1, max_size=6), st.integers(1, 4), st.data())
    def run(lengths, R, data):
        off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.uint64)
        n = int(off[-1])
        codes = np.array(data.draw(st.lists(st.integers(0, 255), min_size=n, max_size=n)), np.uint8)
        rnd = data.draw(st.lists(st.integers(0, R), min_size=n, max_size=n))
        typ = data.draw(st.lists(st.integers(0, 2), min_size=n, max_size=n))
        inst = np.repeat(np.arange(len(lengths)), lengths)
        hb = ol.batch_from_lists(inst, rnd, typ, [0] * n, [0] * n, off)
        cfg = abi.config(abi.MODE_REFERENCE, 0, R)
        offs, recs = ol.edges(cfg, hb, codes)
        poffs, precs = py_edges(cfg, hb, codes)
        assert np.array_equal(offs, poffs)
        assert recs.tobytes() == precs.tobytes()

    run()
