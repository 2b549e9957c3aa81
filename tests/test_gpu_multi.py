"""The native multi-GPU driver (agnes_multi_*, include/agnes.h) on the one GPU of
the box: several contexts on device 0 stand in for several devices, so the
instance-range split, the per-range rebasing (offsets, instance ids, default
instance sets) and the threads are exercised; results equal the checker's."""
import numpy as np
import pytest
import torch

import oracle_lib as ol
from agnes_amd import abi
from agnes_amd.lib import AgnesError
from agnes_amd.multi import MultiEngine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n_dev", [1, 2, 3])
@pytest.mark.parametrize("mode,flags,R,n_sets", [(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4, 16),
                                                 (abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP, 5, 3),
                                                 (abi.MODE_REFERENCE, 0, 1, 1)])
def test_multi_tally_equals_checker(n_dev, mode, flags, R, n_sets):
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    gp = dict(n_instances=4001, n_vals=60, rounds_min=1, rounds_max=max(1, R - 1), nil_permille=250)
    if mode == abi.MODE_DEDUP:
        gp.update(dup_permille=100, equiv_permille=100, higher_permille=50)
    p = abi.gen_params(seed=91 + n_dev, **gp)
    hb = ol.gen_batch(p)
    hb.instance[::997] += 1  # a few votes naming the wrong instance: INVALID on every route
    power = ol.gen_power(91, n_sets, 60, abi.POWER_UNIFORM, 1, 1000)
    cfg = abi.config(mode, flags, R)
    st0 = abi.new_states(4001, 1, abi.STEP_PREVOTE) if flags & abi.FLAG_STATE_MACHINE else None
    m = MultiEngine([0] * n_dev)
    try:
        m.upload_power(power)
        codes, st, stats = m.tally(cfg, hb, st0)
    finally:
        m.close()
    want, want_st, bad = ol.tally(cfg, hb, power, None, st0, threads=8)
    assert np.array_equal(codes, want)
    if st0 is not None:
        assert st.tobytes() == want_st.tobytes()
    assert int(stats["n_invalid"].sum()) == bad > 0
    assert int(stats["n_votes"].sum()) == hb.n_votes
    assert stats["i0"][0] == 0 and stats["i1"][-1] == 4001 and (stats["i1"][:-1] == stats["i0"][1:]).all()


def test_multi_rejects():
    m = MultiEngine([0])
    try:
        hb = ol.gen_batch(abi.gen_params(seed=1, n_instances=4, n_vals=8))
        hb.offsets = hb.offsets.copy()
        hb.offsets[2], hb.offsets[1] = hb.offsets[1], hb.offsets[2] + 1  # not monotone
        with pytest.raises(AgnesError):
            m.tally(abi.config(abi.MODE_REFERENCE, 0, 1), hb)
    finally:
        m.close()


# ------------------------------------------- C5 through the native driver (tally_one)

def _c5_batch(seed, n_vals, dedup, rounds=1):
    gen = dict(n_instances=1, n_vals=n_vals, rounds_min=rounds, rounds_max=rounds, nil_permille=200)
    if dedup:
        gen.update(dup_permille=100, equiv_permille=100)
    return ol.gen_batch(abi.gen_params(seed=seed, **gen))


@pytest.mark.parametrize("n_dev", [1, 2, 3])
@pytest.mark.parametrize("mode", [abi.MODE_REFERENCE, abi.MODE_DEDUP])
@pytest.mark.parametrize("sm", [False, True])
def test_multi_tally_one_equals_checker(n_dev, mode, sm):
    """One instance's stream split over 1..3 contexts (agnes_multi_tally_one): pass A,
    the all-gather of the slice totals, pass B (+ the DEDUP MIN and the State
    machine's MIN / MAX exchanges) through pinned host memory; codes, the State and
    the final executors equal one stream tallied by the checker (round_votes.rs:48-67,
    vote_executor.rs:20-36, state_machine.rs:196-211)."""
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    n_vals = 20_000
    hb = _c5_batch(11 + n_dev, n_vals, mode == abi.MODE_DEDUP, rounds=2)
    power = ol.gen_power(11, 1, n_vals, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(mode, abi.FLAG_STATE_MACHINE if sm else 0, 2)
    st0 = abi.new_states(1, 1, abi.STEP_PREVOTE) if sm else None
    m = MultiEngine([0] * n_dev)
    try:
        m.upload_power(power)
        codes, st, counts, stats = m.tally_one(cfg, hb, st0, segments=97)
    finally:
        m.close()
    want, want_st, bad = ol.tally(cfg, hb, power, None, st0)
    if not np.array_equal(codes, want):
        k = int(np.nonzero(codes != want)[0][0])
        raise AssertionError(f"code {k}: gpu {codes[k]:#x} checker {want[k]:#x}")
    if sm:
        assert st.tobytes() == want_st.tobytes() and st["decided"][0] == 1
    # the final executors: every counted vote's weight (REFERENCE: all; DEDUP: firsts)
    counted = (want & 7) != abi.CODE_INVALID
    counted &= (want & 7) != abi.CODE_REJECTED
    w = power[0][hb.validator]
    for r in range(2):
        for t in range(2):
            sel = counted & (hb.round == r) & (hb.type == t)
            nil = hb.value == abi.NIL
            k = 2 * r + t
            assert counts["value_w"][k] == int(w[sel & ~nil].sum()) and counts["nil_w"][k] == int(w[sel & nil].sum())
    assert int(stats["n_votes"].sum()) == hb.n_votes


def test_multi_tally_one_rccl_one_rank():
    """The RCCL exchange path (ncclCommInitAll, all_gather / all_reduce MIN / MAX)
    with one device (a one-rank communicator: the box has one GPU)."""
    hb = _c5_batch(5, 4096, True)
    power = ol.gen_power(5, 1, 4096, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE, 1)
    st0 = abi.new_states(1, 1, abi.STEP_PREVOTE)
    m = MultiEngine([0])
    try:
        m.exchange(abi.MULTI_EXCHANGE_RCCL)
        m.upload_power(power)
        codes, st, _, _ = m.tally_one(cfg, hb, st0, segments=33)
    finally:
        m.close()
    want, want_st, _ = ol.tally(cfg, hb, power, None, st0)
    assert np.array_equal(codes, want) and st.tobytes() == want_st.tobytes()
    m = MultiEngine([0, 0])
    try:
        with pytest.raises(AgnesError):
            m.exchange(abi.MULTI_EXCHANGE_RCCL)  # one rank per device
    finally:
        m.close()


@pytest.mark.parametrize("ops", [1, 2, 4, 8, 15])
def test_multi_rccl_selfcheck_fallback(ops):
    """The RCCL self-check: the first collective of each kind (MIN u64 = the DEDUP
    first-vote table, MIN i64 = P1 / C, MAX i64 = valid / decision round, all-gather =
    the slice totals) is compared with the host exchange of the same data.  A test
    hook flips a received byte of the chosen kinds: the call must still be exact (the
    host result replaces RCCL's), report AGNES_MULTI_X_FALLBACK, and the handle's next
    call must run on the host exchange."""
    hb = _c5_batch(7, 4096, True)
    power = ol.gen_power(7, 1, 4096, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE, 1)
    st0 = abi.new_states(1, 1, abi.STEP_PREVOTE)
    want, want_st, _ = ol.tally(cfg, hb, power, None, st0)
    m = MultiEngine([0])
    try:
        m.exchange(abi.MULTI_EXCHANGE_RCCL)
        m.upload_power(power)
        codes, st, _, stats = m.tally_one(cfg, hb, st0, segments=33)  # clean: RCCL, checked, no fallback
        assert np.array_equal(codes, want) and st.tobytes() == want_st.tobytes()
        assert int(stats["exchange"][0]) == abi.MULTI_X_RCCL
        m.test_corrupt(ops)
        codes, st, _, stats = m.tally_one(cfg, hb, st0, segments=33)
        assert np.array_equal(codes, want) and st.tobytes() == want_st.tobytes()
        assert int(stats["exchange"][0]) & abi.MULTI_X_FALLBACK
        m.test_corrupt(0)
        codes, st, _, stats = m.tally_one(cfg, hb, st0, segments=33)  # the handle left RCCL
        assert np.array_equal(codes, want) and st.tobytes() == want_st.tobytes()
        assert not int(stats["exchange"][0]) & abi.MULTI_X_RCCL
        assert int(stats["exchange"][0]) & abi.MULTI_X_FALLBACK
    finally:
        m.close()


def test_multi_rccl_broken_every_collective():
    """An RCCL that corrupts EVERY collective (hook bits 4..7), with only the first
    kind's self-check re-armed: once that check fails, the call's later collectives
    (already checked kinds included) must take the host exchange, so the results stay
    exact and the call reports AGNES_MULTI_X_FALLBACK (a failed check had
    only replaced the one collective it checked)."""
    hb = _c5_batch(8, 4096, True)
    power = ol.gen_power(8, 1, 4096, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE, 1)
    st0 = abi.new_states(1, 1, abi.STEP_PREVOTE)
    want, want_st, _ = ol.tally(cfg, hb, power, None, st0)
    m = MultiEngine([0])
    try:
        m.exchange(abi.MULTI_EXCHANGE_RCCL)
        m.upload_power(power)
        codes, st, _, stats = m.tally_one(cfg, hb, st0, segments=33)  # every kind checked, clean
        assert int(stats["exchange"][0]) == abi.MULTI_X_RCCL
        m.test_corrupt(0x1 | 0xF0)  # DEDUP's MIN u64 (the call's first) re-checked; every kind broken
        codes, st, _, stats = m.tally_one(cfg, hb, st0, segments=33)
        assert np.array_equal(codes, want) and st.tobytes() == want_st.tobytes()
        assert int(stats["exchange"][0]) & abi.MULTI_X_FALLBACK
    finally:
        m.close()


@pytest.mark.parametrize("n_dev", [1, 3])
def test_multi_edges_gathered(n_dev):
    """The edge summary of the last agnes_multi_tally, gathered from every range in
    the batch's own numbering, equals the checker's orc_edges over the whole batch."""
    p = abi.gen_params(seed=4, n_instances=3001, n_vals=50, rounds_min=1, rounds_max=3, nil_permille=300)
    hb = ol.gen_batch(p)
    power = ol.gen_power(4, 5, 50, abi.POWER_UNIFORM, 1, 100)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 3)
    m = MultiEngine([0] * n_dev)
    try:
        m.upload_power(power)
        codes, _, _ = m.tally(cfg, hb, abi.new_states(3001, 1, abi.STEP_PREVOTE))
        offs, recs = m.edges(cfg, p.n_instances)
    finally:
        m.close()
    o_offs, o_recs = ol.edges(cfg, hb, codes)
    assert np.array_equal(offs, o_offs)
    assert recs.tobytes() == o_recs.tobytes() and len(recs) > 3001
