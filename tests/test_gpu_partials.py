"""agnes_tally_partials (C5 pass A as one reduction, include/agnes.h) against the
carried tally it replaces, and pass B over the cached weights
(AGNES_FLAG_WEIGHTS_CACHED) against pass B that gathers the power table: equal
VoteCounts (round_votes.rs:48-56), weights, codes, and the whole C5 split equal to
the checker (vote_executor.rs:20-36)."""
import dataclasses

import numpy as np
import pytest
import torch

import oracle_lib as ol
from agnes_amd import abi
from agnes_amd import dist as ad
from agnes_amd.engine import DeviceBatch, Engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    e = Engine(0)
    yield e
    e.close()


def _batch(seed, n_inst, n_vals, rounds):
    p = abi.gen_params(seed=seed, n_instances=n_inst, n_vals=n_vals, rounds_min=1, rounds_max=rounds,
                       nil_permille=250)
    hb = ol.gen_batch(p)
    # invalid votes of every kind: validator, round, type, instance id
    hb.validator[::101] = n_vals + 3
    hb.round[::103] = rounds + 7
    hb.type[::107] = 2
    hb.instance[::109] += 1
    return hb


def _valid_weights(hb, power, R, inst_of_vote, iid_of_vote, set_of_vote):
    n_sets, n_vals = power.shape
    ok = ((hb.instance == iid_of_vote) & (hb.round < R) & (hb.type <= 1) & (hb.validator < n_vals)
          & (set_of_vote < n_sets))
    w = np.zeros(hb.n_votes, dtype=np.int64)
    w[ok] = power[set_of_vote[ok], hb.validator[ok]]
    return w


CASES = [  # (one instance, segments, max_rounds, sets)
    (True, 1, 1, 1), (True, 97, 2, 1), (True, 1024, 3, 1), (False, None, 4, 5),
]


@pytest.mark.parametrize("one,segs,R,n_sets", CASES)
def test_partials_equal_carried_pass_a(eng, one, segs, R, n_sets):
    n_vals = 5000 if one else 40
    hb = _batch(17 + R, 1 if one else 300, n_vals, R)
    power = ol.gen_power(17, n_sets, n_vals, abi.POWER_ZIPF, 1, 1_000_000)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    n = hb.n_votes
    if one:
        off = ad.segment_offsets(n, segs)
        db = dataclasses.replace(db, offsets=torch.from_numpy(off.view(np.int64)).to(eng.device), instance_set=None)
        S = segs
        seg_of_vote = np.zeros(n, dtype=np.int64)
        iid = np.zeros(n, dtype=np.int64)
        set_of_vote = np.zeros(n, dtype=np.int64)
        cfg = abi.Config(abi.MODE_REFERENCE, abi.FLAG_ONE_INSTANCE, R, 0)
    else:
        S = hb.n_instances
        sets = (np.arange(S, dtype=np.uint32) * 7) % (n_sets + 1)  # set n_sets: not a set (votes invalid)
        db = dataclasses.replace(db, instance_set=torch.from_numpy(sets.view(np.int32)).to(eng.device))
        seg_of_vote = np.repeat(np.arange(S), np.diff(hb.offsets.astype(np.int64)))
        iid = seg_of_vote
        set_of_vote = sets[seg_of_vote].astype(np.int64)
        cfg = abi.Config(abi.MODE_REFERENCE, 0, R, 0)
    codes = torch.zeros(n, dtype=torch.uint8, device=eng.device)
    want = torch.empty((S, 2 * R, 3), dtype=torch.int64, device=eng.device)
    eng.fold_counts(want, flags=abi.FOLD_RESET)
    eng.tally_carried(cfg, db, codes, want)
    got = torch.full_like(want, -5)
    w = torch.full((n,), -5, dtype=torch.int64, device=eng.device)
    eng.tally_partials(cfg, db, got, w)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    assert (want[..., 0] > 0).any() and (want[..., 1] > 0).any()
    assert np.array_equal(w.cpu().numpy(), _valid_weights(hb, power, R, seg_of_vote, iid, set_of_vote))

    # pass B over the cached weights == pass B gathering, from the same carry-in
    carry = want.clone()
    carry[..., 2] = torch.where(carry[..., 2] == abi.NIL, torch.zeros_like(carry[..., 2]), carry[..., 2])
    c1, c2 = carry.clone(), carry.clone()
    k1 = torch.zeros(n, dtype=torch.uint8, device=eng.device)
    k2 = torch.zeros(n, dtype=torch.uint8, device=eng.device)
    eng.tally_carried(cfg, db, k1, c1)
    bad1 = eng.last_error_count()
    cached = abi.Config(cfg.mode, cfg.flags | abi.FLAG_WEIGHTS_CACHED, cfg.max_rounds, cfg.reserved)
    eng.tally_carried(cached, dataclasses.replace(db, weight=w), k2, c2)
    bad2 = eng.last_error_count()
    torch.cuda.synchronize()
    assert torch.equal(k1, k2) and torch.equal(c1, c2)
    assert bad1 == bad2 > 0
    assert (k1.cpu().numpy() == abi.CODE_INVALID).sum() == bad1


def test_partials_refuse_caller_weights(eng):
    """Pass A gathers the power table; a batch with caller weights (which carried
    accepts without a valid validator or set) is refused, not silently mis-tallied."""
    from agnes_amd.lib import AgnesError
    hb = _batch(5, 20, 40, 2)
    eng.upload_power(ol.gen_power(5, 1, 40, abi.POWER_UNIFORM, 1, 100))
    db = DeviceBatch.from_host(hb, eng.device)
    w = torch.ones(hb.n_votes, dtype=torch.int64, device=eng.device)
    counts = torch.empty((hb.n_instances, 4, 3), dtype=torch.int64, device=eng.device)
    with pytest.raises(AgnesError) as ex:
        eng.tally_partials(abi.Config(abi.MODE_REFERENCE, 0, 2, 0), dataclasses.replace(db, weight=w), counts)
    assert ex.value.rc == abi.E_UNSUPPORTED


@pytest.mark.parametrize("dedup", [False, True])
def test_c5_split_with_partials_equals_checker(eng, dedup):
    """tally_one_instance[_dedup] with pass A as the reduction and pass B over the
    cached weights: codes equal one stream tallied by the checker."""
    n_vals = 20_000
    gen = dict(n_instances=1, n_vals=n_vals, rounds_min=1, rounds_max=2, nil_permille=200)
    if dedup:
        gen.update(dup_permille=100, equiv_permille=100)
    hb = ol.gen_batch(abi.gen_params(seed=23, **gen))
    power = ol.gen_power(23, 1, n_vals, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(abi.MODE_DEDUP if dedup else abi.MODE_REFERENCE, 0, 2)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    n = hb.n_votes
    codes = torch.zeros(n, dtype=torch.uint8, device=eng.device)
    tmask = torch.empty(n, dtype=torch.uint8, device=eng.device)
    dbm = dataclasses.replace(db, type=tmask) if dedup else db
    wcol = torch.empty(n, dtype=torch.int64, device=eng.device)

    def tc(one, off, counts):
        cached = one.flags & abi.FLAG_WEIGHTS_CACHED
        eng.tally_carried(one, dataclasses.replace(dbm, offsets=off, instance_set=None,
                                                   weight=wcol if cached else None), codes, counts)

    def pa(one, off, counts):
        eng.tally_partials(one, dataclasses.replace(dbm, offsets=off, instance_set=None), counts, wcol)

    off = torch.from_numpy(ad.segment_offsets(n, 333).view(np.int64)).to(eng.device)
    if dedup:
        ad.tally_one_instance_dedup(tc, lambda base, f: eng.dedup_first(cfg, db, base, f),
                                    lambda base, f: eng.dedup_mask(cfg, db, base, f, tmask),
                                    lambda: eng.dedup_reject(tmask, codes, n), n, n_vals, cfg, 333,
                                    eng.device, offsets=off, fold=eng.fold_counts, partials=pa)
    else:
        ad.tally_one_instance(tc, n, cfg, 333, eng.device, offsets=off, fold=eng.fold_counts, partials=pa)
    torch.cuda.synchronize()
    got = codes.cpu().numpy()
    want, _, _ = ol.tally(cfg, hb, power)
    assert np.array_equal(got, want)
    assert (want & abi.CODE_EVENT_MASK).any()
