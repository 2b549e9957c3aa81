"""agnes_tally_events (the tally and its event stream in one C-ABI call, SURVEY.md
§8(b) agnes_tally's d_out / d_n_out) against the checker (orc_tally_labels +
orc_events): codes, States, offsets and every 24-B record bit for bit; and (round 5)
agnes_tally_records, the same records segmented by instance and written by the flow
kernel itself, plus agnes_records_compact's dense stream, on every case.

The fused route (REFERENCE without RoundSkip) counts each instance's records inside
the flow kernel; the instances it hands to its walk list (unaligned offsets, sets
outside its domain) are counted by a list pass after the tally; every other route
(DEDUP, RoundSkip, caller weights, max_rounds 15 with the State machine) runs the
full count pass.  All of them are covered here, with the records a consumer gets
from VoteExecutor::apply (vote_executor.rs:20-36; PolkaValue / PrecommitValue carry
the bucket's last non-nil value, round_votes.rs:50-54)."""
import os

import numpy as np
import pytest
import torch

import oracle_lib as ol
from agnes_amd import abi
from agnes_amd import dist as ad
from agnes_amd.engine import DeviceBatch, Engine, states_to_device, states_to_host

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    e = Engine(0)
    yield e
    e.close()


def _check(eng, cfg, hb, power, states=None, in_place=True):
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.zeros(max(hb.n_votes, 1), dtype=torch.uint8, device=eng.device)
    s_in = s_out = None
    if states is not None:
        s_in = states_to_device(states, eng.device)
        s_out = s_in if in_place else torch.zeros_like(s_in)
    offs, out = eng.tally_events(cfg, db, codes, s_in, s_out)
    torch.cuda.synchronize()
    n = int(offs[-1].item())
    assert n <= eng.events_capacity(cfg, db)
    g_codes = codes[:hb.n_votes].cpu().numpy()
    g_offs = offs.cpu().numpy().view(np.uint64)
    g_ev = out[:n].cpu().numpy().reshape(-1).view(abi.VOTE_EVENT_DTYPE)
    o_codes, o_states, _, o_offs, o_ev = ol.events(cfg, hb, power, None, states, threads=THREADS)
    assert np.array_equal(g_codes, o_codes), "codes differ"
    if states is not None:
        assert states_to_host(s_out).tobytes() == o_states.tobytes(), "States differ"
    assert np.array_equal(g_offs, o_offs), f"offsets differ (first at {np.nonzero(g_offs != o_offs)[0][:1]})"
    if g_ev.tobytes() != o_ev.tobytes():
        bad = np.nonzero(g_ev != o_ev)[0]
        raise AssertionError(f"{len(bad)} of {len(o_ev)} records differ; first {bad[0]}: "
                             f"gpu {g_ev[bad[0]]} checker {o_ev[bad[0]]}")
    # the same records as the two-call stream over the same codes
    e_offs, e_recs = eng.events(cfg, db, codes)
    assert np.array_equal(e_offs.cpu().numpy().view(np.uint64), g_offs)
    assert e_recs.cpu().numpy().tobytes() == out[:n].cpu().numpy().tobytes()
    _check_records(eng, cfg, hb, db, states, in_place, o_codes, o_states, o_offs, o_ev)
    return o_ev


def _check_records(eng, cfg, hb, db, states, in_place, o_codes, o_states, o_offs, o_ev):
    """agnes_tally_records (round 5): the same tally, the records segmented by instance
    (instance i's at rows mult * offsets[i] ..), then agnes_records_compact -> the dense
    stream; every record bit for bit against the checker's."""
    codes = torch.full((max(hb.n_votes, 1),), 0xEE, dtype=torch.uint8, device=eng.device)
    s_in = s_out = None
    if states is not None:
        s_in = states_to_device(states, eng.device)
        s_out = s_in if in_place else torch.zeros_like(s_in)
    cap = eng.events_capacity(cfg, db)
    seg = torch.full((max(cap, 1), 16), 0xCD, dtype=torch.uint8, device=eng.device)
    counts, seg = eng.tally_records(cfg, db, codes, s_in, s_out, out=seg)
    torch.cuda.synchronize()
    assert np.array_equal(codes[:hb.n_votes].cpu().numpy(), o_codes), "codes differ (tally_records)"
    if states is not None:
        assert states_to_host(s_out).tobytes() == o_states.tobytes(), "States differ (tally_records)"
    g_cnt = counts[:hb.n_instances].cpu().numpy().view(np.uint64)
    o_cnt = np.diff(o_offs.astype(np.uint64))
    assert np.array_equal(g_cnt, o_cnt), f"record counts differ (first at {np.nonzero(g_cnt != o_cnt)[0][:1]})"
    mult = 2 if cfg.flags & abi.FLAG_ROUND_SKIP else 1
    g_seg = seg.cpu().numpy().reshape(-1).view(abi.SEG_EVENT_DTYPE)
    off = hb.offsets.astype(np.int64)
    idx = np.concatenate([np.arange(mult * off[i], mult * off[i] + int(o_cnt[i])) for i in range(hb.n_instances)]
                         + [np.zeros(0, np.int64)]).astype(np.int64)
    got = g_seg[idx]
    for f in ["vote", "value", "round", "kind", "message"]:
        if not np.array_equal(got[f], o_ev[f]):
            bad = np.nonzero(got[f] != o_ev[f])[0]
            raise AssertionError(f"segmented records: field {f} differs in {len(bad)} of {len(o_ev)}; first {bad[0]}: "
                                 f"gpu {got[bad[0]]} checker {o_ev[bad[0]]}")
    d_offs, dense = eng.records_compact(cfg, db, counts, seg)
    torch.cuda.synchronize()
    assert np.array_equal(d_offs.cpu().numpy().view(np.uint64), o_offs)
    n = int(o_offs[-1])
    assert dense[:n].cpu().numpy().tobytes() == o_ev.tobytes(), "compacted records differ"


@pytest.mark.parametrize("flags", [abi.FLAG_STATE_MACHINE, 0, abi.FLAG_STATE_MACHINE | abi.FLAG_DISTINCT_VALUES])
def test_tally_events_one_round(eng, flags):
    """C2's shape: the flow kernel counts every instance"""
    p = abi.gen_params(seed=51, n_instances=3000, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200)
    hb = ol.gen_batch(p)
    power = ol.gen_power(51, 1, 100, abi.POWER_UNIFORM, 1, 1000)
    st = abi.new_states(3000, 1, abi.STEP_PREVOTE) if flags else None
    ev = _check(eng, abi.config(abi.MODE_REFERENCE, flags, 1), hb, power, st)
    assert len(ev) > 3000


@pytest.mark.parametrize("in_place", [True, False])
def test_tally_events_rounds(eng, in_place):
    """C3's shape: several rounds per instance (runs mode), 1024 power sets"""
    p = abi.gen_params(seed=52, n_instances=4000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300)
    hb = ol.gen_batch(p)
    hb.instance_set = ad.set_of_instances(ad.Shard(p, 0, p.n_instances), 1024)
    power = ol.gen_power(52, 1024, 150, abi.POWER_UNIFORM, 1, 1000)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4), hb, power,
           abi.new_states(4000, 1, abi.STEP_PREVOTE), in_place=in_place)


def test_tally_events_dedup_skip(eng):
    """C4's shape: the per-instance route, records counted by the count pass"""
    p = abi.gen_params(seed=53, n_instances=2000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                       dup_permille=100, equiv_permille=100, higher_permille=50)
    hb = ol.gen_batch(p)
    hb.instance_set = (np.arange(2000) % 64).astype(np.uint32)
    power = ol.gen_power(53, 64, 150, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP | abi.FLAG_DISTINCT_VALUES, 5)
    ev = _check(eng, cfg, hb, power, abi.new_states(2000, 1, abi.STEP_PREVOTE))
    assert (ev["kind"] == abi.EV_ROUND_SKIP).any()


@pytest.mark.parametrize("route", [abi.ROUTE_INSTANCE, abi.ROUTE_SPLIT, abi.ROUTE_WIDE])
def test_tally_events_forced_routes(eng, route):
    """the record counts by route: tally_fast counts them itself on the per-instance
    routes (INSTANCE / SPLIT, here with REFERENCE and with DEDUP + RoundSkip), the
    wide kernel's route takes the count pass; same records"""
    p = abi.gen_params(seed=65, n_instances=1200, n_vals=80, rounds_min=1, rounds_max=3, nil_permille=300,
                       dup_permille=80, equiv_permille=80, higher_permille=40)
    hb = ol.gen_batch(p)
    power = ol.gen_power(65, 1, 80, abi.POWER_UNIFORM, 1, 5000)
    for mode, flags in [(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE),
                        (abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP)]:
        _check(eng, abi.config(mode, flags | abi.FLAG_ROUTE(route), 4), hb, power,
               abi.new_states(1200, 1, abi.STEP_PREVOTE))


def _ragged(seed, n_inst, max_len, n_vals, rounds, zero_every=7, bad=0.02):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, max_len, n_inst)
    lens[::zero_every] = 0
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    n = int(off[-1])
    inst = np.repeat(np.arange(n_inst, dtype=np.uint32), lens)
    rnd = np.sort(rng.integers(0, rounds, n)).astype(np.uint8)
    typ = rng.integers(0, 2, n).astype(np.uint8)
    val = rng.integers(0, 5, n).astype(np.uint32)
    val[rng.random(n) < 0.3] = abi.NIL
    vdr = rng.integers(0, n_vals, n).astype(np.uint32)
    inst[rng.random(n) < bad] += 1
    rnd[rng.random(n) < bad] = 9
    vdr[rng.random(n) < bad] = n_vals + 5
    return ol.batch_from_lists(inst, rnd, typ, val, vdr, off)


def test_tally_events_walk_list(eng):
    """ragged lengths (offsets not multiples of 4: the walk list), empty instances,
    invalid votes; the list pass counts what the flow kernel handed off"""
    hb = _ragged(54, 3000, 90, 10, 3)
    power = ol.gen_power(54, 1, 10, abi.POWER_UNIFORM, 1, 10)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 3), hb, power,
           abi.new_states(3000, 1, abi.STEP_PREVOTE))
    _check(eng, abi.config(abi.MODE_REFERENCE, 0, 3), hb, power)


def test_tally_events_mixed_batches(eng):
    """some batches one flow stream (lengths multiples of 4), others on the walk list
    (one instance of an odd length), and big powers (instances deferred to the i64 kernel)"""
    rng = np.random.default_rng(55)
    lens = 4 * rng.integers(0, 60, 4096)
    lens[np.arange(0, 4096, 97)] += 3  # one odd instance in about every third batch of 32
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    n = int(off[-1])
    inst = np.repeat(np.arange(4096, dtype=np.uint32), lens)
    rnd = np.zeros(n, dtype=np.uint8)
    typ = rng.integers(0, 2, n).astype(np.uint8)
    val = rng.integers(0, 3, n).astype(np.uint32)
    val[rng.random(n) < 0.25] = abi.NIL
    vdr = rng.integers(0, 64, n).astype(np.uint32)
    set_of = (np.arange(4096) % 3).astype(np.uint32)
    hb = ol.batch_from_lists(inst, rnd, typ, val, vdr, off, instance_set=set_of)
    power = np.stack([ol.gen_power(55, 1, 64, abi.POWER_UNIFORM, 1, 1000)[0],
                      ol.gen_power(56, 1, 64, abi.POWER_UNIFORM, 1, 100_000)[0],   # maxpow > 4096: walk list
                      ol.gen_power(57, 1, 64, abi.POWER_UNIFORM, 1 << 40, 1 << 41)[0]])  # i64 domain
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1), hb, power,
           abi.new_states(4096, 1, abi.STEP_PREVOTE))


@pytest.mark.parametrize("nil", [300, 600])
def test_tally_records_revisited_rounds(eng, nil):
    """flow with rounds revisited inside a chunk (5 % next-round votes, 300-vote rounds
    so every offset stays a multiple of 4): the per-round passes, and nil PolkaValue /
    PrecommitValue votes whose executor's value slot comes from before the chunk
    (the fused records' label walk back, round_votes.rs:50-54)"""
    p = abi.gen_params(seed=62, n_instances=3000, n_vals=120, rounds_min=1, rounds_max=4, nil_permille=nil,
                       dup_permille=100, equiv_permille=100, higher_permille=50)
    hb = ol.gen_batch(p)
    assert (hb.offsets % 4 == 0).all()
    power = ol.gen_power(62, 7, 120, abi.POWER_UNIFORM, 1, 1000)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 5), hb, power,
           abi.new_states(3000, 1, abi.STEP_PREVOTE))
    _check(eng, abi.config(abi.MODE_REFERENCE, 0, 5), hb, power)


@pytest.mark.parametrize("rounds,extra", [(1, {}), (4, {}), (5, dict(higher_permille=50, dup_permille=60))])
def test_tally_records_unaligned(eng, rounds, extra):
    """Round 6: ragged instance lengths (5-12 % abstention: offsets at every residue) on
    the flow kernel's unaligned-stream variant -- counts and records written by it, the
    value of a nil PolkaValue / PrecommitValue from the lane, the segment's earlier lanes,
    or the executor's slot carried in LDS (round_votes.rs:50-54); with next-round votes
    (rounds revisited inside a chunk) the executors one at a time"""
    p = abi.gen_params(seed=66 + rounds, n_instances=3000, n_vals=101, rounds_min=1, rounds_max=min(rounds, 4),
                       nil_permille=450, absent_permille=60 if rounds > 1 else 120, **extra)
    hb = ol.gen_batch(p)
    assert (hb.offsets % 4 != 0).mean() > 0.5
    power = ol.gen_power(66, 5, 101, abi.POWER_UNIFORM, 1, 1000)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, rounds), hb, power,
           abi.new_states(3000, 1, abi.STEP_PREVOTE), in_place=False)
    _check(eng, abi.config(abi.MODE_REFERENCE, 0, rounds), hb, power)


def _shifted(eng, t, shift):
    """a copy of the u8 column t placed `shift` bytes past a 16-B boundary"""
    n = t.numel()
    buf = torch.zeros(n + 16, dtype=torch.uint8, device=eng.device)
    buf[shift:shift + n] = t
    return buf[shift:shift + n]


@pytest.mark.parametrize("shift", [4, 8])
def test_tally_records_unaligned_columns(eng, shift):
    """DEDUP + RoundSkip with the round / type columns off a 16-B boundary: the
    segmented records come from the lane-per-instance walk (seg_walk) instead of the
    stream emit, same records"""
    p = abi.gen_params(seed=63, n_instances=1500, n_vals=90, rounds_min=1, rounds_max=3, nil_permille=300,
                       dup_permille=100, equiv_permille=100, higher_permille=50)
    hb = ol.gen_batch(p)
    power = ol.gen_power(63, 1, 90, abi.POWER_UNIFORM, 1, 5000)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP, 4)
    st = abi.new_states(1500, 1, abi.STEP_PREVOTE)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    db.round, db.type = _shifted(eng, db.round, shift), _shifted(eng, db.type, shift)
    o_codes, o_states, _, o_offs, o_ev = ol.events(cfg, hb, power, None, st, threads=THREADS)
    _check_records(eng, cfg, hb, db, st, True, o_codes, o_states, o_offs, o_ev)


def test_tally_records_many_keys(eng):
    """40 rounds (80 keys: more than the stream emit's LDS value slots hold) on the
    DEDUP route: the segments from seg_walk"""
    p = abi.gen_params(seed=64, n_instances=400, n_vals=20, rounds_min=1, rounds_max=40, nil_permille=300,
                       dup_permille=50, equiv_permille=50)
    hb = ol.gen_batch(p)
    power = ol.gen_power(64, 1, 20, abi.POWER_UNIFORM, 1, 100)
    cfg = abi.config(abi.MODE_DEDUP, 0, 40)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    o_codes, o_states, _, o_offs, o_ev = ol.events(cfg, hb, power, None, None, threads=THREADS)
    assert len(o_ev) > 0
    _check_records(eng, cfg, hb, db, None, True, o_codes, o_states, o_offs, o_ev)


def test_tally_events_fifteen_rounds(eng):
    """max_rounds 15 with the State machine: the counts do not fit the flow kernel's
    LDS, so the count pass runs (same records)"""
    p = abi.gen_params(seed=58, n_instances=800, n_vals=30, rounds_min=1, rounds_max=15, nil_permille=300)
    hb = ol.gen_batch(p)
    power = ol.gen_power(58, 1, 30, abi.POWER_UNIFORM, 1, 100)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 15), hb, power,
           abi.new_states(800, 1, abi.STEP_PREVOTE))


def test_tally_events_weights_and_tiny(eng):
    """caller weights (the i64 route), one instance, an empty batch"""
    p = abi.gen_params(seed=59, n_instances=300, n_vals=50, rounds_min=1, rounds_max=2, nil_permille=200)
    hb = ol.gen_batch(p)
    hb.weight = np.random.default_rng(59).integers(-5, 1 << 33, hb.n_votes).astype(np.int64)
    power = ol.gen_power(59, 1, 50, abi.POWER_UNIFORM, 1, 100)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 2), hb, power,
           abi.new_states(300, 1, abi.STEP_PREVOTE))
    p1 = abi.gen_params(seed=60, n_instances=1, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1), ol.gen_batch(p1),
           ol.gen_power(60, 1, 100, abi.POWER_UNIFORM, 1, 1000), abi.new_states(1, 1, abi.STEP_PREVOTE))
    empty = ol.batch_from_lists([], [], [], [], [], np.zeros(5, dtype=np.uint64))
    _check(eng, abi.config(abi.MODE_REFERENCE, 0, 1), empty, ol.gen_power(61, 1, 4, abi.POWER_UNIFORM, 1, 10))


@pytest.mark.slow
def test_tally_events_full_c2(eng):
    """the bench's c2 batch: 1M instances, 2e8 votes, 6.8e7 records"""
    p = abi.gen_params(seed=0xC2, n_instances=1_000_000, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200)
    hb = ol.gen_batch(p)
    power = ol.gen_power(0xA6E5, 1, 100, abi.POWER_UNIFORM, 1, 1000)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1), hb, power,
           abi.new_states(1_000_000, 1, abi.STEP_PREVOTE), in_place=False)


@pytest.mark.slow
def test_tally_events_full_c3_shard(eng):
    """a C3 shard: 125k instances x 150 validators x 1..4 rounds, 1024 power sets (the
    flow kernel's runs mode counts the records of several rounds per chunk)"""
    p = abi.gen_params(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300)
    hb = ol.gen_batch(p)
    hb.instance_set = ad.set_of_instances(ad.Shard(p, 0, p.n_instances), 1024)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_UNIFORM, 1, 1000)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4), hb, power,
           abi.new_states(125_000, 1, abi.STEP_PREVOTE))


@pytest.mark.slow
def test_tally_events_full_c4_shard(eng):
    """a C4 shard: DEDUP + RoundSkip + DISTINCT_VALUES, Zipf power (the count pass route)"""
    p = abi.gen_params(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                       dup_permille=100, equiv_permille=100, higher_permille=50)
    hb = ol.gen_batch(p)
    hb.instance_set = ad.set_of_instances(ad.Shard(p, 0, p.n_instances), 1024)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP | abi.FLAG_DISTINCT_VALUES, 5)
    ev = _check(eng, cfg, hb, power, abi.new_states(125_000, 1, abi.STEP_PREVOTE))
    assert (ev["kind"] == abi.EV_ROUND_SKIP).any()


@pytest.mark.slow
def test_tally_events_full_c3r_shard(eng):
    """round 6: the bench's c3r batch -- a C3 shard with 5 % abstention (offsets at every
    residue): the counts and records from the unaligned-stream loop, full size"""
    p = abi.gen_params(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                       absent_permille=50)
    hb = ol.gen_batch(p)
    assert (hb.offsets % 4 != 0).mean() > 0.5
    hb.instance_set = ad.set_of_instances(ad.Shard(p, 0, p.n_instances), 1024)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_UNIFORM, 1, 1000)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4), hb, power,
           abi.new_states(125_000, 1, abi.STEP_PREVOTE), in_place=False)


@pytest.mark.parametrize("rounds", [1, 4])
def test_tally_records_mixed_alignment(eng, rounds):
    """Round 6: aligned and unaligned flow batches in one call (the kernel with both loops):
    the record counts, the dense records and the segmented records against the checker"""
    parts = []
    for k, absent in enumerate((0, 60, 0)):
        p = abi.gen_params(seed=150 + 3 * rounds + k, n_instances=1500, n_vals=24, rounds_min=1,
                           rounds_max=rounds, nil_permille=450, absent_permille=absent)
        parts.append(ol.gen_batch(p))
    hb = ol.concat_batches(*parts)
    power = ol.gen_power(150, 3, 24, abi.POWER_UNIFORM, 1, 100)
    _check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, rounds), hb, power,
           abi.new_states(hb.n_instances, 1, abi.STEP_PREVOTE), in_place=False)


@pytest.mark.parametrize("name", ["c2w_ragged", "c3w_ragged"])
def test_tally_records_u64_ragged(eng, name):
    """Round 6: i64 stakes (the u64 domain) with abstention (unaligned instance offsets):
    counts, dense and segmented records"""
    from test_gpu_parity import _make
    p, hb, power, cfg = _make(name)
    assert (hb.offsets % 4 != 0).any()
    _check(eng, cfg, hb, power, abi.new_states(p.n_instances, 1, abi.STEP_PREVOTE), in_place=False)
