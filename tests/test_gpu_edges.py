"""Edge-triggered summary on the GPU (agnes_edge_offsets + agnes_edges through the C
ABI) against the checker's orc_edges — bit-exact offsets and records."""
import numpy as np
import pytest
import torch

import oracle_lib as ol
from agnes_amd import abi
from agnes_amd.engine import DeviceBatch, states_to_device
from test_gpu_parity import CONFIGS, _make, _start_states, eng  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


def _gpu_edges(eng, cfg, hb, power, states=None, shift=0):
    """Tally on the GPU, then summarise; shift > 0 hands the summary copies of the u8
    columns (codes, round, type) placed `shift` bytes past a 16-B boundary (4-B
    windows instead of 16-B)."""
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    n = max(hb.n_votes, 1)
    codes = torch.zeros(n, dtype=torch.uint8, device=eng.device)
    dst = None if states is None else states_to_device(states, eng.device)
    eng.tally(cfg, db, codes, dst)
    if shift:
        def shifted(t):
            buf = torch.zeros(n + 16, dtype=torch.uint8, device=eng.device)
            buf[shift:shift + n] = t[:n]
            return buf[shift:shift + n]
        db.round, db.type = shifted(db.round), shifted(db.type)
        codes = shifted(codes)
    offs, recs = eng.edges(cfg, db, codes)
    torch.cuda.synchronize()
    g_codes = codes[:hb.n_votes].cpu().numpy()
    return g_codes, offs.cpu().numpy().view(np.uint64), recs.cpu().numpy().reshape(-1).view(abi.EDGE_DTYPE)


def _check(cfg, hb, g_codes, g_offs, g_recs):
    o_offs, o_recs = ol.edges(cfg, hb, g_codes)
    assert np.array_equal(g_offs, o_offs)
    if g_recs.tobytes() != o_recs.tobytes():
        k = int(np.nonzero(g_recs != o_recs)[0][0])
        raise AssertionError(f"edge {k}: gpu {g_recs[k]} oracle {o_recs[k]}")


@pytest.mark.parametrize("name", ["c2_small", "c4_small", "c4_ref_skip", "phased_dedup",
                                  "sorted_tiny_sets", "many_rounds", "wide_negative_powers"])
def test_edges_generated(eng, name):
    if name not in CONFIGS:
        pytest.skip(f"{name} not in CONFIGS")
    p, hb, power, cfg = _make(name)
    states = _start_states(p.n_instances) if cfg.flags & abi.FLAG_STATE_MACHINE else None
    g_codes, g_offs, g_recs = _gpu_edges(eng, cfg, hb, power, states)
    o_codes, _, _ = ol.tally(cfg, hb, power, None, states, threads=8)
    assert np.array_equal(g_codes, o_codes)
    _check(cfg, hb, g_codes, g_offs, g_recs)
    assert 0 < len(g_recs) < hb.n_votes


@pytest.mark.parametrize("shift", [4, 8, 12])
def test_edges_unaligned_columns(eng, shift):
    p, hb, power, cfg = _make("c4_small")
    states = _start_states(p.n_instances) if cfg.flags & abi.FLAG_STATE_MACHINE else None
    g_codes, g_offs, g_recs = _gpu_edges(eng, cfg, hb, power, states, shift)
    _check(cfg, hb, g_codes, g_offs, g_recs)


def test_edges_ragged_empty_and_invalid(eng):
    rng = np.random.default_rng(11)
    lengths = [0, 1, 2, 15, 16, 17, 0, 31, 33, 200, 0, 5]
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.uint64)
    n = int(off[-1])
    inst = np.repeat(np.arange(len(lengths)), lengths)
    hb = ol.batch_from_lists(inst, rng.integers(0, 3, n), rng.integers(0, 2, n),
                             np.where(rng.random(n) < 0.3, abi.NIL, 1), rng.integers(0, 8, n), off)
    hb.type[3] = 2           # invalid type
    hb.round[20] = 7         # >= max_rounds
    hb.instance[40] += 1     # wrong segment
    power = ol.gen_power(3, 1, 8, abi.POWER_UNIFORM, 1, 9)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 3)
    st = abi.new_states(len(lengths), 1, abi.STEP_PREVOTE, 0)
    g_codes, g_offs, g_recs = _gpu_edges(eng, cfg, hb, power, st)
    _check(cfg, hb, g_codes, g_offs, g_recs)
    assert g_offs[1] == 0 and g_offs[7] == g_offs[6]


def test_edges_many_instances_scan(eng):
    """1.1M tiny instances: > 1024 scan blocks, so the block totals take more than one
    chunk of the single-block pass (multi-level offsets)."""
    p = abi.gen_params(seed=0x5CA, n_instances=1_100_000, n_vals=2, rounds_min=1, rounds_max=1,
                       nil_permille=300)
    hb = ol.gen_batch(p)
    power = ol.gen_power(0x5CA, 1, 2, abi.POWER_EQUAL, 1, 1)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)
    st = abi.new_states(p.n_instances, 1, abi.STEP_PREVOTE, 0)
    g_codes, g_offs, g_recs = _gpu_edges(eng, cfg, hb, power, st)
    _check(cfg, hb, g_codes, g_offs, g_recs)
    assert g_offs[-1] > 1024


@pytest.mark.slow
def test_edges_full_c2_roundtrip(eng):
    """C2x100 (1M instances, 2e8 votes): offsets monotone, every record's vote inside
    its instance, and per-instance edge counts equal the checker's on a sample."""
    p = abi.gen_params(seed=0xA6E5, n_instances=1_000_000, n_vals=100, rounds_min=1, rounds_max=1,
                       nil_permille=200)
    eng.upload_power(ol.gen_power(0xA6E5, 1, 100, abi.POWER_UNIFORM, 1, 1000))
    db = eng.gen_batch(p)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)
    codes = torch.zeros(db.n_votes, dtype=torch.uint8, device=eng.device)
    dst = states_to_device(abi.new_states(p.n_instances, 1, abi.STEP_PREVOTE, 0), eng.device)
    eng.tally(cfg, db, codes, dst)
    offs, recs = eng.edges(cfg, db, codes)
    torch.cuda.synchronize()
    o = offs.cpu().numpy().view(np.uint64)
    assert (np.diff(o.astype(np.int64)) >= 0).all() and o[0] == 0
    r = recs.cpu().numpy().reshape(-1).view(abi.EDGE_DTYPE)
    inst = r["instance"].astype(np.int64)
    assert np.array_equal(np.repeat(np.arange(p.n_instances), np.diff(o.astype(np.int64))), inst)
    vo = db.offsets.cpu().numpy()
    assert ((r["vote"] >= vo[inst]) & (r["vote"] < vo[inst + 1])).all()
    # the first 2000 instances through the checker
    k = 2000
    sub = ol.gen_batch(abi.gen_params(seed=0xA6E5, n_instances=k, n_vals=100, rounds_min=1,
                                      rounds_max=1, nil_permille=200))
    s_offs, s_recs = ol.edges(cfg, sub, codes[:sub.n_votes].cpu().numpy())
    assert np.array_equal(s_offs, o[:k + 1])
    assert s_recs.tobytes() == r[:int(o[k])].tobytes()


@pytest.mark.parametrize("R", [1, 4, 200])
def test_edges_arbitrary_code_bytes(eng, R):
    """Every code byte (events, RoundSkip, messages, INVALID / REJECTED), rounds up
    to R (some beyond) and types 0..2 straight into agnes_edges, both window paths
    (R = 200: executors beyond the first LDS words)."""
    rng = np.random.default_rng(R)
    lengths = rng.integers(0, 300, 20000)
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.uint64)
    n = int(off[-1])
    inst = np.repeat(np.arange(len(lengths)), lengths)
    rnd = rng.integers(0, R + 1, n)
    hb = ol.batch_from_lists(inst, rnd, rng.integers(0, 3, n), np.zeros(n), np.zeros(n), off)
    codes = rng.integers(0, 256, n).astype(np.uint8)
    codes[rng.random(n) < 0.7] &= 0x0F  # mostly message-free, so levels repeat
    cfg = abi.config(abi.MODE_REFERENCE, 0, R)
    db = DeviceBatch.from_host(hb, eng.device)
    for shift in (0, 4):
        dc = torch.zeros(n + 16, dtype=torch.uint8, device=eng.device)
        dc[shift:shift + n] = torch.from_numpy(codes).to(eng.device)
        d = db
        if shift:
            def shifted(t):
                buf = torch.zeros(n + 16, dtype=torch.uint8, device=eng.device)
                buf[shift:shift + n] = t[:n]
                return buf[shift:shift + n]
            d = DeviceBatch(db.instance, shifted(db.round), shifted(db.type), db.value, db.validator,
                            db.offsets, n_votes=n)
        offs, recs = eng.edges(cfg, d, dc[shift:shift + n])
        torch.cuda.synchronize()
        _check(cfg, hb, codes, offs.cpu().numpy().view(np.uint64),
               recs.cpu().numpy().reshape(-1).view(abi.EDGE_DTYPE))


@pytest.mark.parametrize("R", [1, 4])
def test_edges_offsets_going_back(eng, R):
    """Offsets that go back inside a batch (an instance whose end lies before its start,
    ranges that overlap): the stream kernel walks such a batch instance by instance and
    equals the checker; runs in order, runs revisited (shuffled rounds) and unaligned
    (1-B shifted) columns alike."""
    rng = np.random.default_rng(100 + R)
    lengths = rng.integers(0, 300, 3000)
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    n = int(off[-1])
    inst = np.repeat(np.arange(len(lengths)), lengths)
    rnd = np.sort(rng.integers(0, R + 1, n)) if R == 1 else rng.integers(0, R + 1, n)
    # every 37th instance's start moved past its end, every 41st's start back into the one before
    bad = off.copy()
    bad[37:-1:37] = np.minimum(bad[37:-1:37] + 400, n)
    bad[41:-1:41] = np.maximum(bad[41:-1:41] - 100, 0)
    hb = ol.batch_from_lists(inst, rnd, rng.integers(0, 3, n), np.zeros(n), np.zeros(n), bad.astype(np.uint64))
    codes = rng.integers(0, 256, n).astype(np.uint8)
    codes[rng.random(n) < 0.7] &= 0x0F
    cfg = abi.config(abi.MODE_REFERENCE, 0, R)
    db = DeviceBatch.from_host(hb, eng.device)
    dc = torch.from_numpy(codes).to(eng.device)
    offs, recs = eng.edges(cfg, db, dc)
    torch.cuda.synchronize()
    _check(cfg, hb, codes, offs.cpu().numpy().view(np.uint64), recs.cpu().numpy().reshape(-1).view(abi.EDGE_DTYPE))


# ------------------------------------------------ round 5: agnes_tally_edges (fused)

def _tally_edges_check(eng, cfg, hb, power, states=None, shift=0):
    """agnes_tally_edges: the tally and its edge summary in one call, segmented by
    instance (the flow kernel finds and writes them on the C2 / C3 route), against the
    checker's codes, States and orc_edges over them; then agnes_edges_compact's dense
    layout against orc_edges' offsets and records, byte for byte."""
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    n = max(hb.n_votes, 1)
    if shift:  # round / type off a 16-B boundary: the windowed walks' 4-B path
        def shifted(t):
            buf = torch.zeros(t.numel() + 16, dtype=torch.uint8, device=eng.device)
            buf[shift:shift + t.numel()] = t
            return buf[shift:shift + t.numel()]
        db.round, db.type = shifted(db.round), shifted(db.type)
    codes = torch.full((n,), 0xEE, dtype=torch.uint8, device=eng.device)
    dst = None if states is None else states_to_device(states, eng.device)
    seg = torch.full((n, 16), 0xCD, dtype=torch.uint8, device=eng.device)
    counts, seg = eng.tally_edges(cfg, db, codes, dst, dst, out=seg)
    torch.cuda.synchronize()
    o_codes, o_states, _ = ol.tally(cfg, hb, power, None, states, threads=8)
    g_codes = codes[:hb.n_votes].cpu().numpy()
    assert np.array_equal(g_codes, o_codes), "codes differ"
    if states is not None:
        from agnes_amd.engine import states_to_host
        assert states_to_host(dst).tobytes() == o_states.tobytes(), "States differ"
    o_offs, o_recs = ol.edges(cfg, hb, o_codes)
    g_cnt = counts[:hb.n_instances].cpu().numpy().view(np.uint64)
    o_cnt = np.diff(o_offs.astype(np.int64)).astype(np.uint64)
    assert np.array_equal(g_cnt, o_cnt), f"edge counts differ (first at {np.nonzero(g_cnt != o_cnt)[0][:1]})"
    g_seg = seg.cpu().numpy().reshape(-1).view(abi.EDGE_DTYPE)
    off = hb.offsets.astype(np.int64)
    idx = np.concatenate([np.arange(off[i], off[i] + int(o_cnt[i])) for i in range(hb.n_instances)]
                         + [np.zeros(0, np.int64)]).astype(np.int64)
    got = g_seg[idx]
    if got.tobytes() != o_recs.tobytes():
        k = int(np.nonzero(got != o_recs)[0][0])
        raise AssertionError(f"segmented edge {k} of {len(o_recs)}: gpu {got[k]} checker {o_recs[k]}")
    d_offs, dense = eng.edges_compact(cfg, db, counts, seg)
    torch.cuda.synchronize()
    assert np.array_equal(d_offs.cpu().numpy().view(np.uint64), o_offs)
    assert dense[:len(o_recs)].cpu().numpy().tobytes() == o_recs.tobytes()
    return o_recs


@pytest.mark.parametrize("name", ["c2_small", "c2_sm", "c3_small", "c4_small", "c4_ref_skip", "sorted_tiny_sets",
                                  "many_rounds", "c2w_small", "c3w_small", "c3w_plain", "w64_deferred",
                                  "c2w_ragged", "c3w_ragged"])
def test_tally_edges_generated(eng, name):
    """(the u64-domain configs -- one round, runs mode, the per-round passes, and
    w64_deferred's instances for the i64 LIST kernel -- take the edge walk after the tally)"""
    p, hb, power, cfg = _make(name)
    states = _start_states(p.n_instances) if cfg.flags & abi.FLAG_STATE_MACHINE else None
    recs = _tally_edges_check(eng, cfg, hb, power, states)
    assert len(recs) > 0


@pytest.mark.parametrize("shift", [4, 8])
def test_tally_edges_unaligned_columns(eng, shift):
    """C4's route with the round / type columns off a 16-B boundary: the segmented
    edges from the 4-B-window walk"""
    p, hb, power, cfg = _make("c4_small")
    states = _start_states(p.n_instances) if cfg.flags & abi.FLAG_STATE_MACHINE else None
    assert len(_tally_edges_check(eng, cfg, hb, power, states, shift)) > 0


@pytest.mark.parametrize("nil", [300, 700])
def test_tally_edges_revisited_rounds(eng, nil):
    """flow chunks that revisit rounds (5 % next-round votes, 300-vote rounds: offsets
    stay multiples of 4): the per-key path of the fused edges"""
    p = abi.gen_params(seed=63, n_instances=3000, n_vals=120, rounds_min=1, rounds_max=4, nil_permille=nil,
                       dup_permille=100, equiv_permille=100, higher_permille=50)
    hb = ol.gen_batch(p)
    assert (hb.offsets % 4 == 0).all()
    power = ol.gen_power(63, 7, 120, abi.POWER_UNIFORM, 1, 1000)
    _tally_edges_check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 5), hb, power,
                       _start_states(3000))
    _tally_edges_check(eng, abi.config(abi.MODE_REFERENCE, 0, 5), hb, power)


@pytest.mark.parametrize("name", ["c2r_small", "c3r_small", "c3r_plain", "c4r_ref"])
def test_tally_edges_unaligned_streams(eng, name):
    """Round 6: ragged instance lengths (abstention: offsets at every residue) on the flow
    kernel's unaligned-stream variant -- its units split at any vote; with next-round
    votes (c4r_ref) the per-key path"""
    p, hb, power, cfg = _make(name)
    assert (hb.offsets % 4 != 0).mean() > 0.5
    states = _start_states(p.n_instances) if cfg.flags & abi.FLAG_STATE_MACHINE else None
    assert len(_tally_edges_check(eng, cfg, hb, power, states)) > 0


def test_tally_edges_walk_list_and_empty(eng):
    """ragged lengths (the flow kernel's walk list: the edge walk over the list), empty
    instances, invalid votes, one instance, an empty batch"""
    rng = np.random.default_rng(64)
    lens = rng.integers(0, 90, 3000)
    lens[::7] = 0
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    n = int(off[-1])
    inst = np.repeat(np.arange(3000, dtype=np.uint32), lens)
    rnd = np.sort(rng.integers(0, 3, n)).astype(np.uint8)
    val = rng.integers(0, 5, n).astype(np.uint32)
    val[rng.random(n) < 0.3] = abi.NIL
    vdr = rng.integers(0, 10, n).astype(np.uint32)
    inst[rng.random(n) < 0.02] += 1
    hb = ol.batch_from_lists(inst, rnd, rng.integers(0, 2, n).astype(np.uint8), val, vdr, off)
    power = ol.gen_power(64, 1, 10, abi.POWER_UNIFORM, 1, 10)
    _tally_edges_check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 3), hb, power,
                       abi.new_states(3000, 1, abi.STEP_PREVOTE))
    p1 = abi.gen_params(seed=65, n_instances=1, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200)
    _tally_edges_check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1), ol.gen_batch(p1),
                       ol.gen_power(65, 1, 100, abi.POWER_UNIFORM, 1, 1000), abi.new_states(1, 1, abi.STEP_PREVOTE))
    empty = ol.batch_from_lists([], [], [], [], [], np.zeros(5, dtype=np.uint64))
    _tally_edges_check(eng, abi.config(abi.MODE_REFERENCE, 0, 1), empty, ol.gen_power(66, 1, 4, abi.POWER_UNIFORM, 1, 10))


@pytest.mark.parametrize("rounds", [1, 4])
def test_tally_edges_mixed_alignment(eng, rounds):
    """Round 6: aligned and unaligned flow batches in one call (the kernel with both
    loops), the edges each loop writes against orc_edges"""
    parts = []
    for k, absent in enumerate((0, 60, 0)):
        p = abi.gen_params(seed=160 + 3 * rounds + k, n_instances=1500, n_vals=24, rounds_min=1,
                           rounds_max=rounds, nil_permille=300, absent_permille=absent)
        parts.append(ol.gen_batch(p))
    hb = ol.concat_batches(*parts)
    power = ol.gen_power(160, 3, 24, abi.POWER_UNIFORM, 1, 100)
    states = abi.new_states(hb.n_instances, 1, abi.STEP_PREVOTE)
    assert len(_tally_edges_check(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, rounds), hb, power,
                                  states)) > 0


@pytest.mark.slow
@pytest.mark.parametrize("name", ["c3r", "c4"])
def test_tally_edges_full_shard(eng, name):
    """Round 6, full size: the bench's c3r batch (edges from the unaligned-stream loop) and
    the C4 shard (edges from the State machine's pass on the split route)"""
    from agnes_amd import dist as ad
    kw = dict(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300)
    if name == "c3r":
        p = abi.gen_params(absent_permille=50, **kw)
        power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_UNIFORM, 1, 1000)
        cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4)
    else:
        p = abi.gen_params(dup_permille=100, equiv_permille=100, higher_permille=50, **kw)
        power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_ZIPF, 1, 1_000_000)
        cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP, 5)
    hb = ol.gen_batch(p)
    hb.instance_set = ad.set_of_instances(ad.Shard(p, 0, p.n_instances), 1024)
    recs = _tally_edges_check(eng, cfg, hb, power, _start_states(p.n_instances))
    assert len(recs) > p.n_instances
