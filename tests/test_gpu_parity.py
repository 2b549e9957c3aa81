"""Parity of the HIP engine (through the C ABI) against the CPU checker.

Bar: bit-exact per-vote codes, final per-instance states and invalid counts.
Oracle-checked sizes run in seconds; the full-size case adds size-independent
properties (determinism, shard == whole, message/state consistency).
"""
import ctypes as C
import json
import os

import numpy as np
import pytest
import torch

import oracle_lib as ol
from agnes_amd import abi
from agnes_amd.engine import DeviceBatch, Engine, states_to_device, states_to_host
from agnes_amd.lib import load

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF = json.load(open(os.path.join(GOLD, "reference_tests.json")))
REGRESS = json.load(open(os.path.join(GOLD, "regress_small.json")))
EV_BY_NAME = {n: i for i, n in enumerate(abi.EVENT_NAMES)}
# every route the launcher can take (agnes_kernels.hip launch_mode), forced by the
# cfg route field: the engine's choice (the fused sweep for REFERENCE without
# RoundSkip), the per-instance kernel with the State machine fused, the same
# followed by the apply pass, and the i64 kernel for every instance
ROUTES = {
    "auto": abi.FLAG_ROUTE(abi.ROUTE_AUTO),
    "fused": abi.FLAG_ROUTE(abi.ROUTE_INSTANCE),
    "split": abi.FLAG_ROUTE(abi.ROUTE_SPLIT),
    "wide": abi.FLAG_ROUTE(abi.ROUTE_WIDE),
}


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    e = Engine(0)
    yield e
    e.close()


def run_both(eng, cfg, hb, power, totals=None, states=None, threads=8):
    """Tally hb on the GPU and on the checker; return both results."""
    if power is not None:
        eng.upload_power(power, totals)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.zeros(max(hb.n_votes, 1), dtype=torch.uint8, device=eng.device)
    dst = None if states is None else states_to_device(states, eng.device)
    eng.tally(cfg, db, codes, dst)
    torch.cuda.synchronize()
    g_codes = codes[:hb.n_votes].cpu().numpy()
    g_bad = eng.last_error_count()
    g_states = None if dst is None else states_to_host(dst)
    o_codes, o_states, o_bad = ol.tally(cfg, hb, power, totals, states, threads=threads)
    return (g_codes, g_states, g_bad), (o_codes, o_states, o_bad)


def assert_same(g, o):
    gc, gs, gb = g
    oc, os_, ob = o
    if not np.array_equal(gc, oc):
        bad = np.nonzero(gc != oc)[0]
        k = bad[0]
        raise AssertionError(f"{len(bad)} codes differ; first at {k}: gpu {gc[k]:#x} oracle {oc[k]:#x}")
    assert gb == ob
    if os_ is not None:
        assert gs.tobytes() == os_.tobytes()


# --------------------------------------------------- the reference's own tests


def test_add_votes_through_scalar_mirror():
    """round_votes.rs:107-132 through agnes_ve_apply (VoteExecutor::apply):
    thresholds Init, Init, Any, Value  ==  events None, None, PolkaAny, PolkaValue."""
    L = load()
    g = REF["add_votes"]
    ve = L.agnes_ve_new(1, g["total"])
    assert ve
    got = []
    for t, v in g["votes"]:
        vote = abi.Vote(0, abi.NIL if v is None else v, t)
        ev = abi.Event()
        rc = L.agnes_ve_apply(ve, C.byref(vote), g["weight"], C.byref(ev))
        assert rc in (0, 1)
        got.append(None if rc == 0 else abi.EVENT_NAMES[ev.kind])
    L.agnes_ve_free(ve)
    assert got == [None, None, "PolkaAny", "PolkaValue"]


@pytest.mark.parametrize("name", ["c1_value", "c1_nil", "c1_mixed"])
def test_c1_traces_through_scalar_mirror(name):
    L = load()
    g = REF[name]
    ve = L.agnes_ve_new(1, g["total"])
    got = []
    for t, v in g["votes"]:
        ev = abi.Event()
        rc = L.agnes_ve_apply(ve, C.byref(abi.Vote(0, abi.NIL if v is None else v, t)),
                              g["weight"], C.byref(ev))
        got.append(None if rc == 0 else abi.EVENT_NAMES[ev.kind])
        if rc == 1 and ev.kind in (abi.EV_POLKA_VALUE, abi.EV_PRECOMMIT_VALUE):
            assert ev.value == v
    L.agnes_ve_free(ve)
    assert got == g["events"]


def test_happy_case_through_scalar_mirror():
    """state_machine.rs:331-345 through agnes_state_apply."""
    L = load()
    g = REF["happy_case"]
    s = abi.StateRec()
    L.agnes_state_init(g["height"], C.byref(s))
    for ev, want in zip(g["events"], g["messages"]):
        e = abi.Event(ev["round"], ev.get("pol_round", 0), ev.get("value", 0), EV_BY_NAME[ev["kind"]])
        out, m = abi.StateRec(), abi.Message()
        rc = L.agnes_state_apply(C.byref(s), ev["round"], C.byref(e), 0, C.byref(out), C.byref(m))
        assert rc == 1
        assert abi.MSG_NAMES[m.kind] == want["kind"] and m.round == want["round"]
        assert m.value == want["value"]
        s = out
    assert abi.STEP_NAMES[s.step] == "Commit"


def test_scalar_mirror_wrapping_i64():
    """Rust release i64 wrap: 3*w overflows, compare signed (round_votes.rs:32)."""
    L = load()
    big = (1 << 62) + 5
    for total in [4, -7, (1 << 62), -(1 << 63)]:
        ve = L.agnes_ve_new(1, total)
        rv = ol.RoundVotes(1, 0, total)
        for k, (t, v, w) in enumerate([(0, 3, big), (0, abi.NIL, -big), (0, 3, big), (1, 3, 1),
                                       (1, abi.NIL, (1 << 63) - 1), (0, abi.NIL, 2)]):
            ev = abi.Event()
            rc = L.agnes_ve_apply(ve, C.byref(abi.Vote(0, v, t)), w, C.byref(ev))
            oe, _ = rv.ve_apply(t, v, w)
            assert (abi.EV_NONE if rc == 0 else ev.kind) == oe, (total, k)
        L.agnes_ve_free(ve)


def test_c1_batch_with_state_machine(eng):
    """BASELINE config C1: 4 equal-power validators, polka -> decision."""
    g = REF["c1_value"]
    n = len(g["votes"])
    hb = ol.batch_from_lists([0] * n, [0] * n, [t for t, _ in g["votes"]], [v for _, v in g["votes"]],
                             [k % 4 for k in range(n)], [0, n])
    st = ol.state_new(1)
    st, _ = ol.state_apply(st, 0, abi.Event(0, 0, 7, abi.EV_NEW_ROUND_PROPOSER))
    st, _ = ol.state_apply(st, 0, abi.Event(0, -1, 7, abi.EV_PROPOSAL))
    st0 = np.frombuffer(bytes(st), dtype=abi.STATE_DTYPE).copy()
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)
    g_, o_ = run_both(eng, cfg, hb, np.ones((1, 4), np.int64), states=st0)
    assert_same(g_, o_)
    msgs = [int(c) >> 4 for c in g_[0]]
    assert msgs == [0, 0, abi.VMSG_PRECOMMIT_VALUE, 0, 0, 0, abi.VMSG_DECISION, 0]


@pytest.mark.parametrize("case", REGRESS, ids=[c["name"] for c in REGRESS])
def test_regress_fixtures(eng, case):
    from test_oracle_golden import _states_from_json
    hb = ol.batch_from_lists(case["instance"], case["round"], case["type"], case["value"],
                             case["validator"], case["offsets"])
    cfg = abi.config(case["mode"], case["flags"], case["max_rounds"])
    st_in = _states_from_json(case["states_in"]) if "states_in" in case else None
    g, o = run_both(eng, cfg, hb, np.array(case["power"], np.int64),
                    np.array(case["totals"], np.int64), st_in)
    assert g[0].tolist() == case["codes"]
    assert_same(g, o)


# ----------------------------------------------------------- generated configs

CONFIGS = {
    # name: (gen params, power (kind, lo, hi, n_sets), cfg)
    "c2_small": (dict(n_instances=2000, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200),
                 (abi.POWER_UNIFORM, 1, 1000, 1), (abi.MODE_REFERENCE, 0, 1)),
    "c2_sm": (dict(n_instances=2000, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200),
              (abi.POWER_UNIFORM, 1, 1000, 1), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)),
    "c3_small": (dict(n_instances=3000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300),
                 (abi.POWER_UNIFORM, 1, 1000, 1024),
                 (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4)),
    "c4_small": (dict(n_instances=3000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                      dup_permille=100, equiv_permille=100, higher_permille=50),
                 (abi.POWER_ZIPF, 1, 1000000, 1024),
                 (abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 5)),
    "c4_ref_skip": (dict(n_instances=1500, n_vals=150, rounds_min=1, rounds_max=4,
                         nil_permille=300, dup_permille=100, equiv_permille=100,
                         higher_permille=50),
                    (abi.POWER_ZIPF, 1, 1000000, 64),
                    (abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 5)),
    "phased_dedup": (dict(n_instances=1000, n_vals=77, rounds_min=2, rounds_max=3, nil_permille=500,
                          dup_permille=200, order=abi.ORDER_PHASED),
                     (abi.POWER_UNIFORM, 0, 50, 7), (abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE, 3)),
    "sorted_tiny_sets": (dict(n_instances=4000, n_vals=3, rounds_min=1, rounds_max=8,
                              nil_permille=100, order=abi.ORDER_SORTED),
                         (abi.POWER_EQUAL, 1, 1, 1),
                         (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 8)),
    "wide_huge_powers": (dict(n_instances=500, n_vals=40, rounds_min=1, rounds_max=2,
                              nil_permille=400, dup_permille=300),
                         (abi.POWER_UNIFORM, (1 << 61), (1 << 62), 3),
                         (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 2)),
    "wide_negative_powers": (dict(n_instances=500, n_vals=40, rounds_min=1, rounds_max=2,
                                  nil_permille=400),
                             (abi.POWER_UNIFORM, -30, 100, 3),
                             (abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 3)),
    # the u64 domain (agnes_set_info.w64): powers past 2^31, set totals < 2^61 -> tally_fast
    # with u64 sums; w64_deferred's longer instances reach len * maxpow >= 2^61 (LIST kernel)
    "c2w_small": (dict(n_instances=2000, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200),
                  (abi.POWER_UNIFORM, 1 << 28, 1 << 34, 1), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)),
    "w64_dedup_skip": (dict(n_instances=1500, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                            dup_permille=100, equiv_permille=100, higher_permille=50),
                       (abi.POWER_ZIPF, 1 << 30, 1 << 40, 16),
                       (abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 5)),
    # flow<W64> stages the i64 table in LDS when it fits (c2w_small, c2w_plain); 64 sets x
    # 100 validators x 8 B do not fit, so c2w_sets gathers from HBM
    "c2w_sets": (dict(n_instances=3000, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200),
                 (abi.POWER_UNIFORM, 1 << 28, 1 << 34, 64), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)),
    "c2w_plain": (dict(n_instances=2500, n_vals=90, rounds_min=1, rounds_max=1, nil_permille=350),
                  (abi.POWER_ZIPF, 1 << 31, 1 << 36, 3), (abi.MODE_REFERENCE, 0, 1)),
    "w64_deferred": (dict(n_instances=600, n_vals=300, rounds_min=1, rounds_max=2, nil_permille=250),
                     (abi.POWER_UNIFORM, 1 << 50, 1 << 52, 2), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 2)),
    # flow<W64> over several rounds (round 5): runs mode (c3w_small), the per-round passes
    # when an instance revisits a round inside a chunk (w64_revisit: next-round votes), and
    # the plain tally without the State machine
    "c3w_small": (dict(n_instances=3000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300),
                  (abi.POWER_UNIFORM, 1 << 28, 1 << 34, 1024), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4)),
    "c3w_plain": (dict(n_instances=2500, n_vals=120, rounds_min=2, rounds_max=4, nil_permille=350),
                  (abi.POWER_ZIPF, 1 << 31, 1 << 36, 3), (abi.MODE_REFERENCE, 0, 4)),
    "w64_revisit": (dict(n_instances=2000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                         dup_permille=100, equiv_permille=100, higher_permille=50),
                    (abi.POWER_UNIFORM, 1 << 28, 1 << 34, 5), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 5)),
    # round 6: abstention (absent_permille) -- ragged instance lengths, offsets at any
    # residue: the flow kernel's unaligned-stream variant (c2r / c3r shapes)
    "c2r_small": (dict(n_instances=3000, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200,
                       absent_permille=50),
                  (abi.POWER_UNIFORM, 1, 1000, 1), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)),
    "c3r_small": (dict(n_instances=3000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                       absent_permille=50),
                  (abi.POWER_UNIFORM, 1, 1000, 1024), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4)),
    "c3r_plain": (dict(n_instances=2500, n_vals=101, rounds_min=1, rounds_max=4, nil_permille=350,
                       absent_permille=120),
                  (abi.POWER_ZIPF, 1, 4000, 5), (abi.MODE_REFERENCE, 0, 4)),
    "c4r_ref": (dict(n_instances=2000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                     dup_permille=100, equiv_permille=100, higher_permille=50, absent_permille=30),
                (abi.POWER_UNIFORM, 1, 1000, 64), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 5)),
    # the u64 domain with abstention: the u64 flow kernel's unaligned-stream variant walks
    # these batches (an instance of 1..7 votes sends its batch to the walk list)
    "c2w_ragged": (dict(n_instances=2000, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200,
                        absent_permille=60),
                   (abi.POWER_UNIFORM, 1 << 28, 1 << 34, 1), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)),
    "c3w_ragged": (dict(n_instances=2000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                        absent_permille=50),
                   (abi.POWER_UNIFORM, 1 << 28, 1 << 34, 64), (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4)),
    "many_rounds": (dict(n_instances=200, n_vals=20, rounds_min=30, rounds_max=60,
                         nil_permille=300, higher_permille=100),
                    (abi.POWER_UNIFORM, 1, 100, 5),
                    (abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 61)),
}


def _make(name, seed=0xA6E5):
    gp, (kind, lo, hi, n_sets), (mode, flags, R) = CONFIGS[name]
    p = abi.gen_params(seed=seed, **gp)
    hb = ol.gen_batch(p)
    power = ol.gen_power(seed, n_sets, gp["n_vals"], kind, lo, hi)
    return p, hb, power, abi.config(mode, flags, R)


def _start_states(n, rounds=1, seed=1):
    """Instances already past NewRoundProposer + Proposal at round 0 (Prevote step)."""
    st = abi.new_states(n, 1, abi.STEP_PREVOTE, 0)
    rng = np.random.default_rng(seed)
    k = rng.random(n)
    st["step"][k < 0.1] = abi.STEP_NEW_ROUND
    st["step"][(k >= 0.1) & (k < 0.15)] = abi.STEP_PRECOMMIT
    st["round"][k > 0.95] = 1
    return st


@pytest.mark.parametrize("name", list(CONFIGS))
def test_generated_parity(eng, name):
    p, hb, power, cfg = _make(name)
    states = _start_states(p.n_instances) if cfg.flags & abi.FLAG_STATE_MACHINE else None
    g, o = run_both(eng, cfg, hb, power, None, states)
    assert_same(g, o)
    # the stream must actually exercise the path
    ev = g[0] & abi.CODE_EVENT_MASK
    assert (ev != 0).any()


def test_device_generator_equals_host_generator(eng):
    p, hb, _, _ = _make("c4_small")
    db = eng.gen_batch(p)
    torch.cuda.synchronize()
    h = db.to_host()
    for f in ["instance", "round", "type", "value", "validator", "offsets"]:
        assert np.array_equal(h[f], getattr(hb, f)), f


def test_invalid_votes_counted(eng):
    p, hb, power, cfg = _make("c2_small")
    rng = np.random.default_rng(5)
    idx = rng.choice(hb.n_votes, 500, replace=False)
    hb.validator[idx[:200]] = 100 + idx[:200] % 7     # out of range
    hb.round[idx[200:300]] = 9                          # >= max_rounds
    hb.type[idx[300:400]] = 2                           # bad type
    hb.instance[idx[400:]] += 1                         # wrong segment
    g, o = run_both(eng, cfg, hb, power)
    assert_same(g, o)
    assert g[2] == 500


def test_caller_weights_and_instance_sets(eng):
    p, hb, power, cfg = _make("c3_small")
    rng = np.random.default_rng(9)
    hb.instance_set = rng.integers(0, 1024, hb.n_instances, dtype=np.uint32)
    hb.instance_set[:10] = 5000  # unknown set -> invalid
    g, o = run_both(eng, cfg, hb, power, None, _start_states(hb.n_instances))
    assert_same(g, o)
    hb.weight = rng.integers(-(1 << 62), 1 << 62, hb.n_votes, dtype=np.int64)
    hb.instance_set = None
    cfg2 = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4)
    st = _start_states(hb.n_instances)
    g, o = run_both(eng, cfg2, hb, power, None, st)
    assert_same(g, o)


def test_apply_events_batch(eng):
    rng = np.random.default_rng(3)
    n = 3000
    counts = rng.integers(0, 40, n)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    m = int(off[-1])
    ev = np.zeros(m, abi.EVENT_DTYPE)
    ev["kind"] = rng.integers(0, 13, m)
    ev["round"] = rng.integers(-1, 4, m)
    ev["pol_round"] = rng.integers(-2, 4, m)
    ev["value"] = rng.integers(0, 3, m)
    st = abi.new_states(n, 1)
    for flags in (0, abi.FLAG_DISTINCT_VALUES):
        o_st, o_msgs = ol.apply_events(st, off, ev, flags)
        d_st = states_to_device(st, eng.device)
        d_off = torch.from_numpy(off.view(np.int64)).to(eng.device)
        d_ev = torch.from_numpy(ev.view(np.uint8)).to(eng.device)
        d_msg = torch.zeros(m * 24, dtype=torch.uint8, device=eng.device)
        eng.apply_events(d_st, d_off, d_ev, d_msg, flags)
        torch.cuda.synchronize()
        assert states_to_host(d_st).tobytes() == o_st.tobytes()
        assert d_msg.cpu().numpy().tobytes() == o_msgs.tobytes()


def test_determinism_and_sharding(eng):
    """Same input twice -> identical bytes; a shard of instances tallied alone
    equals the same instances inside the whole batch (instances independent)."""
    p, _, power, cfg = _make("c4_small")
    eng.upload_power(power)
    whole = eng.gen_batch(p)
    st = _start_states(p.n_instances)
    outs = []
    for _ in range(2):
        codes = torch.zeros(whole.n_votes, dtype=torch.uint8, device=eng.device)
        dst = states_to_device(st, eng.device)
        eng.tally(cfg, whole, codes, dst)
        outs.append((codes.cpu().numpy(), states_to_host(dst)))
    assert np.array_equal(outs[0][0], outs[1][0])
    assert outs[0][1].tobytes() == outs[1][1].tobytes()
    # shard = instances [1000, 2000) generated with instance_base
    p2 = abi.gen_params(**{f: getattr(p, f) for f, _ in abi.GenParams._fields_ if f != "reserved"})
    p2.n_instances, p2.instance_base = 1000, 1000
    shard = eng.gen_batch(p2)
    codes = torch.zeros(shard.n_votes, dtype=torch.uint8, device=eng.device)
    sh_set = torch.arange(1000, 2000, dtype=torch.int32, device=eng.device) % 1024
    shard.instance_set = sh_set
    dst = states_to_device(st[1000:2000], eng.device)
    eng.tally(cfg, shard, codes, dst)
    torch.cuda.synchronize()
    off = whole.offsets.cpu().numpy()
    assert np.array_equal(codes.cpu().numpy(), outs[0][0][off[1000]:off[2000]])
    assert states_to_host(dst).tobytes() == outs[0][1][1000:2000].tobytes()


def _ragged_batch(seed, n_inst, n_vals, max_rounds, lengths):
    """Instances with the given vote counts (0 allowed), random fields."""
    rng = np.random.default_rng(seed)
    lens = rng.choice(lengths, n_inst)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    n = int(off[-1])
    inst = np.repeat(np.arange(n_inst, dtype=np.uint32), lens)
    rnd = rng.integers(0, max_rounds, n).astype(np.uint8)
    typ = rng.integers(0, 2, n).astype(np.uint8)
    val = np.where(rng.random(n) < 0.3, abi.NIL, rng.integers(0, 3, n)).astype(np.uint32)
    vid = rng.integers(0, n_vals, n).astype(np.uint32)
    return ol.batch_from_lists(inst, rnd, typ, val, vid, off)


@pytest.mark.parametrize("mode,flags", [
    (abi.MODE_REFERENCE, 0),
    (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE),
    (abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP),
    (abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE)])
def test_ragged_tiny_and_empty_instances(eng, mode, flags):
    """Many instance boundaries per 64-vote chunk, zero-length instances,
    instances longer than a chunk: the lane->instance map and the carries."""
    hb = _ragged_batch(21, 20000, 9, 3, [0, 0, 1, 2, 3, 5, 8, 13, 63, 64, 65, 130, 200])
    power = ol.gen_power(21, 13, 9, abi.POWER_UNIFORM, 1, 20)
    cfg = abi.config(mode, flags, 3)
    st = _start_states(hb.n_instances) if flags & abi.FLAG_STATE_MACHINE else None
    g, o = run_both(eng, cfg, hb, power, None, st)
    assert_same(g, o)


@pytest.mark.parametrize("lengths", [[0, 1, 2, 3, 5, 8, 13, 63, 65, 130, 201],  # walk list + unaligned streams
                                     [0, 97, 150, 203, 299, 301, 411]])        # unaligned streams only
def test_ragged_states_out_of_place(eng, lengths):
    """agnes_tally_states with distinct input and output State arrays on ragged
    batches: every instance's State must come from states_in, including the instances
    of batches the flow kernel hands to another kernel (the walk list, the unaligned
    stream variant) -- the output array starts as garbage."""
    hb = _ragged_batch(23, 12000, 9, 3, lengths)
    power = ol.gen_power(23, 13, 9, abi.POWER_UNIFORM, 1, 20)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 3)
    st = _start_states(hb.n_instances)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.zeros(max(hb.n_votes, 1), dtype=torch.uint8, device=eng.device)
    s_in = states_to_device(st, eng.device)
    s_out = torch.full_like(s_in, 0x5A)
    eng.tally_states(cfg, db, codes, s_in, s_out)
    torch.cuda.synchronize()
    o_codes, o_states, _ = ol.tally(cfg, hb, power, None, st, threads=8)
    assert np.array_equal(codes[:hb.n_votes].cpu().numpy(), o_codes)
    g_st = states_to_host(s_out)
    bad = np.nonzero(g_st.view(np.uint8).reshape(-1, 64).any(axis=1) !=
                     o_states.view(np.uint8).reshape(-1, 64).any(axis=1))[0]
    assert g_st.tobytes() == o_states.tobytes(), f"States differ (first mismatched instance near {bad[:3]})"


@pytest.mark.parametrize("mode,flags", [
    (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE),
    (abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP)])
def test_early_quorum_labels(eng, mode, flags):
    """Two equal validators: every second vote crosses a threshold, so nil votes
    carry Value events whose label comes from another lane / tile / instance."""
    hb = _ragged_batch(8, 30000, 2, 2, [1, 2, 3, 4, 5, 7, 9, 17, 33, 80])
    power = np.ones((1, 2), np.int64)
    cfg = abi.config(mode, flags, 2)
    g, o = run_both(eng, cfg, hb, power, None, _start_states(hb.n_instances))
    assert_same(g, o)


@pytest.mark.parametrize("route", ["auto", "fused", "split"])
@pytest.mark.parametrize("flags", [0, abi.FLAG_STATE_MACHINE])
@pytest.mark.parametrize("lengths", [
    [0, 4, 8, 12, 60, 64, 68, 200, 252, 256, 260, 300, 516],   # lane-aligned: stream batches
    [4, 8, 12, 16, 20, 24, 28, 32],                            # many segments per chunk
    [200], [300, 600, 900, 1200]])                             # C2 / C3 shapes
def test_stream_segments(eng, route, flags, lengths):
    """Instance lengths that are multiples of 4 make every batch a vote stream
    whose chunks straddle instances (agnes_sweep.hip): segments, per-segment
    thresholds and carries, per-segment State::apply, several power sets."""
    if route == "split" and not flags:
        pytest.skip("same launch as fused without the State machine")
    hb = _ragged_batch(31 + len(lengths), 6000, 17, 3, lengths)
    power = ol.gen_power(3, 5, 17, abi.POWER_UNIFORM, 1, 50)
    hb.instance_set = (np.arange(hb.n_instances) * 7 % 5).astype(np.uint32)
    cfg = abi.config(abi.MODE_REFERENCE, flags | ROUTES[route], 3)
    st = _start_states(hb.n_instances) if flags & abi.FLAG_STATE_MACHINE else None
    g, o = run_both(eng, cfg, hb, power, None, st)
    assert_same(g, o)
    assert (g[0] & abi.CODE_EVENT_MASK != 0).any()


def test_stream_mixed_domains(eng):
    """Lane-aligned batches with instances outside the stream domain (i64 powers
    for some sets; an instance_set beyond n_sets): those batches run instance by
    instance, the out-of-domain instances on the i64 kernel."""
    hb = _ragged_batch(77, 4000, 11, 2, [0, 8, 40, 96, 200])
    power = ol.gen_power(7, 4, 11, abi.POWER_UNIFORM, 1, 30)
    power[3, :] = (1 << 40)  # set 3 needs i64 sums
    hb.instance_set = (np.arange(hb.n_instances) % 5).astype(np.uint32)  # set 4 does not exist
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 2)
    g, o = run_both(eng, cfg, hb, power, None, _start_states(hb.n_instances))
    assert_same(g, o)


@pytest.mark.parametrize("route", ["auto", "split", "fused"])
@pytest.mark.parametrize("mode,flags", [
    (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE),
    (abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP)])
def test_deferred_instances_and_set_fallback(eng, route, mode, flags):
    """Instances whose sums may reach 2^31 (len * maxpow) deferred by the u32 kernels
    to the i64 LIST kernel, mixed with fast ones, with the State machine; no
    instance_set, so the set of instance i is i % n_sets."""
    hb = _ragged_batch(91, 6000, 13, 3, [8, 40, 200, 1200])
    power = ol.gen_power(91, 3, 13, abi.POWER_UNIFORM, 1 << 20, 1 << 21)
    hb.instance_set = None
    g, o = run_both(eng, abi.config(mode, flags | ROUTES[route], 3), hb, power, None,
                    _start_states(hb.n_instances))
    assert_same(g, o)


def _with_invalid(hb, seed, n_vals, max_rounds, permille=30):
    """hb with a sprinkle of invalid votes: round >= max_rounds, validator >= n_vals,
    type outside {Prevote, Precommit} (round_votes.rs has no such votes; the engine
    counts and skips them)."""
    rng = np.random.default_rng(seed)
    n = hb.n_votes
    k = rng.random(n) < permille / 1000.0
    which = rng.integers(0, 3, n)
    hb.round[k & (which == 0)] = max_rounds
    hb.validator[k & (which == 1)] = n_vals + 3
    hb.type[k & (which == 2)] = 5
    return hb


def test_invalid_counts_across_routes_and_calls(eng):
    """The queued routes publish the invalid count from the LIST kernel's last wave
    and leave the counters zeroed for the next call (no memset nodes); the other
    routes reset on the host.  One ctx, a sequence mixing them, every count and code
    against the checker: a stale or unreset counter shows as a wrong count."""
    hb = _with_invalid(_ragged_batch(61, 5000, 9, 3, [0, 4, 8, 40, 200]), 61, 9, 3)
    hbd = _with_invalid(_ragged_batch(62, 3000, 13, 3, [8, 40, 200, 1200]), 62, 13, 3)
    hbd.instance_set = None
    p_small = ol.gen_power(61, 2, 9, abi.POWER_UNIFORM, 1, 30)
    p_big = ol.gen_power(62, 3, 13, abi.POWER_UNIFORM, 1 << 20, 1 << 21)
    seq = [("auto", hb, p_small, abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE),
           ("auto", hb, p_small, abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE),
           ("wide", hb, p_small, abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE),
           ("auto", hbd, p_big, abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE),
           ("split", hbd, p_big, abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP),
           ("auto", hb, p_small, abi.MODE_REFERENCE, 0),
           ("wide", hbd, p_big, abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE),
           ("auto", hb, p_small, abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP),
           ("auto", hb, p_small, abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE)]
    for route, b, pw, mode, flags in seq:
        g, o = run_both(eng, abi.config(mode, flags | ROUTES[route], 3), b, pw, None, _start_states(b.n_instances))
        assert o[2] > 0
        assert_same(g, o)


def test_epoch_table_recycling(eng):
    """DEDUP/RoundSkip tables tag entries with per-instance epochs; with few
    epoch bits (AGNES_FLAG_EPOCH_BITS(30)) the tables are cleared every 3 instances."""
    hb = _ragged_batch(5, 6000, 11, 2, [0, 1, 4, 9, 40, 70, 150])
    power = ol.gen_power(5, 4, 11, abi.POWER_UNIFORM, 1, 9)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE | abi.FLAG_EPOCH_BITS(30), 2)
    g, o = run_both(eng, cfg, hb, power, None, _start_states(hb.n_instances))
    assert_same(g, o)
    assert (g[0] & 7 == abi.CODE_REJECTED).any()


@pytest.mark.slow
def test_full_c2_height_parity(eng):
    """BASELINE C2 at full size: 10k instances x 100 validators, one height."""
    p = abi.gen_params(seed=0xA6E5, n_instances=10000, n_vals=100, nil_permille=200)
    hb = ol.gen_batch(p)
    power = ol.gen_power(0xA6E5, 1, 100, abi.POWER_UNIFORM, 1, 1000)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1)
    g, o = run_both(eng, cfg, hb, power, None, _start_states(10000), threads=16)
    assert_same(g, o)


@pytest.mark.slow
def test_c3_shard_parity(eng):
    """BASELINE C3 per-GPU shard: 125k instances (1M / 8) x 150 validators x 1..4 rounds."""
    p = abi.gen_params(seed=0xA6E5, n_instances=125000, n_vals=150, rounds_min=1, rounds_max=4,
                       nil_permille=300)
    hb = ol.gen_batch(p)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_UNIFORM, 1, 1000)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4)
    g, o = run_both(eng, cfg, hb, power, None, _start_states(125000), threads=16)
    assert_same(g, o)


@pytest.mark.parametrize("route", list(ROUTES))
@pytest.mark.parametrize("name", ["c2_sm", "c3_small", "c4_small", "c2w_small", "w64_dedup_skip", "c3w_small",
                                  "w64_revisit", "c2r_small", "c3r_small", "c4r_ref", "c3w_ragged"])
def test_routes_generated(eng, route, name):
    p, hb, power, cfg = _make(name)
    cfg = abi.config(cfg.mode, cfg.flags | ROUTES[route], cfg.max_rounds)
    g, o = run_both(eng, cfg, hb, power, None, _start_states(p.n_instances))
    assert_same(g, o)


@pytest.mark.parametrize("route", list(ROUTES))
@pytest.mark.parametrize("mode,flags", [
    (abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE),
    (abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP)])
def test_routes_ragged_and_labels(eng, route, mode, flags):
    """Ragged instances (many per chunk, empty ones) and early quorums whose nil
    votes carry labels from earlier lanes / chunks."""
    flags |= ROUTES[route]
    hb = _ragged_batch(21, 20000, 9, 3, [0, 0, 1, 2, 3, 5, 8, 13, 63, 64, 65, 130, 200])
    power = ol.gen_power(21, 13, 9, abi.POWER_UNIFORM, 1, 20)
    g, o = run_both(eng, abi.config(mode, flags, 3), hb, power, None, _start_states(hb.n_instances))
    assert_same(g, o)
    hb = _ragged_batch(8, 30000, 2, 2, [1, 2, 3, 4, 5, 7, 9, 17, 33, 80, 200, 400])
    power = np.ones((1, 2), np.int64)
    g, o = run_both(eng, abi.config(mode, flags, 2), hb, power, None, _start_states(hb.n_instances))
    assert_same(g, o)


@pytest.mark.parametrize("route", list(ROUTES))
def test_routes_valid_from_input(eng, route):
    """States entering in Precommit with `valid` already at their round
    (set_valid_value, state_machine.rs:202): a nil vote that reaches the value
    quorum first must set valid to its bucket's last value (round_votes.rs:50-54)."""
    rng = np.random.default_rng(44)
    hb = _ragged_batch(44, 8000, 3, 2, [4, 8, 12, 40, 200])
    power = np.ones((1, 3), np.int64)
    st = _start_states(hb.n_instances)
    k = rng.random(hb.n_instances)
    sel = k < 0.6
    st["step"][sel] = abi.STEP_PRECOMMIT
    st["round"][sel] = 0
    st["valid_present"][sel] = 1
    st["valid_round"][sel] = 0
    st["valid_value"][sel] = 7  # a value no vote carries
    g, o = run_both(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE | ROUTES[route], 2), hb, power,
                    None, st)
    assert_same(g, o)


# ------------------------------------------------ several rounds in one pass (flow)

def _reorder(hb, key):
    """The batch with each instance's votes stably reordered by key (per vote)."""
    order = np.lexsort((np.arange(hb.n_votes), key, hb.instance))
    return ol.batch_from_lists(hb.instance[order], hb.round[order], hb.type[order], hb.value[order],
                               hb.validator[order], hb.offsets.copy(), hb.instance_set)


def _round_states(n, R, seed):
    """Prevote / Precommit / NewRound States at rounds 0 .. R-1, so that the eqr-guarded
    arms (state_machine.rs:196-209) fire in every round's run."""
    st = _start_states(n, seed=seed)
    st["round"] = np.random.default_rng(seed).integers(0, R, n)
    return st


@pytest.mark.parametrize("lengths", [[8, 9, 10, 11, 12, 13, 14, 15, 17, 23],          # a start in most lanes
                                     [0, 0, 8, 13, 31, 97, 150, 203, 299, 301, 411],  # C2/C3-like, empty ones
                                     [9, 517, 1031, 2049]])                           # long, chunk-straddling
@pytest.mark.parametrize("rounds", ["one", "runs", "mixed"])
@pytest.mark.parametrize("flags", [0, abi.FLAG_STATE_MACHINE])
def test_unaligned_streams(eng, lengths, rounds, flags):
    """The flow kernel's unaligned-stream variant (round 6): instance offsets at every
    residue, a lane's votes split at any position between two instances (or, in runs
    mode, two rounds of one instance); instances of >= 8 votes.  'runs': each
    instance's rounds in order (one tally pass per chunk, run starts anywhere);
    'mixed': rounds in random order (a pass per round)."""
    R = 1 if rounds == "one" else 4
    hb = _ragged_batch(100 + len(lengths), 9000, 13, R, lengths)
    if rounds == "runs":
        hb = _reorder(hb, hb.round.astype(np.int64))
    power = ol.gen_power(5, 7, 13, abi.POWER_UNIFORM, 1, 30)
    st = _round_states(hb.n_instances, R, 9) if flags else None
    g, o = run_both(eng, abi.config(abi.MODE_REFERENCE, flags, R), hb, power, None, st)
    assert_same(g, o)
    if flags:
        assert g[1]["decided"].sum() > 0


@pytest.mark.parametrize("order", ["increasing", "decreasing", "revisit", "unaligned"])
def test_round_runs(eng, order):
    """The flow kernel tallies a chunk whose instances hold several rounds in one pass
    when every 4-vote unit holds one round and each instance's rounds increase inside
    the chunk (the (instance, round) runs are the segments); otherwise one pass per
    round.  4 validators x 2 types = 8 votes per round (unit-aligned round runs, many
    runs and commits per 512-vote chunk); 'unaligned' has 3 validators (6 votes per
    round: units straddle rounds)."""
    n_vals = 3 if order == "unaligned" else 4
    p = abi.gen_params(seed=77, n_instances=6000, n_vals=n_vals, rounds_min=1, rounds_max=8,
                       nil_permille=200)
    hb = ol.gen_batch(p)
    if order == "decreasing":
        hb = _reorder(hb, -hb.round.astype(np.int64))
    elif order == "revisit":
        hb = _reorder(hb, (hb.round.astype(np.int64) % 2) * 16 + hb.round)
    power = ol.gen_power(77, 3, n_vals, abi.POWER_UNIFORM, 1, 20)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 8)
    st = _round_states(p.n_instances, 8, 5)
    g, o = run_both(eng, cfg, hb, power, None, st)
    assert_same(g, o)
    assert g[1]["decided"].sum() > 100
    cfg0 = abi.config(abi.MODE_REFERENCE, 0, 8)
    g, o = run_both(eng, cfg0, hb, power)
    assert_same(g, o)


def _mixed_alignment_batch(seed, rounds):
    """An aligned generated batch (even validator count, no abstention: every offset a
    multiple of 4), a ragged one (abstention), and an aligned one again, as ONE batch: the
    call runs the kernel that holds both loops, which walks the aligned batches with the
    aligned loop and the others with the unaligned-stream loop (round 6)."""
    parts = []
    for k, absent in enumerate((0, 60, 0)):
        p = abi.gen_params(seed=seed + k, n_instances=1500, n_vals=24, rounds_min=1, rounds_max=rounds,
                           nil_permille=300, absent_permille=absent)
        parts.append(ol.gen_batch(p))
    assert (parts[0].offsets % 4 == 0).all() and (parts[1].offsets % 4 != 0).any()
    return ol.concat_batches(*parts)


@pytest.mark.parametrize("rounds", [1, 4])
@pytest.mark.parametrize("flags", [0, abi.FLAG_STATE_MACHINE])
def test_mixed_aligned_and_unaligned_batches(eng, rounds, flags):
    """Aligned and unaligned flow batches in one call (the gate picks the kernel with both
    loops; each batch takes its own loop): codes and States against the checker."""
    hb = _mixed_alignment_batch(140 + rounds, rounds)
    power = ol.gen_power(140, 3, 24, abi.POWER_UNIFORM, 1, 100)
    st = _start_states(hb.n_instances) if flags else None
    g, o = run_both(eng, abi.config(abi.MODE_REFERENCE, flags, rounds), hb, power, None, st)
    assert_same(g, o)
    if flags:
        assert g[1]["decided"].sum() > 0
