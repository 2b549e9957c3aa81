"""GPU event stream (agnes_event_offsets + agnes_events, through the C ABI) against
the checker (orc_tally_labels + orc_events): the same offsets and the same 24-B
records, bit for bit, on the codes the GPU tally wrote (which equal the checker's)."""
import numpy as np
import pytest
import torch

import oracle_lib as ol
from agnes_amd import abi
from agnes_amd.engine import DeviceBatch, Engine, states_to_device

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    e = Engine(0)
    yield e
    e.close()


def _run(eng, cfg, hb, power, states=None, shift=0):
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.zeros(max(hb.n_votes, 1), dtype=torch.uint8, device=eng.device)
    dst = None if states is None else states_to_device(states, eng.device)
    eng.tally(cfg, db, codes, dst)
    if shift:  # u8 columns 4..12 bytes past a 16-B boundary, values 4 bytes: the dword path
        def shifted(t, elem):
            n = t.numel()
            buf = torch.zeros(n + 16 // elem, dtype=t.dtype, device=t.device)
            k = shift // elem
            buf[k:k + n] = t
            return buf[k:k + n]
        db.round, db.type = shifted(db.round, 1), shifted(db.type, 1)
        db.value = shifted(db.value, 4)
        codes = shifted(codes, 1)
    offs, recs = eng.events(cfg, db, codes)
    torch.cuda.synchronize()
    g_codes = codes[:hb.n_votes].cpu().numpy()
    g_offs = offs.cpu().numpy().astype(np.uint64)
    g_ev = recs.cpu().numpy().reshape(-1).view(abi.VOTE_EVENT_DTYPE)
    o_codes, _, _, o_offs, o_ev = ol.events(cfg, hb, power, None, states, threads=8)
    assert np.array_equal(g_codes, o_codes)
    assert np.array_equal(g_offs, o_offs)
    if g_ev.tobytes() != o_ev.tobytes():
        bad = np.nonzero(g_ev != o_ev)[0]
        raise AssertionError(f"{len(bad)} of {len(o_ev)} records differ; first {bad[0]}: "
                             f"gpu {g_ev[bad[0]]} checker {o_ev[bad[0]]}")
    return o_ev


@pytest.mark.parametrize("flags", [abi.FLAG_STATE_MACHINE | abi.FLAG_DISTINCT_VALUES, 0])
def test_gpu_events_one_round(eng, flags):
    p = abi.gen_params(seed=41, n_instances=3000, n_vals=100, rounds_min=1, rounds_max=1, nil_permille=200)
    hb = ol.gen_batch(p)
    power = ol.gen_power(41, 1, 100, abi.POWER_UNIFORM, 1, 1000)
    cfg = abi.config(abi.MODE_REFERENCE, flags, 1)
    st = abi.new_states(3000, 1, abi.STEP_PREVOTE) if flags else None
    ev = _run(eng, cfg, hb, power, st)
    vals = ev[np.isin(ev["kind"], [abi.EV_POLKA_VALUE, abi.EV_PRECOMMIT_VALUE])]
    assert len(vals) and (vals["value"] != abi.NIL).all()


def test_gpu_events_dedup_skip(eng):
    p = abi.gen_params(seed=42, n_instances=2000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                       dup_permille=100, equiv_permille=100, higher_permille=50)
    hb = ol.gen_batch(p)
    power = ol.gen_power(42, 64, 150, abi.POWER_ZIPF, 1, 1_000_000)
    hb.instance_set = (np.arange(2000) % 64).astype(np.uint32)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP | abi.FLAG_DISTINCT_VALUES, 5)
    ev = _run(eng, cfg, hb, power, abi.new_states(2000, 1, abi.STEP_PREVOTE))
    assert (ev["kind"] == abi.EV_ROUND_SKIP).any()


@pytest.mark.parametrize("shift", [4, 8, 12])
def test_gpu_events_unaligned(eng, shift):
    p = abi.gen_params(seed=43, n_instances=500, n_vals=40, rounds_min=1, rounds_max=3, nil_permille=300)
    hb = ol.gen_batch(p)
    power = ol.gen_power(43, 1, 40, abi.POWER_ZIPF, 1, 1000)
    _run(eng, abi.config(abi.MODE_REFERENCE, 0, 3), hb, power, shift=shift)


def test_gpu_events_ragged_and_invalid(eng):
    """empty instances, ragged lengths, invalid votes (wrong instance, round,
    validator) and a vote whose value is nil everywhere"""
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 40, 300)
    lens[::7] = 0
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    n = int(off[-1])
    inst = np.repeat(np.arange(300, dtype=np.uint32), lens)
    rnd = rng.integers(0, 3, n).astype(np.uint8)
    typ = rng.integers(0, 2, n).astype(np.uint8)
    val = rng.integers(0, 5, n).astype(np.uint32)
    val[rng.random(n) < 0.3] = abi.NIL
    vdr = rng.integers(0, 10, n).astype(np.uint32)
    inst[rng.random(n) < 0.02] += 1
    rnd[rng.random(n) < 0.02] = 9
    vdr[rng.random(n) < 0.02] = 50
    hb = ol.batch_from_lists(inst, rnd, typ, val, vdr, off)
    power = ol.gen_power(44, 1, 10, abi.POWER_UNIFORM, 1, 10)
    _run(eng, abi.config(abi.MODE_REFERENCE, 0, 3), hb, power)


GUARD = 64  # records past the capacity handed to the call, filled with a canary


def _guarded(n, width, device):
    """a uint8 [n + GUARD, width] buffer of 0xCD: the call gets capacity n"""
    return torch.full((n + GUARD, width), 0xCD, dtype=torch.uint8, device=device)


def _guard_intact(buf, n):
    return bool((buf[n:].cpu().numpy() == 0xCD).all())


@pytest.mark.parametrize("route", ["walk", "stream"])
def test_records_bounded_by_capacity(eng, route):
    """Round 6 (review item 3): every dense writer is bounded on the device.  agnes_events
    handed an `out` that holds half its offsets' records, or offsets that are not the
    batch's (every instance's segment halved), writes nothing outside `out` and reports
    the dropped records through agnes_records_overflow; the records that fit are the
    right ones.  The same for agnes_records_compact given counts that are not the
    segments' and for agnes_edges / agnes_edges_compact.  ('walk': the value column off
    16-B alignment takes the lane-per-instance emit; 'stream': the batch-stream emit.)"""
    p = abi.gen_params(seed=47, n_instances=3000, n_vals=60, rounds_min=1, rounds_max=2, nil_permille=250)
    hb = ol.gen_batch(p)
    power = ol.gen_power(47, 3, 60, abi.POWER_UNIFORM, 1, 500)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 2)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.zeros(hb.n_votes, dtype=torch.uint8, device=eng.device)
    eng.tally(cfg, db, codes, states_to_device(abi.new_states(3000, 1, abi.STEP_PREVOTE), eng.device))
    dbe = DeviceBatch.from_host(hb, eng.device)  # the two-call stream's batch
    if route == "walk":
        v = torch.zeros(hb.n_votes + 4, dtype=db.value.dtype, device=eng.device)
        v[1:1 + hb.n_votes] = db.value
        dbe.value = v[1:1 + hb.n_votes]
    offs, recs = eng.events(cfg, dbe, codes)
    assert eng.records_overflow() == 0
    total = int(offs[-1].item())
    good = recs.cpu().numpy()
    # (1) out holds half the records
    half = total // 2
    out = _guarded(half, 24, eng.device)
    eng.events_into(cfg, dbe, codes, offs, out[:half])
    torch.cuda.synchronize()
    assert eng.records_overflow() == total - half
    assert _guard_intact(out, half)
    assert np.array_equal(out[:half].cpu().numpy(), good[:half])
    # (2) offsets that are not the batch's: every instance's segment halved
    bad_offs = offs // 2
    out = _guarded(total, 24, eng.device)
    eng.events_into(cfg, dbe, codes, bad_offs, out[:total])
    torch.cuda.synchronize()
    assert eng.records_overflow() > 0
    assert _guard_intact(out, total)
    # (3) the compaction of segmented records with counts that are not the segments'
    st = states_to_device(abi.new_states(3000, 1, abi.STEP_PREVOTE), eng.device)
    counts, seg = eng.tally_records(cfg, db, codes, st, st)
    torch.cuda.synchronize()
    assert eng.records_overflow() == 0
    big = counts * 2 + 5
    dense = _guarded(total, 24, eng.device)
    eng.records_compact(cfg, db, big, seg, out=dense[:total])
    torch.cuda.synchronize()
    assert eng.records_overflow() > 0
    assert _guard_intact(dense, total)
    # (4) edges: a half-size out, then compacted segments with inflated counts
    eoffs, erecs = eng.edges(cfg, db, codes)
    etot = int(eoffs[-1].item())
    assert eng.records_overflow() == 0 and etot > 0
    b = db.c()
    eh = etot // 2
    eout = _guarded(eh, 16, eng.device)
    rc = eng.lib.agnes_edges(eng.ctx, __import__("ctypes").byref(cfg), __import__("ctypes").byref(b),
                             codes.data_ptr(), eoffs.data_ptr(), eout.data_ptr(), eh, None)
    assert rc == abi.OK
    torch.cuda.synchronize()
    assert eng.records_overflow() == etot - eh
    assert _guard_intact(eout, eh)
    st = states_to_device(abi.new_states(3000, 1, abi.STEP_PREVOTE), eng.device)
    ecnt, eseg = eng.tally_edges(cfg, db, codes, st, st)
    torch.cuda.synchronize()
    edense = _guarded(etot, 16, eng.device)
    eng.edges_compact(cfg, db, ecnt * 3 + 1, eseg, out=edense[:etot])
    torch.cuda.synchronize()
    assert eng.records_overflow() > 0
    assert _guard_intact(edense, etot)
