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
