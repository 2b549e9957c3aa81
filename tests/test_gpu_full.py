"""Full-size parity (BASELINE.json configs at the bench's sizes, one GPU's share):
the HIP engine through the C ABI against the CPU checker on the same generated
batch, bit-exact codes, final States and invalid counts.  Slow: each case tallies
10^8 .. 2x10^8 votes on the checker (all CPUs of the process) and moves them
between host and device.

  C2  1M instances x 100 validators x 1 round (the bench's c2 batch), State machine
  C2w the same with i64 stakes U[2^28, 2^34] (the bench's c2w batch, u64 sums)
  C3  a 125k-instance shard of 1M x 150 validators x 1..4 rounds, 1024 power sets
  C3r the C3 shard with 5 % abstention (ragged instance lengths, round 6); C2r likewise
  C3w the same with i64 stakes U[2^28, 2^34] (the bench's c3w batch, flow<W64> runs mode)
  C4  125k instances, Zipf power, 10 % duplicates + 10 % equivocations + 5 %
      next-round votes, DEDUP + RoundSkip + State machine
  C5  one instance x 1M validators (Zipf), REFERENCE and DEDUP (10 % + 10 %),
      split into 1024 slices (agnes_amd/dist.py tally_one_instance[_dedup])
"""
import dataclasses
import os

import numpy as np
import pytest
import torch

import oracle_lib as ol
from agnes_amd import abi
from agnes_amd import dist as ad
from agnes_amd.engine import DeviceBatch, Engine, states_to_device, states_to_host

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

THREADS = max(1, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    e = Engine(0)
    yield e
    e.close()


def _compare(eng, cfg, p, power, n_sets, step=abi.STEP_PREVOTE):
    hb = ol.gen_batch(p)
    sh = ad.Shard(p, 0, p.n_instances)
    hb.instance_set = ad.set_of_instances(sh, n_sets)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    st0 = abi.new_states(p.n_instances, 1, step)
    st_in = states_to_device(st0, eng.device)
    st_out = torch.empty_like(st_in)
    codes = torch.zeros(hb.n_votes, dtype=torch.uint8, device=eng.device)
    eng.tally_states(cfg, db, codes, st_in, st_out)
    torch.cuda.synchronize()
    g_codes = codes.cpu().numpy()
    g_bad = eng.last_error_count()
    g_st = states_to_host(st_out)
    del db, codes, st_in, st_out
    torch.cuda.empty_cache()
    o_codes, o_st, o_bad = ol.tally(cfg, hb, power, None, st0, threads=THREADS)
    if not np.array_equal(g_codes, o_codes):
        bad = np.nonzero(g_codes != o_codes)[0]
        raise AssertionError(f"{len(bad)} of {len(o_codes)} codes differ; first at {bad[0]}: "
                             f"gpu {g_codes[bad[0]]:#x} checker {o_codes[bad[0]]:#x}")
    assert g_bad == o_bad
    assert g_st.tobytes() == o_st.tobytes()
    return o_codes, o_st


def test_full_c2(eng):
    p = abi.gen_params(seed=0xA6E5, n_instances=1_000_000, n_vals=100, rounds_min=1, rounds_max=1,
                       nil_permille=200)
    power = ol.gen_power(0xA6E5, 1, 100, abi.POWER_UNIFORM, 1, 1000)
    codes, st = _compare(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1), p, power, 1)
    assert st["decided"].sum() > 0 and ((codes >> abi.CODE_MSG_SHIFT) != 0).any()


def test_full_c2w(eng):
    """The bench's c2w batch: the C2 shape with i64 stakes U[2^28, 2^34] (set total
    ~8.6e11 > 2^32), through the u64-sum route (agnes_set_info.w64)."""
    p = abi.gen_params(seed=0xA6E5, n_instances=1_000_000, n_vals=100, rounds_min=1, rounds_max=1,
                       nil_permille=200)
    power = ol.gen_power(0xA6E5, 1, 100, abi.POWER_UNIFORM, 1 << 28, 1 << 34)
    assert power.sum() > (1 << 32)
    codes, st = _compare(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1), p, power, 1)
    assert st["decided"].sum() > 0 and ((codes >> abi.CODE_MSG_SHIFT) != 0).any()


def test_full_c3_shard(eng):
    p = abi.gen_params(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                       nil_permille=300)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_UNIFORM, 1, 1000)
    _, st = _compare(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4), p, power, 1024)
    assert st["decided"].sum() > 0


def test_full_c3r_shard(eng):
    """The bench's c3r batch (round 6): the C3 shard with 5 % abstention -- every round
    drops a random subset of its votes, so instance lengths and offsets take any value
    (no 4-aligned stream), as a real validator set with absent validators produces."""
    p = abi.gen_params(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                       nil_permille=300, absent_permille=50)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_UNIFORM, 1, 1000)
    _, st = _compare(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4), p, power, 1024)
    assert st["decided"].sum() > 0


def test_full_c2r(eng):
    """The bench's c2r batch (round 6): C2 with 5 % abstention (ragged 1-round instances)."""
    p = abi.gen_params(seed=0xA6E5, n_instances=1_000_000, n_vals=100, rounds_min=1, rounds_max=1,
                       nil_permille=200, absent_permille=50)
    power = ol.gen_power(0xA6E5, 1, 100, abi.POWER_UNIFORM, 1, 1000)
    codes, st = _compare(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1), p, power, 1)
    assert st["decided"].sum() > 0 and ((codes >> abi.CODE_MSG_SHIFT) != 0).any()


def test_full_c3w_shard(eng):
    """The bench's c3w batch: a 125k-instance C3 shard with i64 stakes U[2^28, 2^34] over
    1024 sets (set totals > 2^32), 1..4 rounds: flow<W64> in runs mode (round 5)."""
    p = abi.gen_params(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                       nil_permille=300)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_UNIFORM, 1 << 28, 1 << 34)
    assert power.sum(axis=1).min() > (1 << 32)
    _, st = _compare(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4), p, power, 1024)
    assert st["decided"].sum() > 0


def test_full_c2wr(eng):
    """The bench's c2wr batch (round 6): c2w with 5 % abstention -- i64 stakes over ragged
    1-round instances, through the u64 flow kernel's unaligned-stream variant."""
    p = abi.gen_params(seed=0xA6E5, n_instances=1_000_000, n_vals=100, rounds_min=1, rounds_max=1,
                       nil_permille=200, absent_permille=50)
    power = ol.gen_power(0xA6E5, 1, 100, abi.POWER_UNIFORM, 1 << 28, 1 << 34)
    codes, st = _compare(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1), p, power, 1)
    assert st["decided"].sum() > 0 and ((codes >> abi.CODE_MSG_SHIFT) != 0).any()


def test_full_c3wr_shard(eng):
    """The bench's c3wr batch (round 6): the c3w shard with 5 % abstention."""
    p = abi.gen_params(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                       nil_permille=300, absent_permille=50)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_UNIFORM, 1 << 28, 1 << 34)
    _, st = _compare(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4), p, power, 1024)
    assert st["decided"].sum() > 0


def test_full_c4_shard(eng):
    p = abi.gen_params(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                       nil_permille=300, dup_permille=100, equiv_permille=100, higher_permille=50)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP, 5)
    codes, _ = _compare(eng, cfg, p, power, 1024)
    assert (codes == abi.CODE_REJECTED).any()


def _c5(eng, dedup, fused=False):
    n_vals = 1_000_000
    gen = dict(n_instances=1, n_vals=n_vals, rounds_min=1, rounds_max=1, nil_permille=200)
    if dedup:
        gen.update(dup_permille=100, equiv_permille=100)
    p = abi.gen_params(seed=0xA6E5, **gen)
    hb = ol.gen_batch(p)
    power = ol.gen_power(0xA6E5, 1, n_vals, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(abi.MODE_DEDUP if dedup else abi.MODE_REFERENCE, 0, 1)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    n = hb.n_votes
    codes = torch.zeros(n, dtype=torch.uint8, device=eng.device)
    tmask = torch.empty(n, dtype=torch.uint8, device=eng.device)
    dbm = dataclasses.replace(db, type=tmask) if dedup else db

    def tc(one, off, counts):
        eng.tally_carried(one, dataclasses.replace(dbm, offsets=off, instance_set=None), codes, counts)

    if dedup:
        ad.tally_one_instance_dedup(tc, lambda base, f: eng.dedup_first(cfg, db, base, f),
                                    lambda base, f: eng.dedup_mask(cfg, db, base, f, tmask),
                                    None if fused else (lambda: eng.dedup_reject(tmask, codes, n)), n, n_vals, cfg, 1024,
                                    eng.device,
                                    dedup_first_mask=(lambda base, f: eng.dedup_first_mask(cfg, db, base, f, tmask))
                                    if fused else None)
    else:
        ad.tally_one_instance(tc, n, cfg, 1024, eng.device)
    torch.cuda.synchronize()
    got = codes.cpu().numpy()
    want, _, _ = ol.tally(cfg, hb, power)
    if not np.array_equal(got, want):
        bad = np.nonzero(got != want)[0]
        raise AssertionError(f"{len(bad)} codes differ; first at {bad[0]}: gpu {got[bad[0]]:#x} "
                             f"checker {want[bad[0]]:#x}")
    return want


def test_full_c5_reference(eng):
    want = _c5(eng, False)
    assert (want & abi.CODE_EVENT_MASK).any()


@pytest.mark.parametrize("fused", [False, True])
def test_full_c5_dedup(eng, fused):
    want = _c5(eng, True, fused)
    assert (want == abi.CODE_REJECTED).sum() > len(want) // 20
