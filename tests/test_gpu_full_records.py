"""Full-size parity of the emitted records (north_star (c)): the
stream-compacted Option<Event> records (agnes_event_offsets + agnes_events) and the
edge-triggered summaries (agnes_edge_offsets + agnes_edges) of the bench's batches,
every record, against the checker (orc_tally_labels + orc_events, orc_edges).

  C2  1M instances x 100 validators x 1 round (the bench's c2 batch, 2e8 votes)
  C3  a 125k-instance shard: 150 validators x 1..4 rounds (up to ~1,200 votes per
      instance: the emit kernel's LDS label carry runs across many 256-vote passes)
  C4  a 125k-instance shard: DEDUP + RoundSkip + DISTINCT_VALUES, Zipf power,
      duplicates, equivocations and next-round votes

Reference semantics: VoteExecutor::apply / to_event (vote_executor.rs:20-36); the
value of PolkaValue(v) / PrecommitValue(v) is the executor bucket's last non-nil
value (round_votes.rs:50-54).  Slow: 1e8..2e8 votes through the checker."""
import os

import numpy as np
import pytest
import torch

import oracle_lib as ol
from agnes_amd import abi
from agnes_amd import dist as ad
from agnes_amd.engine import DeviceBatch, Engine, states_to_device

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

THREADS = max(1, len(os.sched_getaffinity(0)))


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    e = Engine(0)
    yield e
    e.close()


def _first_diff(g, o, what):
    if g.tobytes() != o.tobytes():
        if len(g) != len(o):
            raise AssertionError(f"{what}: {len(g)} records on the GPU, {len(o)} on the checker")
        k = int(np.nonzero(g != o)[0][0])
        raise AssertionError(f"{what} {k} of {len(o)}: gpu {g[k]} checker {o[k]}")


def _records(eng, cfg, p, power, n_sets, step=abi.STEP_PREVOTE):
    hb = ol.gen_batch(p)
    hb.instance_set = ad.set_of_instances(ad.Shard(p, 0, p.n_instances), n_sets)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    st0 = abi.new_states(p.n_instances, 1, step)
    codes = torch.zeros(hb.n_votes, dtype=torch.uint8, device=eng.device)
    eng.tally(cfg, db, codes, states_to_device(st0, eng.device))
    e_offs, e_recs = eng.events(cfg, db, codes)
    g_e_offs = e_offs.cpu().numpy().view(np.uint64)
    g_ev = e_recs.cpu().numpy().reshape(-1).view(abi.VOTE_EVENT_DTYPE)
    del e_offs, e_recs
    d_offs, d_recs = eng.edges(cfg, db, codes)
    g_d_offs = d_offs.cpu().numpy().view(np.uint64)
    g_ed = d_recs.cpu().numpy().reshape(-1).view(abi.EDGE_DTYPE)
    g_codes = codes.cpu().numpy()
    del d_offs, d_recs, codes, db
    torch.cuda.empty_cache()

    o_codes, _, _, o_e_offs, o_ev = ol.events(cfg, hb, power, None, st0, threads=THREADS)
    if not np.array_equal(g_codes, o_codes):
        k = int(np.nonzero(g_codes != o_codes)[0][0])
        raise AssertionError(f"code {k}: gpu {g_codes[k]:#x} checker {o_codes[k]:#x}")
    assert np.array_equal(g_e_offs, o_e_offs)
    _first_diff(g_ev, o_ev, "event")
    o_d_offs, o_ed = ol.edges(cfg, hb, o_codes)
    assert np.array_equal(g_d_offs, o_d_offs)
    _first_diff(g_ed, o_ed, "edge")
    return hb, o_ev, o_ed


def test_full_records_c2(eng):
    p = abi.gen_params(seed=0xA6E5, n_instances=1_000_000, n_vals=100, rounds_min=1, rounds_max=1,
                       nil_permille=200)
    power = ol.gen_power(0xA6E5, 1, 100, abi.POWER_UNIFORM, 1, 1000)
    hb, ev, ed = _records(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 1), p, power, 1)
    assert len(ev) > hb.n_votes // 4 and len(ed) > p.n_instances
    assert (ev["kind"] == abi.EV_PRECOMMIT_VALUE).any()


def test_full_records_c3_shard(eng):
    p = abi.gen_params(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                       nil_permille=300)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_UNIFORM, 1, 1000)
    hb, ev, _ = _records(eng, abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 4), p, power, 1024)
    lens = np.diff(hb.offsets.astype(np.int64))
    assert lens.max() > 1000  # instances longer than four 256-vote emit passes
    assert (ev["round"] == 3).any()


def test_full_records_c4_shard(eng):
    p = abi.gen_params(seed=0xA6E5, n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                       nil_permille=300, dup_permille=100, equiv_permille=100, higher_permille=50)
    power = ol.gen_power(0xA6E5, 1024, 150, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(abi.MODE_DEDUP,
                     abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP | abi.FLAG_DISTINCT_VALUES, 5)
    _, ev, _ = _records(eng, cfg, p, power, 1024)
    assert (ev["kind"] == abi.EV_ROUND_SKIP).any()
    vals = ev[np.isin(ev["kind"], [abi.EV_POLKA_VALUE, abi.EV_PRECOMMIT_VALUE])]
    assert len(vals) and (vals["value"] != abi.NIL).all()
