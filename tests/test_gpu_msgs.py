"""GPU batched apply_msg (agnes_apply_msgs through the C ABI) against the checker
(orc_apply_msgs) on generated multi-round scripts: codes, final States, every
Option<Message> and the invalid count, bit for bit."""
import numpy as np
import pytest
import torch

import oracle_lib as ol
from agnes_amd import abi
from agnes_amd.engine import DeviceBatch, Engine, states_to_device, states_to_host
from agnes_amd.lib import AgnesError
from agnes_amd.script import gen_script

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    e = Engine(0)
    yield e
    e.close()


def _dev(eng, sc):
    db = DeviceBatch.from_host(sc, eng.device)
    kinds = torch.from_numpy(np.ascontiguousarray(sc.kinds)).to(eng.device)
    pol = torch.from_numpy(np.ascontiguousarray(sc.pol_round)).to(eng.device)
    return db, kinds, pol


def _run(eng, cfg, sc, power, states, with_pol=True):
    eng.upload_power(power)
    db, kinds, pol = _dev(eng, sc)
    n = max(sc.n_votes, 1)
    codes = torch.full((n,), 0xEE, dtype=torch.uint8, device=eng.device)
    msgs = torch.full((n, 24), 0xEE, dtype=torch.uint8, device=eng.device)
    dst = states_to_device(states, eng.device)
    eng.apply_msgs(cfg, db, kinds, pol if with_pol else None, codes, dst, msgs)
    torch.cuda.synchronize()
    g_bad = eng.last_error_count()
    g_codes = codes[:sc.n_votes].cpu().numpy()
    g_msgs = msgs[:sc.n_votes].cpu().numpy().reshape(-1).view(abi.MESSAGE_DTYPE)
    g_st = states_to_host(dst)
    o_codes, o_st, o_msgs, o_bad = ol.apply_msgs(cfg, sc, sc.kinds, sc.pol_round if with_pol else None, power,
                                                 states)
    if not np.array_equal(g_codes, o_codes):
        bad = np.nonzero(g_codes != o_codes)[0]
        raise AssertionError(f"{len(bad)} codes differ; first {bad[0]}: gpu {g_codes[bad[0]]} "
                             f"checker {o_codes[bad[0]]}")
    if g_msgs.tobytes() != o_msgs.tobytes():
        bad = np.nonzero(g_msgs != o_msgs)[0]
        raise AssertionError(f"{len(bad)} of {len(o_msgs)} messages differ; first {bad[0]}: "
                             f"gpu {g_msgs[bad[0]]} checker {o_msgs[bad[0]]}")
    assert g_st.tobytes() == o_st.tobytes()
    assert g_bad == o_bad
    return o_codes, o_st, o_msgs


@pytest.mark.parametrize("flags", [0, abi.FLAG_DISTINCT_VALUES])
def test_gpu_msgs_multi_round(eng, flags):
    sc = gen_script(71, 5000, 20, 4)
    power = ol.gen_power(71, 16, 20, abi.POWER_UNIFORM, 1, 1000)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE | flags, 4)
    _, st, msgs = _run(eng, cfg, sc, power, abi.new_states(5000, 3, abi.STEP_NEW_ROUND))
    assert st["decided"].sum() > 1000 and (msgs["kind"] == abi.MSG_NEW_ROUND).any()


def test_gpu_msgs_max_rounds_and_weights(eng):
    sc = gen_script(72, 700, 9, 16, late_permille=150)
    rng = np.random.default_rng(72)
    sc.weight = rng.integers(-3, 100, size=sc.n_votes).astype(np.int64)
    power = ol.gen_power(72, 3, 9, abi.POWER_ZIPF, 1, 1_000_000)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_DISTINCT_VALUES, 16)
    _run(eng, cfg, sc, power, abi.new_states(700, 1, abi.STEP_NEW_ROUND))


def test_gpu_msgs_no_pol_and_ragged(eng):
    """pol_round NULL (-1 for every proposal); instances of different lengths
    (a script cut at ragged points) and empty instances."""
    sc = gen_script(73, 300, 6, 3)
    per = np.diff(sc.offsets.astype(np.int64))
    rng = np.random.default_rng(73)
    keep = rng.integers(0, per[0] + 1, size=sc.n_instances)
    keep[::7] = 0
    idx = np.concatenate([np.arange(int(o), int(o) + int(k)) for o, k in zip(sc.offsets[:-1], keep)])
    for f in ("instance", "round", "type", "value", "validator", "kinds", "pol_round"):
        setattr(sc, f, np.ascontiguousarray(getattr(sc, f)[idx]))
    sc.offsets = np.concatenate([[0], np.cumsum(keep)]).astype(np.uint64)
    power = ol.gen_power(73, 1, 6, abi.POWER_UNIFORM, 1, 10)
    cfg = abi.config(abi.MODE_REFERENCE, abi.FLAG_STATE_MACHINE, 3)
    _run(eng, cfg, sc, power, abi.new_states(300, 1, abi.STEP_NEW_ROUND), with_pol=False)


def test_gpu_msgs_unsupported(eng):
    sc = gen_script(74, 4, 3, 1)
    eng.upload_power(np.ones((1, 3), np.int64))
    db, kinds, pol = _dev(eng, sc)
    codes = torch.zeros(sc.n_votes, dtype=torch.uint8, device=eng.device)
    msgs = torch.zeros((sc.n_votes, 24), dtype=torch.uint8, device=eng.device)
    st = states_to_device(abi.new_states(4, 1, abi.STEP_NEW_ROUND), eng.device)
    for cfg in (abi.config(abi.MODE_DEDUP, 0, 1), abi.config(abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP, 1),
                abi.config(abi.MODE_REFERENCE, 0, 17)):
        with pytest.raises(AgnesError):
            eng.apply_msgs(cfg, db, kinds, pol, codes, st, msgs)
