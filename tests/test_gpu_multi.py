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
