"""C5 with the State machine: one instance split into slices (and ranks), its
State and the votes' message nibbles from agnes_one_sm_scan / _apply / _finish
(agnes_amd/dist.py one_instance_states) against the checker's whole-instance
orc_tally with AGNES_FLAG_STATE_MACHINE (one stream, state_machine.rs:183-214 per
vote event).  CPU: the pass stand-ins (tests/carried_fake.py OneSmFake), a
world_size-2 gloo run; GPU: the HIP passes, alone and behind the split tally."""
import dataclasses
import os
import socket
import sys

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from agnes_amd import abi  # noqa: E402
from agnes_amd import dist as ad  # noqa: E402
import oracle_lib as ol  # noqa: E402
from carried_fake import OneSmFake  # noqa: E402

# (step, round) the State enters with
STARTS = [(abi.STEP_PREVOTE, 0), (abi.STEP_PROPOSE, 0), (abi.STEP_PRECOMMIT, 0), (abi.STEP_NEW_ROUND, 0),
          (abi.STEP_COMMIT, 0), (abi.STEP_PREVOTE, 1)]


def _instance(seed, n_vals, R, nil, dedup=False):
    gen = dict(n_instances=1, n_vals=n_vals, rounds_min=R, rounds_max=R, nil_permille=nil)
    if dedup:
        gen.update(dup_permille=150, equiv_permille=150)
    p = abi.gen_params(seed=seed, **gen)
    hb = ol.gen_batch(p)
    power = ol.gen_power(seed, 1, n_vals, abi.POWER_ZIPF, 1, 1000)
    mode = abi.MODE_DEDUP if dedup else abi.MODE_REFERENCE
    return hb, power, mode


def _want(hb, power, mode, R, st0):
    """the checker: the whole instance as one stream, State machine on"""
    codes, st, _ = ol.tally(abi.config(mode, abi.FLAG_STATE_MACHINE, R), hb, power, states=st0)
    plain, _, _ = ol.tally(abi.config(mode, 0, R), hb, power)
    return codes, st, plain


def _start(step, rnd):
    return abi.new_states(1, 1, step, rnd)


def _cuts(n, parts):
    return [0] + [(n * k // parts) // 4 * 4 for k in range(1, parts)] + [n]


@pytest.mark.parametrize("step,rnd", STARTS)
@pytest.mark.parametrize("parts", [1, 3])
def test_one_sm_passes_equal_whole_cpu(step, rnd, parts):
    hb, power, mode = _instance(21 + parts, 200, 2, 250)
    st0 = _start(step, rnd)
    want, want_st, plain = _want(hb, power, mode, 2, st0)
    codes = plain.copy()
    st = st0.copy()
    fake = OneSmFake(st[0])
    marks = [OneSmFake.MAXM, OneSmFake.MAXM, 0, 0]
    cuts = _cuts(hb.n_votes, parts)
    for a, b in zip(cuts[:-1], cuts[1:]):  # every slice scans, then (after the MIN) every slice applies
        fake.scan(codes[a:b], hb.round[a:b], hb.value[a:b], a, marks)
    for a, b in zip(cuts[:-1], cuts[1:]):
        sub = codes[a:b]
        fake.apply(sub, hb.round[a:b], hb.value[a:b], a, marks)
        codes[a:b] = sub
    fake.finish(marks)
    assert np.array_equal(codes, want)
    assert st.tobytes() == want_st.tobytes()


def test_one_sm_covers_every_message_cpu():
    """the reference messages the split-instance State machine must produce (over
    a few generated instances: whether P1 comes before the commit varies)"""
    msgs, decided = set(), 0
    for seed in range(23, 29):
        hb, power, mode = _instance(seed, 200, 1, 250)
        want, st, _ = _want(hb, power, mode, 1, _start(abi.STEP_PREVOTE, 0))
        msgs |= set(int(x) for x in (want >> abi.CODE_MSG_SHIFT))
        decided += int(st["decided"][0])
    assert {abi.VMSG_TIMEOUT_PREVOTE, abi.VMSG_TIMEOUT_PRECOMMIT, abi.VMSG_DECISION} <= msgs
    assert msgs & {abi.VMSG_PRECOMMIT_NIL, abi.VMSG_PRECOMMIT_VALUE}
    assert decided > 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hb, power, mode = _instance(29, 300, 2, 250)
        _, _, plain = _want(hb, power, mode, 2, _start(abi.STEP_PREVOTE, 0))
        cuts = _cuts(hb.n_votes, world)
        a, b = cuts[rank], cuts[rank + 1]
        codes = plain[a:b].copy()
        st = _start(abi.STEP_PREVOTE, 0)
        fake = OneSmFake(st[0])
        marks = ad.new_one_sm_marks(torch.device("cpu"))

        def run(f):
            def go(m):
                mm = [int(x) for x in m]
                f(mm)
                m.copy_(torch.tensor(mm, dtype=torch.int64))
            return go
        ad.one_instance_states(run(lambda m: fake.scan(codes, hb.round[a:b], hb.value[a:b], a, m)),
                               run(lambda m: fake.apply(codes, hb.round[a:b], hb.value[a:b], a, m)),
                               run(lambda m: fake.finish(m)), marks)
        q.put((rank, codes.tobytes(), st.tobytes()))
    finally:
        dist.destroy_process_group()


def test_one_sm_two_ranks_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    hb, power, mode = _instance(29, 300, 2, 250)
    want, want_st, _ = _want(hb, power, mode, 2, _start(abi.STEP_PREVOTE, 0))
    assert b"".join(r[1] for r in res) == want.tobytes()
    assert res[0][2] == res[1][2] == want_st.tobytes()  # every rank ends with the instance's State


# ------------------------------------------------------------------ GPU

@pytest.fixture(scope="module")
def eng():
    from agnes_amd.engine import Engine
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return Engine(0)


def _gpu_passes(eng, cfg, db, codes, st, cuts):
    """the three HIP passes over consecutive slices of one GPU's batch (each slice
    as a rank would run it: scan all, then apply all -- the MIN / MAX combine is
    the atomics on the shared marks)"""
    marks = ad.new_one_sm_marks(eng.device)
    subs = [dataclasses.replace(db, round=db.round[a:b], value=db.value[a:b], n_votes=b - a)
            for a, b in zip(cuts[:-1], cuts[1:])]
    for (a, _), sb in zip(zip(cuts[:-1], cuts[1:]), subs):
        eng.one_sm_scan(cfg, sb, a, codes[a:], st, marks)
    for (a, _), sb in zip(zip(cuts[:-1], cuts[1:]), subs):
        eng.one_sm_apply(cfg, sb, a, codes[a:], st, marks)
    eng.one_sm_finish(marks, st)


@pytest.mark.gpu
@pytest.mark.parametrize("step,rnd", STARTS)
@pytest.mark.parametrize("parts,n_vals,R,nil", [(1, 3000, 1, 200), (5, 20000, 2, 300), (2, 100000, 1, 950)])
def test_gpu_one_sm_passes(eng, step, rnd, parts, n_vals, R, nil):
    from agnes_amd.engine import DeviceBatch, states_to_device, states_to_host
    hb, power, mode = _instance(41 + parts, n_vals, R, nil)
    st0 = _start(step, rnd)
    want, want_st, plain = _want(hb, power, mode, R, st0)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.from_numpy(plain.copy()).to(eng.device)
    st = states_to_device(st0, eng.device)
    _gpu_passes(eng, abi.config(mode, 0, R), db, codes, st, _cuts(hb.n_votes, parts))
    torch.cuda.synchronize()
    got = codes.cpu().numpy()
    if not np.array_equal(got, want):
        bad = np.nonzero(got != want)[0]
        raise AssertionError(f"{len(bad)} codes differ; first {bad[0]}: gpu {got[bad[0]]:#x} checker {want[bad[0]]:#x}")
    assert states_to_host(st).tobytes() == want_st.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("dedup", [False, True])
def test_gpu_split_instance_with_states(eng, dedup):
    """the whole C5 step with the State machine: split tally (HIP folds), then the
    State machine passes; codes and State equal the one-stream checker"""
    from agnes_amd.engine import DeviceBatch, states_to_device, states_to_host
    hb, power, mode = _instance(47, 200000, 1, 200, dedup=dedup)
    st0 = _start(abi.STEP_PREVOTE, 0)
    want, want_st, _ = _want(hb, power, mode, 1, st0)
    cfg = abi.config(mode, 0, 1)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    n = hb.n_votes
    codes = torch.zeros(n, dtype=torch.uint8, device=eng.device)

    def tc_for(b):
        def tc(one, off, counts):
            eng.tally_carried(one, dataclasses.replace(b, offsets=off, instance_set=None), codes, counts)
        return tc
    if dedup:
        tmask = torch.empty(n, dtype=torch.uint8, device=eng.device)
        ad.tally_one_instance_dedup(tc_for(dataclasses.replace(db, type=tmask)),
                                    lambda base, f: eng.dedup_first(cfg, db, base, f),
                                    lambda base, f: eng.dedup_mask(cfg, db, base, f, tmask),
                                    lambda: eng.dedup_reject(tmask, codes, n), n, power.shape[1], cfg, 256,
                                    eng.device, fold=eng.fold_counts)
    else:
        ad.tally_one_instance(tc_for(db), n, cfg, 256, eng.device, fold=eng.fold_counts)
    st = states_to_device(st0, eng.device)
    ad.one_instance_states(lambda m: eng.one_sm_scan(cfg, db, 0, codes, st, m),
                           lambda m: eng.one_sm_apply(cfg, db, 0, codes, st, m),
                           lambda m: eng.one_sm_finish(m, st), ad.new_one_sm_marks(eng.device))
    torch.cuda.synchronize()
    assert np.array_equal(codes.cpu().numpy(), want)
    assert states_to_host(st).tobytes() == want_st.tobytes()
    assert want_st["decided"][0] == 1


@pytest.mark.gpu
def test_gpu_one_sm_rejects(eng):
    from agnes_amd.engine import DeviceBatch, states_to_device
    from agnes_amd.lib import AgnesError
    hb, power, mode = _instance(5, 100, 1, 200)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.zeros(hb.n_votes, dtype=torch.uint8, device=eng.device)
    st = states_to_device(_start(abi.STEP_PREVOTE, 0), eng.device)
    marks = ad.new_one_sm_marks(eng.device)
    with pytest.raises(AgnesError):
        eng.one_sm_scan(abi.config(abi.MODE_REFERENCE, abi.FLAG_ROUND_SKIP, 1), db, 0, codes, st, marks)
    with pytest.raises(AgnesError):
        eng.one_sm_scan(abi.config(abi.MODE_REFERENCE, 0, 1), db, (1 << 31) - 10, codes, st, marks)
