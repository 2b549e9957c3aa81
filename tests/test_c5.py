"""C5 — one instance split into contiguous slices over waves and GPUs (SURVEY.md
§8(e): per-slice partial tallies, one exchange step, an exact rescan).

Parity bar: the per-vote codes of the split computation equal the checker's on
the whole instance tallied as one stream (oracle/agnes_oracle.c orc_tally).  The
CPU tests drive agnes_amd/dist.py tally_one_instance with the carried-tally
stand-in (tests/carried_fake.py), including a world_size-2 gloo run; the GPU tests
drive it on agnes_tally_carried through the C ABI.
"""
import copy
import dataclasses
import os
import socket
import sys
import types

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
from carried_fake import CarriedFake, DedupFake  # noqa: E402


def _instance(seed=5, n_vals=300, R=2, nil=250, kind=abi.POWER_ZIPF):
    """One instance: n_vals validators prevote and precommit in each of R rounds."""
    p = abi.gen_params(seed=seed, n_instances=1, n_vals=n_vals, rounds_min=R, rounds_max=R,
                       nil_permille=nil)
    hb = ol.gen_batch(p)
    power = ol.gen_power(seed, 1, n_vals, kind, 1, 1000)
    return hb, power, abi.config(abi.MODE_REFERENCE, 0, R)


def _slice(n, rank, world):
    lo = (n * rank // world) // 4 * 4
    hi = n if rank == world - 1 else (n * (rank + 1) // world) // 4 * 4
    return lo, hi


def _fake_tc(fake, hb, lo, hi, codes):
    def tc(one, off, counts):
        b = types.SimpleNamespace(instance=hb.instance[lo:hi], round=hb.round[lo:hi],
                                  type=hb.type[lo:hi], value=hb.value[lo:hi],
                                  validator=hb.validator[lo:hi],
                                  offsets=off.cpu().numpy().astype(np.int64), instance_set=None)
        cv = counts.numpy().view(abi.VOTE_COUNT_DTYPE).reshape(counts.shape[0], counts.shape[1])
        fake.tally_carried(one, b, codes, cv)
    return tc


def test_segment_offsets_partition():
    for n, s in [(0, 1), (3, 4), (1001, 7), (4096, 64)]:
        b = ad.segment_offsets(n, s)
        assert b[0] == 0 and b[-1] == n and len(b) == s + 1
        assert np.all(np.diff(b.astype(np.int64)) >= 0)
        assert np.all(b[:-1] % 4 == 0)


def test_fold_counts_is_the_sequential_fold():
    rng = np.random.default_rng(1)
    S, K = 9, 4
    w = torch.from_numpy(rng.integers(-1000, 1000, (S, K, 2)))
    lab = torch.from_numpy(np.where(rng.random((S, K)) < 0.4, abi.NIL,
                                    rng.integers(0, 7, (S, K))).astype(np.int64))
    ex_w, ex_lab, tot_w, tot_lab = ad.fold_counts(w, lab)
    acc_w = np.zeros((K, 2), np.int64)
    acc_l = np.full(K, abi.NIL, np.int64)
    for s in range(S):
        assert np.array_equal(ex_w[s].numpy(), acc_w)
        assert np.array_equal(ex_lab[s].numpy(), acc_l)
        acc_w = acc_w + w[s].numpy()
        acc_l = np.where(lab[s].numpy() != abi.NIL, lab[s].numpy(), acc_l)
    assert np.array_equal(tot_w.numpy(), acc_w) and np.array_equal(tot_lab.numpy(), acc_l)


@pytest.mark.parametrize("segments", [1, 3, 16])
def test_split_instance_equals_whole_cpu(segments):
    hb, power, cfg = _instance()
    want, _, _ = ol.tally(cfg, hb, power)
    codes = np.zeros(hb.n_votes, np.uint8)
    ad.tally_one_instance(_fake_tc(CarriedFake(power), hb, 0, hb.n_votes, codes), hb.n_votes, cfg,
                          segments, torch.device("cpu"))
    assert np.array_equal(codes, want)
    assert (want & abi.CODE_EVENT_MASK != 0).any()


def test_split_instance_continued_across_calls_cpu():
    """two calls on consecutive slices, the second continuing from the first's
    result (prior): a stream continued across calls"""
    hb, power, cfg = _instance(seed=9)
    want, _, _ = ol.tally(cfg, hb, power)
    fake = CarriedFake(power)
    mid = (hb.n_votes // 2) // 4 * 4
    c0 = np.zeros(mid, np.uint8)
    c1 = np.zeros(hb.n_votes - mid, np.uint8)
    fw, fl = ad.tally_one_instance(_fake_tc(fake, hb, 0, mid, c0), mid, cfg, 4, torch.device("cpu"))
    ad.tally_one_instance(_fake_tc(fake, hb, mid, hb.n_votes, c1), hb.n_votes - mid, cfg, 4,
                          torch.device("cpu"), prior=(fw, fl))
    assert np.array_equal(np.concatenate([c0, c1]), want)


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
        hb, power, cfg = _instance()
        lo, hi = _slice(hb.n_votes, rank, world)
        codes = np.zeros(hi - lo, np.uint8)
        fw, fl = ad.tally_one_instance(_fake_tc(CarriedFake(power), hb, lo, hi, codes), hi - lo, cfg, 5,
                                       torch.device("cpu"))
        q.put((rank, codes.tobytes(), fw.numpy().tobytes(), fl.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


def test_split_instance_two_ranks_gloo():
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
    hb, power, cfg = _instance()
    want, _, _ = ol.tally(cfg, hb, power)
    assert b"".join(r[1] for r in res) == want.tobytes()
    assert res[0][2] == res[1][2] and res[0][3] == res[1][3]  # every rank has the final tally
    # ... and it is the whole instance's
    codes = np.zeros(hb.n_votes, np.uint8)
    fw, fl = ad.tally_one_instance(_fake_tc(CarriedFake(power), hb, 0, hb.n_votes, codes), hb.n_votes,
                                   cfg, 1, torch.device("cpu"))
    assert res[0][2] == fw.numpy().tobytes() and res[0][3] == fl.numpy().tobytes()


# --------------------------------------------------- DEDUP across slices (CPU)

def _dedup_instance(seed=5, n_vals=300, R=2, nil=250):
    """One instance with 15 % exact duplicates and 15 % equivocations (DEDUP mode)."""
    p = abi.gen_params(seed=seed, n_instances=1, n_vals=n_vals, rounds_min=R, rounds_max=R,
                       nil_permille=nil, dup_permille=150, equiv_permille=150)
    hb = ol.gen_batch(p)
    power = ol.gen_power(seed, 1, n_vals, abi.POWER_ZIPF, 1, 1000)
    return hb, power, abi.config(abi.MODE_DEDUP, 0, R)


def _cpu_dedup_slice(hb, power, cfg, lo, hi, segments, in_pass=False):
    """This rank's slice [lo, hi) through tally_one_instance_dedup on the CPU stand-ins."""
    dd = DedupFake(*power.shape)
    sl = types.SimpleNamespace(instance=hb.instance[lo:hi], round=hb.round[lo:hi], type=hb.type[lo:hi],
                               validator=hb.validator[lo:hi])
    view = types.SimpleNamespace(instance=hb.instance, round=hb.round, type=hb.type.copy(),
                                 value=hb.value, validator=hb.validator)
    codes = np.zeros(hi - lo, np.uint8)

    def mask(base, f):
        view.type[lo:hi] = dd.mask(cfg, sl, base, f.numpy())

    fw, fl = ad.tally_one_instance_dedup(
        _fake_tc(CarriedFake(power), view, lo, hi, codes),
        lambda base, f: dd.first(cfg, sl, base, f.numpy()), mask,
        None if in_pass else (lambda: dd.reject(view.type[lo:hi], codes)), hi - lo, power.shape[1], cfg, segments,
        torch.device("cpu"), base=lo)
    return codes, fw, fl


@pytest.mark.parametrize("in_pass", [False, True])  # True: FLAG_MASKED_REJECTED, no reject call
@pytest.mark.parametrize("segments", [1, 3, 16])
def test_split_instance_dedup_equals_whole_cpu(segments, in_pass):
    hb, power, cfg = _dedup_instance()
    want, _, _ = ol.tally(cfg, hb, power)
    assert (want == abi.CODE_REJECTED).sum() > hb.n_votes // 10  # the stream has duplicates
    codes, _, _ = _cpu_dedup_slice(hb, power, cfg, 0, hb.n_votes, segments, in_pass)
    assert np.array_equal(codes, want)


def _with_instance_id(hb, iid):
    """The same single-instance stream with every vote naming instance `iid` (the
    split path's id, cfg.reserved; the one-stream reference keeps id 0 = its
    segment index)."""
    h = copy.copy(hb)
    h.instance = np.full_like(np.asarray(hb.instance), iid)
    return h


@pytest.mark.parametrize("segments", [1, 5])
def test_split_instance_dedup_nonzero_instance_id_cpu(segments):
    """the DEDUP checks and the carried tally take the instance id from one place
    (cfg.reserved): a nonzero id still masks every duplicate"""
    hb, power, cfg = _dedup_instance(seed=17, n_vals=200)
    hb.validator[[5, 50, 500]] = 10 ** 6  # out of range: INVALID in the one-stream DEDUP tally
    want, _, _ = ol.tally(cfg, hb, power)
    cfg9 = abi.config(abi.MODE_DEDUP, 0, cfg.max_rounds, 9)
    codes, _, _ = _cpu_dedup_slice(_with_instance_id(hb, 9), power, cfg9, 0, hb.n_votes, segments)
    assert (want == abi.CODE_REJECTED).any() and (want == abi.CODE_INVALID).any()
    assert np.array_equal(codes, want)


def _dedup_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hb, power, cfg = _dedup_instance(seed=8)
        lo, hi = _slice(hb.n_votes, rank, world)
        codes, fw, fl = _cpu_dedup_slice(hb, power, cfg, lo, hi, 3, in_pass=rank == 1)  # both ways
        q.put((rank, codes.tobytes(), fw.numpy().tobytes(), fl.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


def test_split_instance_dedup_two_ranks_gloo():
    """all_reduce(MIN) of the first-seen table + all_gather of the partial tallies:
    the ranks' codes concatenate to the whole instance's DEDUP codes"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dedup_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    hb, power, cfg = _dedup_instance(seed=8)
    want, _, _ = ol.tally(cfg, hb, power)
    assert b"".join(r[1] for r in res) == want.tobytes()
    assert res[0][2] == res[1][2] and res[0][3] == res[1][3]


# ------------------------------------------------------------------ GPU (C ABI)

@pytest.fixture(scope="module")
def eng():
    from agnes_amd.engine import Engine
    return Engine(0)


def _gpu_tc(eng, db, codes):
    def tc(one, off, counts):
        eng.tally_carried(one, dataclasses.replace(db, offsets=off, instance_set=None), codes, counts)
    return tc


@pytest.mark.gpu
@pytest.mark.parametrize("hip_fold", [False, True])
@pytest.mark.parametrize("segments,n_vals,R,nil", [(1, 3000, 1, 200), (7, 3000, 2, 200),
                                                   (64, 20000, 1, 200), (300, 20000, 3, 300),
                                                   (33, 5000, 2, 900)])
def test_gpu_split_instance(eng, segments, n_vals, R, nil, hip_fold):
    from agnes_amd.engine import DeviceBatch
    hb, power, cfg = _instance(seed=11 + segments, n_vals=n_vals, R=R, nil=nil)
    want, _, _ = ol.tally(cfg, hb, power)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.zeros(hb.n_votes, dtype=torch.uint8, device=eng.device)
    fw, fl = ad.tally_one_instance(_gpu_tc(eng, db, codes), hb.n_votes, cfg, segments, eng.device,
                                   fold=eng.fold_counts if hip_fold else None)
    torch.cuda.synchronize()
    assert np.array_equal(codes.cpu().numpy(), want)
    assert eng.last_error_count() == 0
    # the final VoteCounts equal the checker stand-in's one-stream fold
    cw, cl = ad.tally_one_instance(_fake_tc(CarriedFake(power), hb, 0, hb.n_votes, np.zeros(hb.n_votes, np.uint8)),
                                   hb.n_votes, cfg, 1, torch.device("cpu"))
    assert np.array_equal(fw.cpu().numpy(), cw.numpy()) and np.array_equal(fl.cpu().numpy(), cl.numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("S,K", [(1, 2), (7, 4), (1000, 2), (5000, 8), (8192, 2), (9000, 3)])
def test_gpu_fold_counts_equals_torch_fold(eng, S, K):
    """agnes_fold_counts (reset / apply / totals, carry, label conventions) against
    dist.fold_counts on random partials (wrapping weights, sparse labels)"""
    rng = np.random.default_rng(S * 31 + K)
    w = rng.integers(-(1 << 62), 1 << 62, (S, K, 2), dtype=np.int64)
    lab = np.where(rng.random((S, K)) < 0.3, rng.integers(0, 1 << 31, (S, K)), ad.NIL).astype(np.int64)
    carry = np.concatenate([rng.integers(-(1 << 62), 1 << 62, (K, 2), dtype=np.int64),
                            rng.choice([0, 5, 77], (K, 1))], axis=1).astype(np.int64)
    counts = torch.from_numpy(np.concatenate([w, lab[..., None]], axis=-1)).to(eng.device).contiguous()
    cr = torch.from_numpy(carry).to(eng.device).contiguous()
    tot = torch.empty((K, 3), dtype=torch.int64, device=eng.device)
    orig = counts.clone()
    eng.fold_counts(counts, carry=cr, totals=tot,
                    flags=abi.FOLD_APPLY | abi.FOLD_ZERO_LABELS | abi.FOLD_CARRY_ZERO_NONE | abi.FOLD_TOTAL_ZERO_LABELS)
    # torch: prior (label 0 = none) as the first "slice"
    pl = np.where(carry[:, 2] == 0, ad.NIL, carry[:, 2])
    allw = torch.from_numpy(np.concatenate([carry[None, :, :2], w])).contiguous()
    alll = torch.from_numpy(np.concatenate([pl[None], lab])).contiguous()
    ex_w, ex_lab, t_w, t_lab = ad.fold_counts(allw, alll)
    ex_lab = torch.where(ex_lab == ad.NIL, torch.zeros_like(ex_lab), ex_lab)
    t_lab = torch.where(t_lab == ad.NIL, torch.zeros_like(t_lab), t_lab)
    got = counts.cpu().numpy()
    assert np.array_equal(got[..., :2], ex_w[1:].numpy())
    assert np.array_equal(got[..., 2], ex_lab[1:].numpy())
    tg = tot.cpu().numpy()
    assert np.array_equal(tg[:, :2], t_w.numpy()) and np.array_equal(tg[:, 2], t_lab.numpy())
    # totals only (no APPLY): the slices stay as they are
    before = orig.clone()
    tot2 = torch.empty((K, 3), dtype=torch.int64, device=eng.device)
    eng.fold_counts(orig, carry=cr, totals=tot2, flags=abi.FOLD_CARRY_ZERO_NONE | abi.FOLD_TOTAL_ZERO_LABELS)
    assert torch.equal(orig, before) and torch.equal(tot2, tot)
    eng.fold_counts(counts, flags=abi.FOLD_RESET)
    r = counts.cpu().numpy()
    assert (r[..., :2] == 0).all() and (r[..., 2] == ad.NIL).all()


@pytest.mark.gpu
def test_gpu_split_instance_continued_across_calls(eng):
    from agnes_amd.engine import DeviceBatch
    hb, power, cfg = _instance(seed=21, n_vals=8000, R=2)
    want, _, _ = ol.tally(cfg, hb, power)
    eng.upload_power(power)
    mid = (hb.n_votes * 3 // 5) // 4 * 4
    out = []
    prior = None
    for lo, hi in [(0, mid), (mid, hb.n_votes)]:
        part = types.SimpleNamespace(instance=hb.instance[lo:hi], round=hb.round[lo:hi],
                                     type=hb.type[lo:hi], value=hb.value[lo:hi],
                                     validator=hb.validator[lo:hi],
                                     offsets=np.array([0, hi - lo], np.uint64))
        db = DeviceBatch.from_host(part, eng.device)
        codes = torch.zeros(hi - lo, dtype=torch.uint8, device=eng.device)
        prior = ad.tally_one_instance(_gpu_tc(eng, db, codes), hi - lo, cfg, 16, eng.device,
                                      prior=prior)
        out.append(codes.cpu().numpy())
    assert np.array_equal(np.concatenate(out), want)


@pytest.mark.gpu
def test_gpu_tally_carried_rejects(eng):
    """ONE_INSTANCE and MASKED_REJECTED need the carried entry point; the carried path is
    REFERENCE only"""
    from agnes_amd.engine import DeviceBatch
    from agnes_amd.lib import AgnesError
    hb, power, cfg = _instance(seed=3, n_vals=64, R=1)
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    codes = torch.zeros(hb.n_votes, dtype=torch.uint8, device=eng.device)
    with pytest.raises(AgnesError):
        eng.tally(abi.config(abi.MODE_REFERENCE, abi.FLAG_ONE_INSTANCE, 1), db, codes)
    with pytest.raises(AgnesError):
        eng.tally(abi.config(abi.MODE_REFERENCE, abi.FLAG_MASKED_REJECTED, 1), db, codes)
    counts = torch.zeros((1, 2, 3), dtype=torch.int64, device=eng.device)
    with pytest.raises(AgnesError):
        eng.tally_carried(abi.config(abi.MODE_DEDUP, 0, 1), db, codes, counts)


def _gpu_dedup_run(eng, hb, power, cfg, segments, hip_fold=True, fused=False, in_pass=False):
    from agnes_amd.engine import DeviceBatch
    eng.upload_power(power)
    db = DeviceBatch.from_host(hb, eng.device)
    n = hb.n_votes
    tmask = torch.empty(n, dtype=torch.uint8, device=eng.device)
    dbm = dataclasses.replace(db, type=tmask)
    codes = torch.zeros(n, dtype=torch.uint8, device=eng.device)
    ad.tally_one_instance_dedup(_gpu_tc(eng, dbm, codes),
                                lambda base, f: eng.dedup_first(cfg, db, base, f),
                                lambda base, f: eng.dedup_mask(cfg, db, base, f, tmask),
                                None if in_pass else (lambda: eng.dedup_reject(tmask, codes, n)),
                                n, power.shape[1], cfg, segments, eng.device,
                                fold=eng.fold_counts if hip_fold else None,
                                dedup_first_mask=(lambda base, f: eng.dedup_first_mask(cfg, db, base, f, tmask))
                                if fused else None)
    torch.cuda.synchronize()
    return codes.cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("in_pass", [False, True])  # AGNES_FLAG_MASKED_REJECTED instead of agnes_dedup_reject
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("segments,n_vals,R", [(1, 3000, 1), (16, 5000, 2), (300, 20000, 2),
                                               (64, 100000, 1)])
def test_gpu_split_instance_dedup(eng, segments, n_vals, R, fused, in_pass):
    hb, power, cfg = _dedup_instance(seed=31 + segments, n_vals=n_vals, R=R)
    want, _, _ = ol.tally(cfg, hb, power)
    got = _gpu_dedup_run(eng, hb, power, cfg, segments, fused=fused, in_pass=in_pass)
    assert np.array_equal(got, want)
    assert (got == abi.CODE_REJECTED).any()


@pytest.mark.gpu
@pytest.mark.parametrize("weights", [False, True])
def test_gpu_split_instance_dedup_id_weights(eng, weights):
    """nonzero instance id (cfg.reserved, one source) and an explicit weight column
    with out-of-range validators: the split DEDUP codes equal the one-stream DEDUP
    tally (a vote failing the DEDUP checks is INVALID there, whatever the weights)"""
    hb, power, cfg = _dedup_instance(seed=23, n_vals=3000, R=2)
    if weights:
        hb.weight = np.random.default_rng(5).integers(1, 5000, hb.n_votes).astype(np.int64)
    hb.validator[[3, 40, 400, hb.n_votes - 1]] = 10 ** 6
    want, _, _ = ol.tally(cfg, hb, power)
    cfg7 = abi.config(abi.MODE_DEDUP, 0, cfg.max_rounds, 7)
    got = _gpu_dedup_run(eng, _with_instance_id(hb, 7), power, cfg7, 9)
    assert (want == abi.CODE_INVALID).sum() >= 4
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_dedup_slices_with_bases(eng):
    """Two slices with their global bases, first-seen tables min-combined (the
    all_reduce), give the whole stream's mask — and a vote failing the DEDUP checks
    is never masked: it is made invalid (0xFF) for the carried tally."""
    from agnes_amd.engine import DeviceBatch
    hb, power, cfg = _dedup_instance(seed=13, n_vals=4000, R=2)
    hb.type[7] = 5
    hb.type[11] = 0xFE          # an invalid vote whose type byte is the mask value
    hb.validator[19] = 10 ** 6  # out of range
    eng.upload_power(power)
    n, K = hb.n_votes, 2 * cfg.max_rounds * power.shape[1]
    mid = (n // 3) // 4 * 4

    def part(lo, hi):
        return DeviceBatch.from_host(types.SimpleNamespace(
            instance=hb.instance[lo:hi], round=hb.round[lo:hi], type=hb.type[lo:hi], value=hb.value[lo:hi],
            validator=hb.validator[lo:hi], offsets=np.array([0, hi - lo], np.uint64)), eng.device)

    whole, a, b = part(0, n), part(0, mid), part(mid, n)
    fw = torch.full((K,), ad.INT64_MAX, dtype=torch.int64, device=eng.device)
    fa, fb = fw.clone(), fw.clone()
    eng.dedup_first(cfg, whole, 0, fw)
    eng.dedup_first(cfg, a, 0, fa)
    eng.dedup_first(cfg, b, mid, fb)
    fab = torch.minimum(fa, fb)
    assert torch.equal(fab, fw)
    tw = torch.empty(n, dtype=torch.uint8, device=eng.device)
    ta = torch.empty(mid, dtype=torch.uint8, device=eng.device)
    tb = torch.empty(n - mid, dtype=torch.uint8, device=eng.device)
    eng.dedup_mask(cfg, whole, 0, fw, tw)
    eng.dedup_mask(cfg, a, 0, fab, ta)
    eng.dedup_mask(cfg, b, mid, fab, tb)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat([ta, tb]), tw)
    t = tw.cpu().numpy()
    assert t[7] == 0xFF and t[11] == 0xFF and t[19] == 0xFF  # failing the DEDUP checks: always invalid
    dd = DedupFake(*power.shape)
    f = np.full(K, ad.INT64_MAX, np.int64)
    dd.first(cfg, hb, 0, f)
    assert np.array_equal(fw.cpu().numpy(), f)
    assert np.array_equal(t, dd.mask(cfg, hb, 0, f))


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("shift,max_rounds", [(0, 1), (1, 1), (3, 1), (0, 64)])
def test_gpu_dedup_first_table_prefilled(eng, shift, max_rounds, fused):
    """agnes_dedup_first (the counting sort over key buckets and LDS minima) and
    agnes_dedup_mask: the table equals the checker's min over valid votes, with
    entries the caller set lower kept (the API lowers, it does not overwrite), many
    buckets (200k keys) and many count blocks (~2.6e5 votes), invalid votes of every
    kind ignored; shift > 0 hands columns `shift` votes past their allocation (not
    16-B aligned: the one-vote-per-thread kernels), and the mask equals the checker's."""
    from agnes_amd.engine import DeviceBatch
    hb, power, cfg = _dedup_instance(seed=41, n_vals=100_000, R=1)
    # max_rounds 64: 12.8M keys, more buckets than the sort handles -> the atomic kernel
    # (and, fused, a filled table and the mask pass)
    cfg = abi.config(abi.MODE_DEDUP, 0, max_rounds)
    hb.type[::997] = 3
    hb.round[::1009] = 9
    hb.validator[::1013] = 10 ** 7
    eng.upload_power(power)
    K = 2 * cfg.max_rounds * power.shape[1]
    base = 123_456_789
    f0 = np.full(K, ad.INT64_MAX, np.int64)
    f0[::7] = np.arange(0, K, 7) % 5000   # lower than any base + j: must survive
    fw = torch.from_numpy(f0.copy()).to(eng.device)
    db = DeviceBatch.from_host(hb, eng.device)
    n = hb.n_votes - shift
    if shift:
        db = dataclasses.replace(db, instance=db.instance[shift:], round=db.round[shift:], type=db.type[shift:],
                                 value=db.value[shift:], validator=db.validator[shift:],
                                 offsets=torch.tensor([0, n], dtype=torch.int64, device=eng.device), n_votes=n)
    tm = torch.empty(n + 4, dtype=torch.uint8, device=eng.device)[shift:shift + n]
    if fused:  # agnes_dedup_first_mask: the table written whole (the prefill is not kept) and the mask
        f0 = np.full(K, ad.INT64_MAX, np.int64)
        fw.fill_(-7)
        eng.dedup_first_mask(cfg, db, base, fw, tm)
    else:
        eng.dedup_first(cfg, db, base, fw)
        eng.dedup_mask(cfg, db, base, fw, tm)
    torch.cuda.synchronize()
    sl = types.SimpleNamespace(instance=hb.instance[shift:], round=hb.round[shift:], type=hb.type[shift:],
                               validator=hb.validator[shift:])
    want = f0.copy()
    dd = DedupFake(*power.shape)
    dd.first(cfg, sl, base, want)
    got = fw.cpu().numpy()
    assert np.array_equal(got, want)
    assert (got[1::7] < ad.INT64_MAX).any() and (got[1::7] >= base).all()
    assert (got == ad.INT64_MAX).any()  # keys without a valid vote
    assert np.array_equal(tm.cpu().numpy(), dd.mask(cfg, sl, base, want))
