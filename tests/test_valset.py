"""Validator sets (include/agnes.h agnes_valset_build /
agnes_valset_find; agnes_amd/valset.py).  ValidatorSet (validators.rs:23-56) does
not compile, so no reference output pins this row ("parity unpinned"): the
checker orc_valset_build is cross-checked against a pure-Python restatement of the
intended behaviour (sort by address, Vec::dedup of equal validators, wrapping
total), and the GPU against the checker."""
import bisect

import numpy as np
import pytest
import torch

import oracle_lib as ol

M64 = (1 << 64) - 1


def _s64(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def py_build(addr, power, set_of, n_sets):
    """ValidatorSet::new per set: sorted by address (equal addresses by power, then
    index), consecutive equal (address, power) dropped, wrapping total"""
    n = len(power)
    so = [0] * n if set_of is None else [int(x) for x in set_of]
    keys = sorted(range(n), key=lambda i: (so[i], bytes(addr[i]), int(power[i]), i))
    order, prev = [], None
    for i in keys:
        if so[i] >= n_sets:
            continue
        k = (so[i], bytes(addr[i]), int(power[i]))
        if k == prev:
            continue
        prev = k
        order.append(i)
    offs = [sum(1 for i in order if so[i] < s) for s in range(n_sets)] + [len(order)]
    tot = []
    for s in range(n_sets):
        t = 0
        for i in order[offs[s]:offs[s + 1]]:
            t = _s64(t + int(power[i]))
        tot.append(t)
    return order, offs, tot


def _data(seed, n, L, n_sets, dup=0.2):
    rng = np.random.default_rng(seed)
    addr = rng.integers(0, 4 if L > 2 else 256, size=(n, L)).astype(np.uint8)  # small alphabet: equal addresses
    power = rng.integers(-5, 50, size=n).astype(np.int64)
    if n:
        d = rng.random(n) < dup  # exact copies of earlier validators
        src = rng.integers(0, n, size=n)
        addr[d] = addr[src[d]]
        power[d] = power[src[d]]
        power[:3] = [(1 << 62), (1 << 62), (1 << 62)][:min(3, n)]  # the total wraps
    set_of = rng.integers(0, n_sets + 1, size=n).astype(np.uint32)  # ids == n_sets are dropped
    return addr, power, set_of


@pytest.mark.parametrize("seed,n,L,n_sets", [(1, 0, 4, 1), (2, 1, 1, 1), (3, 300, 1, 3), (4, 500, 20, 5),
                                             (5, 400, 32, 1), (6, 1000, 3, 17)])
def test_oracle_valset_matches_python(seed, n, L, n_sets):
    addr, power, set_of = _data(seed, n, L, n_sets)
    so = set_of if n_sets > 1 else None
    order, offs, pout, tot = ol.valset_build(addr, power, so, n_sets)
    w_order, w_offs, w_tot = py_build(addr, power, so, n_sets)
    assert [int(x) for x in order] == w_order
    assert [int(x) for x in offs] == w_offs
    assert [int(x) for x in tot] == w_tot
    assert np.array_equal(pout, power[order.astype(np.int64)])


# ------------------------------------------------------------------ GPU

@pytest.fixture(scope="module")
def eng():
    from agnes_amd.engine import Engine
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    return Engine(0)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,L,n_sets", [(1, 0, 4, 1), (2, 1, 1, 1), (3, 5000, 2, 7), (4, 20000, 20, 1024),
                                             (5, 1_000_000, 32, 1), (6, 300000, 8, 3)])
def test_gpu_valset_build(eng, seed, n, L, n_sets):
    addr, power, set_of = _data(seed, n, L, n_sets)
    if n_sets == 1:
        set_of = None
    order, offs, pout, tot = ol.valset_build(addr, power, set_of, n_sets)
    d = eng.device
    g = eng.valset_build(torch.from_numpy(addr).to(d), torch.from_numpy(power).to(d),
                         None if set_of is None else torch.from_numpy(set_of.view(np.int32)).to(d), n_sets)
    g_order, g_offs, g_pout, g_tot, g_addr = (t.cpu().numpy() for t in g)
    assert np.array_equal(g_order.view(np.uint32), order)
    assert np.array_equal(g_offs.view(np.uint64), offs)
    assert np.array_equal(g_pout, pout) and np.array_equal(g_tot, tot)
    assert np.array_equal(g_addr, addr[order.astype(np.int64)])
    # find: every built validator is found at its first position; absent addresses are not
    if len(order):
        q = g_addr[::97]
        qs = None if set_of is None else set_of[order.astype(np.int64)][::97]
        k = eng.valset_find(g[4], g[1], torch.from_numpy(np.ascontiguousarray(q)).to(d),
                            None if qs is None else torch.from_numpy(qs.view(np.int32)).to(d)).cpu().numpy()
        keys = [bytes(a) for a in g_addr]
        for qi, kk in zip(range(len(q)), k):
            s = 0 if qs is None else int(qs[qi])
            lo, hi = int(offs[s]), int(offs[s + 1])
            first = bisect.bisect_left(keys, bytes(q[qi]), lo, hi)  # sorted within the set
            assert kk == first and keys[first] == bytes(q[qi])
        absent = np.full((1, L), 255, np.uint8)
        if not any(bytes(a) == bytes(absent[0]) for a in g_addr):
            assert eng.valset_find(g[4], g[1], torch.from_numpy(absent).to(d)).cpu().numpy()[0] == -1


@pytest.mark.gpu
def test_gpu_valset_add_update_remove(eng):
    """ValidatorSet::add / update / remove against the list model on the host"""
    from agnes_amd.valset import ValidatorSets
    d = eng.device
    rng = np.random.default_rng(9)
    L = 20
    addr = rng.integers(0, 256, size=(1000, L)).astype(np.uint8)
    power = rng.integers(1, 100, size=1000).astype(np.int64)
    vs = ValidatorSets(eng, torch.from_numpy(addr).to(d), torch.from_numpy(power).to(d), None, 1)
    model = {bytes(a): int(p) for a, p in zip(addr, power)}  # distinct random addresses
    # add 50 new + 10 exact copies (deduplicated)
    new = rng.integers(0, 256, size=(50, L)).astype(np.uint8)
    newp = rng.integers(1, 100, size=50).astype(np.int64)
    vs.add(torch.from_numpy(np.concatenate([new, addr[:10]])).to(d),
           torch.from_numpy(np.concatenate([newp, power[:10]])).to(d))
    model.update({bytes(a): int(p) for a, p in zip(new, newp)})
    # update 30 powers, remove 40 validators (5 absent)
    up = addr[100:130]
    upp = rng.integers(100, 200, size=30).astype(np.int64)
    vs.update(torch.from_numpy(up).to(d), torch.from_numpy(upp).to(d))
    model.update({bytes(a): int(p) for a, p in zip(up, upp)})
    rm = np.concatenate([addr[200:235], rng.integers(0, 256, size=(5, L)).astype(np.uint8)])
    vs.remove(torch.from_numpy(rm).to(d))
    for a in rm:
        model.pop(bytes(a), None)
    want = sorted(model.items())
    got_a = [bytes(a) for a in vs.addr.cpu().numpy()]
    got_p = [int(p) for p in vs.power.cpu().numpy()]
    assert list(zip(got_a, got_p)) == want
    assert int(vs.totals.cpu()[0]) == sum(p for _, p in want)
    assert vs.power_table(len(want) + 3).shape == (1, len(want) + 3)
