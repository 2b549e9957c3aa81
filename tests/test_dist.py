"""Multi-process (world_size 2, gloo, CPU) tests of the sharded path.

The device work is per-rank and collective-free, so what must hold for
multi-GPU correctness is checked here with the CPU checker standing in for each
rank's device result: shards partition the instances, every rank generates
exactly its slice of the global streams, per-shard results equal the global
result's slice (instance independence), and the collectives (max/sum timing
reductions, decision-summary all_gather) combine ranks correctly.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


GEN = dict(n_instances=600, n_vals=31, rounds_min=1, rounds_max=3, nil_permille=300,
           dup_permille=100, equiv_permille=100, higher_permille=50)


def _worker(rank, world, port, strong, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_lib as ol
        from agnes_amd import abi
        from agnes_amd import dist as ad

        sh = ad.make_shard(GEN, rank, world, strong)
        hb = ol.gen_batch(sh.params)
        hb.instance_set = ad.set_of_instances(sh, 64)
        power = ol.gen_power(7, 64, GEN["n_vals"], abi.POWER_ZIPF, 1, 10000)
        cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 4)
        st0 = abi.new_states(sh.params.n_instances, 1, abi.STEP_PREVOTE)
        codes, st, _ = ol.tally(cfg, hb, power, None, st0)
        local_dec = ad.decisions(st, sh.base)
        all_dec = ad.gather_decisions(local_dec)
        # the bench's exchange of emitted edge records (variable length per rank)
        import torch
        _, recs = ol.edges(cfg, hb, codes)
        recs = recs.copy()
        recs["instance"] += sh.base                       # global instance / vote indices
        recs["vote"] += int(ol.gen_offsets(abi.gen_params(seed=0xA6E5, **dict(
            GEN, n_instances=sh.base + sh.params.n_instances)))[sh.base]) if sh.base else 0
        parts = ad.gather_edges(torch.from_numpy(recs.view(np.uint8).reshape(len(recs), -1).copy()))
        edges_all = b"".join(bytes(p_.numpy().tobytes()) for p_ in parts)
        timed = ad.gather_edges_timed(torch.from_numpy(recs.view(np.uint8).reshape(len(recs), -1).copy()))
        total_votes = ad.sum_over_ranks(hb.n_votes)
        tmax = ad.max_over_ranks(float(rank + 1))
        q.put((rank, sh.base, sh.params.n_instances, codes.tobytes(), st.tobytes(),
               all_dec.tobytes(), total_votes, tmax, edges_all, timed["records"]))
    finally:
        dist.destroy_process_group()


def _run(strong):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, strong, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res)


@pytest.mark.parametrize("strong", [True, False])
def test_sharded_equals_whole(strong):
    import oracle_lib as ol
    from agnes_amd import abi
    from agnes_amd import dist as ad

    res = _run(strong)
    world = 2
    n_total = GEN["n_instances"] * (1 if strong else world)
    # shards partition the global instance range
    bases = [r[1] for r in res]
    sizes = [r[2] for r in res]
    assert bases[0] == 0 and bases[1] == sizes[0] and sum(sizes) == n_total
    # the whole batch, generated and tallied once
    whole = ad.Shard(abi.gen_params(seed=0xA6E5, **dict(GEN, n_instances=n_total)), 0, n_total)
    hb = ol.gen_batch(whole.params)
    hb.instance_set = ad.set_of_instances(whole, 64)
    power = ol.gen_power(7, 64, GEN["n_vals"], abi.POWER_ZIPF, 1, 10000)
    cfg = abi.config(abi.MODE_DEDUP, abi.FLAG_ROUND_SKIP | abi.FLAG_STATE_MACHINE, 4)
    codes, st, _ = ol.tally(cfg, hb, power, None, abi.new_states(n_total, 1, abi.STEP_PREVOTE))
    assert b"".join(r[3] for r in res) == codes.tobytes()
    assert b"".join(r[4] for r in res) == st.tobytes()
    # collectives
    dec = ad.decisions(st, 0)
    _, erecs = ol.edges(cfg, hb, codes)
    for r in res:
        assert r[8] == erecs.tobytes()        # all_gather of edge records, rank order
        assert r[9] == len(erecs)
        assert r[5] == dec.tobytes()          # all_gather of decision summaries, rank order
        assert r[6] == hb.n_votes              # sum of per-rank votes
        assert r[7] == 2.0                     # max over ranks
    assert len(dec) > 0
