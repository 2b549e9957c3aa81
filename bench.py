#!/usr/bin/env python3
"""Agnes vote-tally bench: votes tallied/sec on MI355X (BASELINE.json metric).

One step = one pass of the fused hot path (agnes_tally: ingest -> weight gather
-> ordered tally -> quorum -> event -> State::apply) over one batch of
synthetic votes already resident in HBM, plus the per-height State::new reset
of the batch's instances (a device copy, timed).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4]

N > 1: launched by torch.distributed.run, one rank per GPU; instances shard
with no data-path collective (c2/c4: every rank its own batch = weak scaling;
c3: the 1M-instance batch split over ranks = strong scaling).
"""
from __future__ import annotations

import argparse
import json
import math
import struct
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from agnes_amd import abi  # noqa: E402
from agnes_amd import dist as adist  # noqa: E402
from agnes_amd.engine import Engine, states_to_device, states_to_host  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)
BYTES_PER_VOTE = 15            # 14 B canonical SoA in + 1 B code out
# algorithmic bytes per vote of each engine kernel (names: agnes_kernel_times)
KERNEL_BYTES_PER_VOTE = {
    "flow": 15,          # instance, value, validator u32 + round, type u8 in; code u8 out
    "flow_ragged": 15,   # the same, the kernel that also holds the unaligned-stream loop (round 6: c2r / c3r)
    "flow_prep": 0,      # the flow route's gate: 8 B per instance (the offsets), not per vote
    "tally_fast": 15,
    "tally_wide": 15,
    "tally_list": 15,    # the i64 kernel over the instances the u32 kernels hand over (c2w: all)
    "sweep_walk": 15,
    "apply_codes": 2,    # code + round u8 in (+ the message bytes written back)
    "dedup_first": 10,   # C5 DEDUP: instance, validator u32 + round, type u8 in (bucket sort: + 2x8 B pairs)
    "dedup_mask": 11,    # the same in, the masked type u8 out
    "dedup_first_mask": 11,  # one rank: both in one counting sort (10 B in, the masked type out)
    "partials": 22,      # C5 pass A: the 14 B in + the i64 weight column out (the power table
                         # gather hits the cache-resident table: not compulsory HBM traffic)
}
# C5 pass B reads the weight column pass A wrote (AGNES_FLAG_WEIGHTS_CACHED) on top of the 15 B
C5_PASS_B_BYTES_PER_VOTE = 23
# SURVEY.md §8(d), amortized extras: with the State machine on, each instance's State is
# read and written once per step (64-B agnes_state in, 64 B out) by the kernel that
# applies the events (flow on the fused route, apply_codes on the split one)
STATE_BYTES_PER_INSTANCE = 128
KERNEL_STATE_IO = {"flow", "flow_ragged", "apply_codes", "tally_list", "sweep_walk"}
KERNEL_SYMBOLS = {
    # template parameters: PC (power table in LDS), SM (State machine), R1 (one round);
    # c2 runs flow<true, true, true>, c3 flow<false, true, false> (rocprofv3 names them)
    "flow": "agnes::flow::flow<PC, SM, R1>",
    "flow_ragged": "agnes::flow::flow<PC, SM, R1, ..., RG=true>",
    "flow_prep": "agnes::flow::flow_prep",
    "sweep_walk": "agnes::sweep::sweep<PC, SM>",
    "tally_fast": "agnes::fast::tally_fast<...>",
    "tally_wide": "agnes::tally_kernel<true, ...>",
    "tally_list": "agnes::tally_kernel<true, MODE, SKIP, SM, LIST=true>",
    "apply_codes": "agnes::apply::apply_codes<RoundSkip>",
    "partials": "agnes::partials::partials_kernel",
    "dedup_first": "agnes::dedup::bucket_{count,prefix,scatter,min}",
    "dedup_mask": "agnes::dedup::mask_kernel",
    "dedup_first_mask": "agnes::dedup::bucket_{count,prefix,scatter,min}<MASK>",
}

WORKLOADS = {
    # BASELINE configs[1] = C2, timed over 100 batched heights
    "c2": dict(desc="C2x100: 10k instances x 100 weighted validators x 1 round, 100 heights "
                    "per batch, 80/20 value/nil, shuffled",
               gen=dict(n_instances=10_000 * 100, n_vals=100, rounds_min=1, rounds_max=1,
                        nil_permille=200),
               power=(abi.POWER_UNIFORM, 1, 1000, 1), mode=abi.MODE_REFERENCE,
               flags=abi.FLAG_STATE_MACHINE, max_rounds=1, scaling="weak"),
    "c3": dict(desc="C3: 1M instances x 150 validators x 1..4 rounds, 30% nil, 1024 power sets, "
                    "sharded over ranks",
               gen=dict(n_instances=1_000_000, n_vals=150, rounds_min=1, rounds_max=4,
                        nil_permille=300),
               power=(abi.POWER_UNIFORM, 1, 1000, 1024), mode=abi.MODE_REFERENCE,
               flags=abi.FLAG_STATE_MACHINE, max_rounds=4, scaling="strong"),
    # one C3 rank's share on 8 GPUs (125k instances, global ids 0..125k): the strong-scaling
    # shard size, measured on one GPU (queue tail and per-wave imbalance at 1/8 the work)
    "c3shard": dict(desc="C3 8-GPU shard: 125k instances x 150 validators x 1..4 rounds, 30% nil, "
                         "1024 power sets (one rank's share of C3 on 8 GPUs)",
                    gen=dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                             nil_permille=300),
                    power=(abi.POWER_UNIFORM, 1, 1000, 1024), mode=abi.MODE_REFERENCE,
                    flags=abi.FLAG_STATE_MACHINE, max_rounds=4, scaling="weak"),
    # round 6: the same shapes with 5 % abstention -- each round drops a random subset of
    # its votes (absent validators), so instance lengths and offsets take any value: the
    # ragged streams a real validator set produces (no 4-aligned instance starts)
    "c2r": dict(desc="C2x100 with 5% abstention: 1M instances x 100 weighted validators x 1 round, "
                     "ragged lengths (absent validators), 80/20 value/nil, shuffled",
                gen=dict(n_instances=10_000 * 100, n_vals=100, rounds_min=1, rounds_max=1,
                         nil_permille=200, absent_permille=50),
                power=(abi.POWER_UNIFORM, 1, 1000, 1), mode=abi.MODE_REFERENCE,
                flags=abi.FLAG_STATE_MACHINE, max_rounds=1, scaling="weak"),
    "c3r": dict(desc="C3 8-GPU shard with 5% abstention: 125k instances x 150 validators x 1..4 rounds, "
                     "30% nil, 1024 power sets, ragged lengths (absent validators)",
                gen=dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                         nil_permille=300, absent_permille=50),
                power=(abi.POWER_UNIFORM, 1, 1000, 1024), mode=abi.MODE_REFERENCE,
                flags=abi.FLAG_STATE_MACHINE, max_rounds=4, scaling="weak"),
    # the C2 shape with i64 stakes: powers U[2^28, 2^34], set totals ~8.6e11 > 2^32 (the
    # reference's i64 arithmetic, round_votes.rs:9,16-18,31-33), through the route the
    # engine picks for a set outside the u32 domain
    "c2w": dict(desc="C2x100 with i64 stakes: 1M instances x 100 validators x 1 round, powers "
                     "U[2^28, 2^34] (set totals > 2^32), 80/20 value/nil, shuffled",
                gen=dict(n_instances=10_000 * 100, n_vals=100, rounds_min=1, rounds_max=1,
                         nil_permille=200),
                power=(abi.POWER_UNIFORM, 1 << 28, 1 << 34, 1), mode=abi.MODE_REFERENCE,
                flags=abi.FLAG_STATE_MACHINE, max_rounds=1, scaling="weak"),
    # one C3 rank's shard with i64 stakes: powers U[2^28, 2^34] over 1024 sets (set totals
    # > 2^32), 1..4 rounds (round_votes.rs:9,16-18,31-33; validators.rs:7): flow<W64> runs mode
    "c3w": dict(desc="C3 8-GPU shard with i64 stakes: 125k instances x 150 validators x 1..4 rounds, "
                     "30% nil, powers U[2^28, 2^34] over 1024 sets (set totals > 2^32)",
                gen=dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300),
                power=(abi.POWER_UNIFORM, 1 << 28, 1 << 34, 1024), mode=abi.MODE_REFERENCE,
                flags=abi.FLAG_STATE_MACHINE, max_rounds=4, scaling="weak"),
    # the i64-stake shapes with 5 % abstention (round 6): flow<W64>'s unaligned-stream loop
    "c2wr": dict(desc="C2x100 with i64 stakes and 5% abstention: 1M instances x 100 validators x 1 round, "
                      "powers U[2^28, 2^34], ragged lengths",
                 gen=dict(n_instances=10_000 * 100, n_vals=100, rounds_min=1, rounds_max=1,
                          nil_permille=200, absent_permille=50),
                 power=(abi.POWER_UNIFORM, 1 << 28, 1 << 34, 1), mode=abi.MODE_REFERENCE,
                 flags=abi.FLAG_STATE_MACHINE, max_rounds=1, scaling="weak"),
    "c3wr": dict(desc="C3 8-GPU shard with i64 stakes and 5% abstention: 125k instances x 150 validators x "
                      "1..4 rounds, powers U[2^28, 2^34] over 1024 sets, ragged lengths",
                 gen=dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4, nil_permille=300,
                          absent_permille=50),
                 power=(abi.POWER_UNIFORM, 1 << 28, 1 << 34, 1024), mode=abi.MODE_REFERENCE,
                 flags=abi.FLAG_STATE_MACHINE, max_rounds=4, scaling="weak"),
    "c4": dict(desc="C4: C3 shape per rank (125k instances), Zipf power, 10% dup + 10% "
                    "equivocation + 5% next-round votes, DEDUP + RoundSkip",
               gen=dict(n_instances=125_000, n_vals=150, rounds_min=1, rounds_max=4,
                        nil_permille=300, dup_permille=100, equiv_permille=100,
                        higher_permille=50),
               power=(abi.POWER_ZIPF, 1, 1_000_000, 1024), mode=abi.MODE_DEDUP,
               flags=abi.FLAG_STATE_MACHINE | abi.FLAG_ROUND_SKIP, max_rounds=5, scaling="weak"),
    "c5": dict(desc="C5: 1 instance x 1M validators (Zipf power), prevote + precommit: 2e6 votes in one "
                    "stream, split over ranks and per rank over segments; one all_gather of partial tallies",
               gen=dict(n_instances=1, n_vals=1_000_000, rounds_min=1, rounds_max=1, nil_permille=200),
               power=(abi.POWER_ZIPF, 1, 1_000_000, 1), mode=abi.MODE_REFERENCE, flags=0,
               max_rounds=1, scaling="strong", one_instance=True, segments=2048),
    "c5d": dict(desc="C5 in DEDUP mode: 1 instance x 1M validators (Zipf power), 10% duplicates + 10% "
                     "equivocations; one all_reduce(MIN) of first-seen indices + one all_gather of "
                     "partial tallies",
                gen=dict(n_instances=1, n_vals=1_000_000, rounds_min=1, rounds_max=1, nil_permille=200,
                         dup_permille=100, equiv_permille=100),
                power=(abi.POWER_ZIPF, 1, 1_000_000, 1), mode=abi.MODE_DEDUP, flags=0,
                max_rounds=1, scaling="strong", one_instance=True, segments=2048),
    # signed wire records -> verified SoA columns (not a BASELINE config)
    "wire": dict(desc="wire ingest: 104-byte signed vote records (Ed25519, OpenSSL-made fixture records "
                      "replicated to 2^20 per GPU, 48 of every 92 valid) -> verified SoA columns",
                 records=1 << 20, scaling="weak", wire=True),
}


def start_states(n: int) -> np.ndarray:
    """Every instance past NewRoundProposer + Proposal of round 0 (Prevote step)."""
    return abi.new_states(n, height=1, step=abi.STEP_PREVOTE, round_=0)


def measured_traffic(config: str):
    """HBM bytes per launch of each engine kernel for this workload, from the
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this same command committed under
    profiles/ (tools/pmc_traffic.py applies the gfx950 corrections of
    MI355X_MICROARCH.md: FETCH_SIZE x2, WRITE_SIZE as is): {kernel: record}."""
    try:
        with open(os.path.join(ROOT, "profiles", "traffic.json")) as f:
            rec = json.load(f).get(config) or {}
    except (OSError, ValueError):
        return {}
    return rec.get("kernels", {})


def host_cpu() -> dict:
    """The host the CPU baseline ran on: model, logical CPUs, the CPUs this process
    may run on, and the cgroup CPU quota when one is set."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    return {"model": model, "nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "cgroup_cpu_quota": quota}


def cpu_threads(cpu: dict) -> int:
    """Threads the CPU legs use: the CPUs this process may run on, capped by the
    cgroup CPU quota (a box may show 256 CPUs in its affinity mask and grant 16)."""
    n = max(1, cpu["affinity"])
    q = cpu.get("cgroup_cpu_quota")
    return max(1, min(n, math.ceil(q))) if q else n


def cpu_baseline(eng, cfg, batch, power, states0, set_of_instance):
    """The checker (oracle/, scalar C, one pthread per CPU this process may use,
    over instances) on the same batch; best of 5."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol  # test infrastructure: the CPU baseline leg only
    h = batch.to_host()
    n_inst = len(h["offsets"]) - 1
    # bounded sample: up to 1M instances (the whole c2 batch: ~2e8 votes)
    limit = min(n_inst, 1_000_000)
    off = h["offsets"][: limit + 1]
    nv = int(off[-1])
    hb = ol.HostBatch(h["instance"][:nv], h["round"][:nv], h["type"][:nv], h["value"][:nv],
                      h["validator"][:nv], off.copy(), set_of_instance[:limit].copy())
    cpu = host_cpu()
    threads = cpu_threads(cpu)
    best = None
    for _ in range(5):
        t0 = time.perf_counter()
        codes, st, _ = ol.tally(cfg, hb, power, None, states0[:limit], threads=threads)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return {"value": nv / best, "unit": "votes/s", "cores": threads, "kind": "port",
            "host": cpu,
            "sample": f"first {limit} instances ({nv} votes) of the same batch, "
                      f"oracle/agnes_oracle.c orc_tally_mt on {threads} threads, best of 5",
            "codes_prefix": codes, "states_prefix": st, "_sample": (hb, states0[:limit])}


def records_check(cfg, hb, power, states0, codes, ev_offs, ev_recs, ed_offs, ed_recs):
    """The GPU's event and edge records of the CPU-baseline sample (the first instances
    of the batch) against the checker's, every record.  Test infrastructure only: runs
    after the timed region."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol
    t0 = time.perf_counter()
    n = hb.n_instances
    threads = cpu_threads(host_cpu())
    _, _, _, o_offs, o_ev = ol.events(cfg, hb, power, None, states0, threads=threads)
    g_offs = ev_offs[: n + 1].cpu().numpy().view(np.uint64)
    g_ev = ev_recs[: int(g_offs[-1])].cpu().numpy().reshape(-1).view(abi.VOTE_EVENT_DTYPE)
    ev_ok = bool(np.array_equal(g_offs, o_offs) and g_ev.tobytes() == o_ev.tobytes())
    o_doffs, o_ed = ol.edges(cfg, hb, codes)
    g_doffs = ed_offs[: n + 1].cpu().numpy().view(np.uint64)
    g_ed = ed_recs[: int(g_doffs[-1])].cpu().numpy().reshape(-1).view(abi.EDGE_DTYPE)
    ed_ok = bool(np.array_equal(g_doffs, o_doffs) and g_ed.tobytes() == o_ed.tobytes())
    return {"instances": n, "votes": hb.n_votes, "events": len(o_ev), "events_equal": ev_ok,
            "edges": len(o_ed), "edges_equal": ed_ok, "seconds": time.perf_counter() - t0}


def edge_summary(eng, cfg, batch, codes, reps: int = 5):
    """The edge-triggered summary (agnes_edge_offsets + agnes_edges, §8(f) 1) of the
    last step's codes, timed OUTSIDE the bench's timed region (it is not part of
    `value`).  Algorithmic bytes: each walk reads code + round + type (3 B/vote) and
    one offset pair per instance; the count walk writes 8 B per instance, the emit
    walk 16 B per edge."""
    eng.edges(cfg, batch, codes)
    torch.cuda.synchronize()
    eng.kernel_timing(True)
    for _ in range(reps):
        offs, recs = eng.edges(cfg, batch, codes)
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.kernel_timing(False)
    nv, ni, ne = batch.n_votes, batch.n_instances, recs.shape[0]
    ab = {"edge_count": 3 * nv + 24 * ni, "edge_scan": 16 * ni, "edge_emit": 3 * nv + 16 * ni + 16 * ne}
    res = {"edges": int(ne), "edges_per_vote": ne / max(nv, 1), "_records": recs, "_offsets": offs}
    for name, (launches, total) in kt.items():
        avg = total / max(launches, 1)
        res[name] = {"avg_ms": avg, "algorithmic_bytes": ab.get(name),
                     "GBps": ab[name] / (avg * 1e-3) / 1e9 if name in ab and avg > 0 else None}
    return res


def with_traffic(res: dict, traffic: dict) -> dict:
    """Per-launch HBM bytes (the committed PMC passes) next to each timed kernel."""
    for name, rec in res.items():
        if isinstance(rec, dict) and "avg_ms" in rec:
            t = traffic.get(name)
            rec["traffic"] = t.get("traffic_bytes") if t else None
    return res


def event_stream(eng, cfg, batch, codes, reps: int = 3):
    """The stream-compacted event output (agnes_event_offsets + agnes_events: every
    Some(Event) with its payload) of the last step's codes, timed OUTSIDE the
    bench's timed region.  Algorithmic bytes: the count walk reads the codes (1 B /
    vote) and writes 8 B per instance; the emit walk reads code, round, type and
    value (7 B / vote) and writes 24 B per event."""
    eng.events(cfg, batch, codes)
    torch.cuda.synchronize()
    eng.kernel_timing(True)
    for _ in range(reps):
        offs, recs = eng.events(cfg, batch, codes)
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.kernel_timing(False)
    nv, ni, ne = batch.n_votes, batch.n_instances, recs.shape[0]
    ab = {"event_count": nv + 16 * ni, "event_scan": 16 * ni, "event_emit": 7 * nv + 8 * ni + 24 * ne}
    res = {"events": int(ne), "events_per_vote": ne / max(nv, 1), "_records": recs, "_offsets": offs}
    for name, (launches, total) in kt.items():
        avg = total / max(launches, 1)
        res[name] = {"avg_ms": avg, "algorithmic_bytes": ab.get(name),
                     "GBps": ab[name] / (avg * 1e-3) / 1e9 if name in ab and avg > 0 else None}
    return res


def tally_events_timed(eng, cfg, batch, codes, st0, states, steps, ref_offs, ref_recs):
    """agnes_tally_events: the step and its event stream in ONE call (SURVEY.md §8(b),
    the records counted inside the tally kernel), captured in a HIP graph and timed
    like the step, outside the timed region of `value`; its records must equal the
    two-call stream's (ref_offs / ref_recs) byte for byte."""
    cap = eng.events_capacity(cfg, batch)
    offs = torch.empty(batch.n_instances + 1, dtype=torch.int64, device=eng.device)
    out = torch.empty((max(cap, 1), 24), dtype=torch.uint8, device=eng.device)

    def call():
        eng.tally_events(cfg, batch, codes, st0, states, offs, out)

    call()
    torch.cuda.synchronize()
    eng.kernel_timing(True)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.kernel_timing(False)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        call()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        call()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    n = int(offs[-1].item())
    equal = bool(torch.equal(offs, ref_offs) and torch.equal(out[:n], ref_recs))
    del g, out
    return {"ms_per_call": ms, "records": n, "equal_to_two_call_stream": equal,
            "kernels": {name: {"launches": k, "avg_ms": t / max(k, 1)} for name, (k, t) in kt.items()}}


def tally_edges_timed(eng, cfg, batch, codes, st0, states, steps, ref_offs, ref_recs):
    """agnes_tally_edges (round 5): the step and its edge summary segmented by instance,
    found and written by the flow kernel (no pass over the codes), graph-captured and
    timed like the step outside the timed region of `value`; agnes_edges_compact's dense
    layout must equal the two-call summary's (ref_offs / ref_recs) byte for byte."""
    counts = torch.empty(max(batch.n_instances, 1), dtype=torch.int64, device=eng.device)
    seg = torch.empty((max(batch.n_votes, 1), 16), dtype=torch.uint8, device=eng.device)

    def call():
        eng.tally_edges(cfg, batch, codes, st0, states, counts, seg)

    call()
    torch.cuda.synchronize()
    eng.kernel_timing(True)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.kernel_timing(False)
    ms = graph_timed(call, steps)
    offs = torch.empty(batch.n_instances + 1, dtype=torch.int64, device=eng.device)
    dense = torch.empty((max(batch.n_votes, 1), 16), dtype=torch.uint8, device=eng.device)
    ms_c = graph_timed(lambda: eng.edges_compact(cfg, batch, counts, seg, offs, dense), steps)
    n = int(offs[-1].item())
    equal = bool(torch.equal(offs, ref_offs) and torch.equal(dense[:n], ref_recs))
    del seg, dense
    return {"ms_per_call": ms, "compact_ms": ms_c, "edges": n, "compacted_equal_to_two_call_summary": equal,
            "kernels": {name: {"launches": k, "avg_ms": t / max(k, 1)} for name, (k, t) in kt.items()}}


def graph_timed(fn, steps):
    """ms per call of fn captured in a HIP graph and replayed steps times"""
    fn()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    del g
    return (time.perf_counter() - t0) * 1e3 / steps


def tally_records_timed(eng, cfg, batch, codes, st0, states, steps, ref_offs, ref_recs):
    """agnes_tally_records (round 5): the step and its records SEGMENTED by instance, the
    flow kernel writing them while the votes are in registers (no pass over the votes
    after the tally), graph-captured and timed like the step, outside the timed region
    of `value`; then agnes_records_compact (one pass over the records) to the dense
    stream, which must equal the two-call stream's (ref_offs / ref_recs) byte for byte."""
    cap = eng.events_capacity(cfg, batch)
    counts = torch.empty(max(batch.n_instances, 1), dtype=torch.int64, device=eng.device)
    seg = torch.empty((max(cap, 1), 16), dtype=torch.uint8, device=eng.device)

    def call():
        eng.tally_records(cfg, batch, codes, st0, states, counts, seg)

    call()
    torch.cuda.synchronize()
    eng.kernel_timing(True)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    kt = eng.kernel_times()
    eng.kernel_timing(False)
    ms = graph_timed(call, steps)
    offs = torch.empty(batch.n_instances + 1, dtype=torch.int64, device=eng.device)
    dense = torch.empty((max(cap, 1), 24), dtype=torch.uint8, device=eng.device)
    ms_c = graph_timed(lambda: eng.records_compact(cfg, batch, counts, seg, offs, dense), steps)
    n = int(offs[-1].item())
    equal = bool(torch.equal(offs, ref_offs) and torch.equal(dense[:n], ref_recs))
    del seg, dense
    return {"ms_per_call": ms, "compact_ms": ms_c, "records": n, "compacted_equal_to_two_call_stream": equal,
            "kernels": {name: {"launches": k, "avg_ms": t / max(k, 1)} for name, (k, t) in kt.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--route", choices=["auto", "instance", "split", "wide"], default="auto",
                    help="force a tally route (AGNES_ROUTE_*; diagnostics: every route gives identical results)")
    ap.add_argument("--segments", type=int, default=0,
                    help="c5/c5d: segments per GPU (one wave each; default: the workload's)")
    args = ap.parse_args()

    rank, world, local = adist.env()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    # one rank per GPU; a rehearsal of the N > 1 path on a one-GPU box runs its ranks
    # on the same device over gloo (AGNES_BENCH_BACKEND=gloo: RCCL needs a GPU per rank)
    backend = os.environ.get("AGNES_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    w = WORKLOADS[args.config]
    eng = Engine(local)
    if w.get("wire"):
        return bench_wire(args, w, eng, rank, world)
    if w.get("one_instance"):
        return bench_one_instance(args, w, eng, rank, world)
    shard = adist.make_shard(w["gen"], rank, world, strong=w["scaling"] == "strong")
    p = shard.params
    kind, lo, hi, n_sets = w["power"]
    power = eng.gen_power(0xA6E5, n_sets, p.n_vals, kind, lo, hi)
    eng.upload_power(power)
    stream = torch.cuda.current_stream()
    batch = eng.gen_batch(p)
    set_of = adist.set_of_instances(shard, n_sets)   # global instance id mod n_sets
    batch.instance_set = torch.from_numpy(set_of.view(np.int32)).to(eng.device)
    route = {"auto": 0, "instance": 1, "split": 2, "wide": 3}[args.route]
    cfg = abi.config(w["mode"], w["flags"] | (route << 8), w["max_rounds"])
    st0_host = start_states(p.n_instances)
    st0 = states_to_device(st0_host, eng.device)
    states = torch.empty_like(st0)
    codes = torch.empty(batch.n_votes, dtype=torch.uint8, device=eng.device)
    torch.cuda.synchronize()

    def step():
        # State::new for this batch of heights (st0, read in place) -> the States after it
        eng.tally_states(cfg, batch, codes, st0, states)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if eng.last_error_count() != 0:
        raise SystemExit("bench batch has invalid votes")

    # per-kernel times: K eager steps with HIP events around every engine launch (on
    # the launch stream); the roofline's kernel duration comes from here
    eng.kernel_timing(True)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ktimes = eng.kernel_times()
    eng.kernel_timing(False)

    # the step (queue reset + flow + walk + list launches) captured once in a HIP graph
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        step()
    g.replay()
    torch.cuda.synchronize()

    # one HIP event pair around the K replays (events between the replays would sit in
    # the stream between the steps and be timed with them)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        g.replay()
    ev1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = adist.max_over_ranks(elapsed)
    total_votes_step = adist.sum_over_ranks(batch.n_votes)
    if world > 1:
        dist.barrier()
    step_gpu_ms = ev0.elapsed_time(ev1) / args.steps

    events = event_stream(eng, cfg, batch, codes)
    edges = edge_summary(eng, cfg, batch, codes)
    ev_offs, ev_recs = events.pop("_offsets"), events.pop("_records")
    te = tally_events_timed(eng, cfg, batch, codes, st0, states, args.steps, ev_offs, ev_recs)
    te["records_ms"] = te["ms_per_call"] - elapsed * 1e3 / args.steps  # over the tally step alone
    events["tally_events"] = te
    tr = tally_records_timed(eng, cfg, batch, codes, st0, states, args.steps, ev_offs, ev_recs)
    tr["records_ms"] = tr["ms_per_call"] - elapsed * 1e3 / args.steps
    events["tally_records"] = tr
    ed_offs = edges.pop("_offsets")
    tg = tally_edges_timed(eng, cfg, batch, codes, st0, states, args.steps, ed_offs, edges["_records"])
    tg["edges_ms"] = tg["ms_per_call"] - elapsed * 1e3 / args.steps  # over the tally step alone
    edges["tally_edges"] = tg
    if world > 1:  # every rank's edge records to every rank (RCCL), outside the timed region
        edges["all_gather"] = adist.gather_edges_timed(edges.pop("_records"))
        ed_recs = None
    else:
        ed_recs = edges.pop("_records")

    if rank == 0:
        ms_per_step = elapsed * 1e3 / args.steps
        value = total_votes_step * args.steps / elapsed
        # the States this GPU's step reads and writes (State machine on)
        st_bytes = STATE_BYTES_PER_INSTANCE * p.n_instances if w["flags"] & abi.FLAG_STATE_MACHINE else 0
        traffic = measured_traffic(args.config)
        with_traffic(events, traffic)
        with_traffic(edges, traffic)
        # per-kernel: launches, average ms, algorithmic bytes per launch
        kernels = {}
        for name, (launches, total) in ktimes.items():
            avg = total / max(launches, 1)
            ab = KERNEL_BYTES_PER_VOTE.get(name, 0) * batch.n_votes + (st_bytes if name in KERNEL_STATE_IO else 0)
            t = traffic.get(name)
            kernels[name] = {"launches": launches, "avg_ms": avg, "algorithmic_bytes": ab,
                             "GBps": ab / (avg * 1e-3) / 1e9 if ab and avg > 0 else None,
                             "traffic": t.get("traffic_bytes") if t else None}
        dom = max(kernels, key=lambda k: kernels[k]["avg_ms"] * kernels[k]["launches"])
        dom_ms = kernels[dom]["avg_ms"]
        ab_dom = KERNEL_BYTES_PER_VOTE[dom] * batch.n_votes + (st_bytes if dom in KERNEL_STATE_IO else 0)
        achieved = ab_dom / (dom_ms * 1e-3) / 1e9
        path_bytes = BYTES_PER_VOTE * batch.n_votes + st_bytes
        path_achieved = path_bytes / (ms_per_step * 1e-3) / 1e9
        td = traffic.get(dom)
        out = {
            "metric": "votes_tallied_per_sec",
            "value": value,
            "unit": "votes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": w["scaling"],
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (counter-based splitmix64 streams, agnes_gen.h; random powers)",
            "config": {"workload": w["desc"], "config": args.config,
                       "instances_per_gpu": p.n_instances, "validators": p.n_vals,
                       "votes_per_gpu_per_step": batch.n_votes,
                       "mode": "DEDUP" if w["mode"] else "REFERENCE",
                       "flags": w["flags"], "parallelism": f"instance-sharded x{world}",
                       "hip_graph": True},
            "kernel_ms": step_gpu_ms,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": td.get("traffic_bytes") if td else None,
                         "traffic_source": td.get("sources") if td else None,
                         "kernel": KERNEL_SYMBOLS.get(dom, dom),
                         "kernel_avg_ms": dom_ms,
                         "bytes_per_vote": KERNEL_BYTES_PER_VOTE[dom],
                         "state_bytes": st_bytes if dom in KERNEL_STATE_IO else 0,
                         "algorithmic_bytes": ab_dom,
                         # the whole step (every launch agnes_tally_states enqueues, wall
                         # clock of the timed region) at 15 B/vote against the same peak
                         "path_bytes": path_bytes,
                         "path_achieved": path_achieved,
                         "path_frac": path_achieved / HBM_PEAK_GBS},
            "kernels": kernels,
            "edge_summary": edges,
            "event_stream": events,
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(eng, cfg, batch, power, st0_host, set_of)
            cprefix = cb.pop("codes_prefix")
            sprefix = cb.pop("states_prefix")
            hb, st_s = cb.pop("_sample")
            # the GPU's codes and States of the last step against the checker's
            g_codes = codes[: len(cprefix)].cpu().numpy()
            g_states = states_to_host(states)[: len(sprefix)]
            ok_codes = bool(np.array_equal(g_codes, cprefix)
                            and np.array_equal(g_states.view(np.uint8), sprefix.view(np.uint8)))
            # ... and the emitted records of the same sample: the stream-compacted events
            # and the edge summaries (checker: orc_tally_labels + orc_events, orc_edges)
            out["cpu_check"] = records_check(cfg, hb, power, st_s, cprefix, ev_offs, ev_recs, ed_offs, ed_recs)
            out["cpu_check"]["codes_states_equal"] = ok_codes
            out["cpu_check_equal"] = ok_codes and out["cpu_check"]["events_equal"] and out["cpu_check"]["edges_equal"]
            out["cpu_baseline"] = cb
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def bench_one_instance(args, w, eng, rank, world):
    """C5: one instance's stream split over ranks (agnes_amd/dist.py
    tally_one_instance): two carried-tally passes + one all_gather per step."""
    import dataclasses
    from agnes_amd.engine import DeviceBatch
    p = abi.gen_params(seed=0xA6E5, **w["gen"])
    kind, plo, phi, n_sets = w["power"]
    power = eng.gen_power(0xA6E5, n_sets, p.n_vals, kind, plo, phi)
    eng.upload_power(power)
    stream = torch.cuda.current_stream()
    whole = eng.gen_batch(p)  # the whole instance on every rank (generation is not timed)
    n = whole.n_votes
    lo = (n * rank // world) // 4 * 4
    hi = n if rank == world - 1 else (n * (rank + 1) // world) // 4 * 4
    batch = DeviceBatch(whole.instance[lo:hi], whole.round[lo:hi], whole.type[lo:hi],
                        whole.value[lo:hi], whole.validator[lo:hi],
                        torch.tensor([0, hi - lo], dtype=torch.int64, device=eng.device), n_votes=hi - lo)
    codes = torch.empty(max(hi - lo, 1), dtype=torch.uint8, device=eng.device)
    cfg = abi.config(w["mode"], w["flags"], w["max_rounds"])
    dedup = w["mode"] == abi.MODE_DEDUP
    src = batch
    if dedup:  # the carried tally reads the type column with the later duplicates masked
        tmask = torch.empty(max(hi - lo, 1), dtype=torch.uint8, device=eng.device)
        batch = dataclasses.replace(batch, type=tmask)

    segs = max(1, min(args.segments or w["segments"], max(1, (hi - lo) // 4)))
    off = torch.from_numpy(adist.segment_offsets(hi - lo, segs).view(np.int64)).to(eng.device)

    # pass A as one reduction (agnes_tally_partials), which keeps the votes' weights
    # for pass B (AGNES_FLAG_WEIGHTS_CACHED): the power table is gathered once
    wcol = torch.empty(max(hi - lo, 1), dtype=torch.int64, device=eng.device)

    def tc(one, o, counts):  # on the current stream: a graph capture's while capturing
        cached = one.flags & abi.FLAG_WEIGHTS_CACHED
        eng.tally_carried(one, dataclasses.replace(batch, offsets=o, weight=wcol if cached else None), codes, counts)

    def pa(one, o, counts):
        eng.tally_partials(one, dataclasses.replace(batch, offsets=o), counts, wcol)

    def step():
        if dedup:
            return adist.tally_one_instance_dedup(
                tc, lambda base, f: eng.dedup_first(cfg, src, base, f),
                lambda base, f: eng.dedup_mask(cfg, src, base, f, tmask),
                None, hi - lo, p.n_vals, cfg, segs,  # pass B writes REJECTED (FLAG_MASKED_REJECTED)
                eng.device, base=lo, offsets=off, fold=eng.fold_counts, partials=pa,
                dedup_first_mask=lambda base, f: eng.dedup_first_mask(cfg, src, base, f, tmask))
        return adist.tally_one_instance(tc, hi - lo, cfg, segs, eng.device, 0, None, offsets=off,
                                        fold=eng.fold_counts, partials=pa)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # (DEDUP: the masked duplicates are counted as invalid by the carried tally)
    if not dedup and eng.last_error_count() != 0:
        raise SystemExit("bench batch has invalid votes")
    # per-kernel times: one eager step with the engine's event timing
    eng.kernel_timing(True)
    step()
    torch.cuda.synchronize()
    ktimes = eng.kernel_times()
    eng.kernel_timing(False)
    # one GPU: the step is ~20 short launches (two tallies + the folds), so it is
    # captured once in a HIP graph and replayed; over ranks the all_gather stays eager
    run = step
    graph = world == 1
    if graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            step()
        run = g.replay
        run()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = adist.max_over_ranks(elapsed)
    if world > 1:
        dist.barrier()
    if rank == 0:
        kernels = {}
        for name, (launches, total) in ktimes.items():
            avg = total / max(launches, 1)
            bpv = C5_PASS_B_BYTES_PER_VOTE if name == "tally_wide" else KERNEL_BYTES_PER_VOTE.get(name, 0)
            ab = bpv * (hi - lo)
            kernels[name] = {"launches": launches, "avg_ms": avg, "algorithmic_bytes": ab,
                             "GBps": ab / (avg * 1e-3) / 1e9 if ab and avg > 0 else None}
        # the roofline's kernel: the dominant one among those that stream the votes
        # (the slice fold and the exchange work on per-slice records)
        streaming = [k for k in kernels if kernels[k]["algorithmic_bytes"]]
        dom = max(streaming, key=lambda k: kernels[k]["avg_ms"] * kernels[k]["launches"])
        dom_ms = kernels[dom]["avg_ms"]
        dom_bpv = kernels[dom]["algorithmic_bytes"] // max(hi - lo, 1)
        achieved = kernels[dom]["algorithmic_bytes"] / (dom_ms * 1e-3) / 1e9
        traffic = measured_traffic(args.config) if world == 1 else {}
        with_traffic(kernels, traffic)
        td = traffic.get(dom)
        out = {
            "metric": "votes_tallied_per_sec", "value": n * args.steps / elapsed, "unit": "votes/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": w["scaling"], "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (counter-based splitmix64 streams, agnes_gen.h; Zipf powers)",
            "config": {"workload": w["desc"], "config": args.config, "instances": 1,
                       "validators": p.n_vals, "votes_total": n, "votes_per_gpu_per_step": hi - lo,
                       "segments_per_gpu": segs, "mode": "DEDUP" if dedup else "REFERENCE",
                       "flags": w["flags"],
                       "parallelism": f"stream-sliced x{world} (" + ("one all_reduce(MIN) + " if dedup else "")
                                      + "one all_gather per step)",
                       "hip_graph": graph},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": td.get("traffic_bytes") if td else None,
                         "traffic_source": td.get("sources") if td else None,
                         "kernel": KERNEL_SYMBOLS.get(dom, dom), "kernel_avg_ms": dom_ms,
                         "bytes_per_vote": dom_bpv,
                         "algorithmic_bytes": kernels[dom]["algorithmic_bytes"],
                         "note": "pass A: one reduction (agnes_tally_partials, keeps the weights); "
                                 "pass B: the carried tally over the cached weights; latency-bound at 2e6 votes"},
            "kernels": kernels,
        }
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle_lib as ol  # test infrastructure: the CPU baseline leg only
            h = whole.to_host()
            hb = ol.HostBatch(h["instance"], h["round"], h["type"], h["value"], h["validator"],
                              h["offsets"].copy(), None)
            best = None
            for _ in range(3):
                t1 = time.perf_counter()
                want, _, _ = ol.tally(cfg, hb, power)
                dt = time.perf_counter() - t1
                best = dt if best is None else min(best, dt)
            out["cpu_baseline"] = {"value": n / best, "unit": "votes/s", "cores": 1, "kind": "port",
                                   "sample": f"the whole instance ({n} votes), oracle/agnes_oracle.c "
                                             "orc_tally (one instance: one thread), best of 3"}
            out["cpu_check_equal"] = bool(np.array_equal(codes[: hi - lo].cpu().numpy(), want[lo:hi]))
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()



def openssl_verifier():
    """Ed25519 verification by the host's OpenSSL 3 libcrypto (EVP_DigestVerify) over
    ctypes: the CPU baseline of the wire config (ctypes releases the GIL, so one
    Python thread per CPU verifies in parallel)."""
    import ctypes as C
    import ctypes.util
    name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
    lc = C.CDLL(name)
    lc.EVP_PKEY_new_raw_public_key.restype = C.c_void_p
    lc.EVP_PKEY_new_raw_public_key.argtypes = [C.c_int, C.c_void_p, C.c_char_p, C.c_size_t]
    lc.EVP_MD_CTX_new.restype = C.c_void_p
    lc.EVP_MD_CTX_free.argtypes = [C.c_void_p]
    lc.EVP_MD_CTX_reset.argtypes = [C.c_void_p]
    lc.EVP_DigestVerifyInit.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    lc.EVP_DigestVerify.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
    lc.EVP_PKEY_free.argtypes = [C.c_void_p]
    EVP_PKEY_ED25519 = 1087

    def verify_many(items):
        ctx = lc.EVP_MD_CTX_new()
        keys = {}
        out = []
        for pub, msg, sig in items:
            k = keys.get(pub)
            if k is None:
                k = keys[pub] = lc.EVP_PKEY_new_raw_public_key(EVP_PKEY_ED25519, None, pub, 32)
            lc.EVP_MD_CTX_reset(ctx)  # a one-shot Ed25519 verify finalizes the context
            lc.EVP_DigestVerifyInit(ctx, None, None, None, k)
            out.append(lc.EVP_DigestVerify(ctx, sig, 64, msg, len(msg)) == 1)
        for k in keys.values():
            lc.EVP_PKEY_free(k)
        lc.EVP_MD_CTX_free(ctx)
        return out
    return verify_many, name


def bench_wire(args, w, eng, rank, world):
    """--config wire: agnes_wire_ingest over 2^20 signed records per
    GPU (weak scaling), records resident in HBM; value = records verified and decoded
    per second over all ranks."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "wire_ed25519.json")))
    recs = [bytes.fromhex(r) for r in g["records"]]
    pubs = b"".join(bytes.fromhex(p) for p in g["pubkeys"])
    n = w["records"]
    reps = (n + len(recs) - 1) // len(recs)
    host = np.frombuffer(b"".join(recs) * reps, dtype=np.uint8).reshape(-1, abi.WIRE_BYTES)[:n].copy()
    dev = eng.device
    rt = torch.from_numpy(host).to(dev)
    kt = torch.from_numpy(np.frombuffer(pubs, dtype=np.uint8).copy()).to(dev)
    offsets = torch.tensor([0, n], dtype=torch.int64, device=dev)

    def step():
        return eng.wire_ingest(rt, kt, 1, g["n_vals"], g["height"], 4, offsets)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    eng.kernel_timing(True)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ktimes = eng.kernel_times()
    eng.kernel_timing(False)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b, verdict = step()
    torch.cuda.synchronize()
    elapsed = adist.max_over_ranks(time.perf_counter() - t0)
    total = adist.sum_over_ranks(n)
    if rank == 0:
        launches, tot = ktimes["wire_ingest"]
        avg = tot / max(launches, 1)
        v = verdict.cpu().numpy()
        want_ok = np.tile(np.array(g["openssl_verifies"], dtype=bool), reps)[:n]
        ab = 151 * n  # record 104 + key 32 in, 14-B columns + verdict out
        out = {
            "metric": "wire_records_verified_per_sec", "value": total * args.steps / elapsed,
            "unit": "records/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32/int64 (GF(2^255-19) limbs)",
            "data": "OpenSSL-signed fixture records (tests/golden/wire_ed25519.json) replicated",
            "config": {"workload": w["desc"], "config": "wire", "records_per_gpu": n},
            "roofline": {"bound": "hbm", "achieved": ab / (avg * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": ab / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "agnes::wire::ingest_kernel", "kernel_avg_ms": avg,
                         "note": "VALU bound (one Ed25519 verification per lane, ~4k field products); "
                                 "the HBM fraction is reported only for the contract"},
            "gpu_verdicts_equal_openssl": bool(np.array_equal(v == abi.WIRE_OK, want_ok)),
        }
        if not args.no_cpu_baseline:
            # the host's OpenSSL Ed25519 verify rate over every CPU the cgroup grants
            # (`openssl speed -multi`: one process per CPU, OpenSSL's own timing loop),
            # and OpenSSL's verdicts on the fixture records through libcrypto (check)
            import subprocess
            cpu = host_cpu()
            procs = cpu_threads(cpu)
            rate = None
            try:
                r = subprocess.run(["openssl", "speed", "-seconds", "3", "-multi", str(procs), "ed25519"],
                                   capture_output=True, text=True, timeout=120)
                for line in r.stdout.splitlines():
                    if "Ed25519" in line:
                        rate = float(line.split()[-1])
            except (OSError, subprocess.SubprocessError, ValueError):
                rate = None
            verify_many, libname = openssl_verifier()
            items = [(bytes.fromhex(g["pubkeys"][struct.unpack_from("<I", r_, 24)[0]]), r_[:40], r_[40:])
                     for r_ in recs]
            out["cpu_check_equal"] = verify_many(items) == list(map(bool, g["openssl_verifies"]))
            if rate is not None:
                out["cpu_baseline"] = {"value": rate, "unit": "records/s", "cores": procs, "kind": "port",
                                       "host": cpu,
                                       "sample": f"`openssl speed -seconds 3 -multi {procs} ed25519` verify/s "
                                                 "(OpenSSL 3's Ed25519 verification, one process per granted "
                                                 "CPU; an independent implementation: the reference verifies "
                                                 "nothing)"}
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
