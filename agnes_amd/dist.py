"""Multi-GPU sharding of the tally path: one process per GPU (torch.distributed;
backend "nccl" is RCCL over xGMI on ROCm, "gloo" for CPU tests).

Instances are independent (one executor set + State per instance), so a batch
shards into contiguous instance ranges with NO collective on the data path.
Collectives are used only for
  * the bench's max-over-ranks timing and vote totals (all_reduce), and
  * gathering edge-triggered decision summaries (all_gather of a few bytes per
    decided instance) — never the level-triggered per-vote stream.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import abi


def env() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    import os
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) slice of n instances for `rank`."""
    return n * rank // world, n * (rank + 1) // world


@dataclass
class Shard:
    params: abi.GenParams   # generator parameters of this rank's batch
    base: int               # global id of the rank's instance 0
    n_total: int            # instances over all ranks


def make_shard(gen: dict, rank: int, world: int, strong: bool, seed: int = 0xA6E5) -> Shard:
    """strong: the configured instance count is split over ranks (same total work);
    weak: every rank gets the configured count (work grows with ranks).  Global
    instance ids keep the streams identical to one big batch either way."""
    g = dict(gen)
    n = g["n_instances"]
    if strong:
        lo, hi = shard_range(n, rank, world)
        g["n_instances"], base, total = hi - lo, lo, n
    else:
        base, total = rank * n, n * world
    return Shard(abi.gen_params(seed=seed, instance_base=base, **g), base, total)


def set_of_instances(shard: Shard, n_sets: int) -> np.ndarray:
    """instance -> power set by GLOBAL id (instance mod n_sets), as u32."""
    return ((np.arange(shard.params.n_instances, dtype=np.int64) + shard.base) % n_sets).astype(np.uint32)


def _device_for(group=None) -> torch.device:
    backend = dist.get_backend(group)
    return torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")


def max_over_ranks(x: float, group=None) -> float:
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_device_for(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def sum_over_ranks(x: int, group=None) -> int:
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return x
    t = torch.tensor([x], dtype=torch.int64, device=_device_for(group))
    dist.all_reduce(t, group=group)
    return int(t.item())


DECISION_DTYPE = np.dtype([("instance", "<u4"), ("value", "<u4"), ("round", "<i8")])


def decisions(states: np.ndarray, base: int) -> np.ndarray:
    """Edge-triggered summary of a rank's batch: one record per decided instance
    (the Decision message, state_machine.rs:320-322, recorded in the State)."""
    idx = np.nonzero(states["decided"])[0]
    out = np.zeros(len(idx), DECISION_DTYPE)
    out["instance"] = idx + base
    out["value"] = states["decision_value"][idx]
    out["round"] = states["decision_round"][idx]
    return out


def gather_decisions(local: np.ndarray, group=None) -> np.ndarray:
    """all_gather of every rank's decision records (variable length), ordered by rank."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return local
    world = dist.get_world_size(group)
    dev = _device_for(group)
    n = torch.tensor([len(local)], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    counts = [int(c.item()) for c in ns]
    m = max(counts) if counts else 0
    rec = DECISION_DTYPE.itemsize
    buf = torch.zeros(m * rec, dtype=torch.uint8, device=dev)
    if len(local):
        buf[: len(local) * rec] = torch.from_numpy(local.view(np.uint8).copy()).to(dev)
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    parts = [bufs[r][: counts[r] * rec].cpu().numpy().view(DECISION_DTYPE) for r in range(world)]
    return np.concatenate(parts) if parts else local


def gather_edges(recs: torch.Tensor, group=None) -> list:
    """all_gather of every rank's edge records (agnes_edge, 16 B each; any device
    tensor whose rows are records), variable length: the counts first, then the
    records padded to the longest; returns the list of each rank's records (rows
    in rank order), on recs' device.  One rank: [recs]."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [recs]
    world = dist.get_world_size(group)
    if recs.is_cuda and dist.get_backend(group) != "nccl":  # gloo: host buffers
        return [p.to(recs.device) for p in gather_edges(recs.cpu(), group)]
    flat = recs.contiguous().view(torch.uint8).reshape(recs.shape[0], -1) if recs.numel() else \
        torch.zeros((0, 16), dtype=torch.uint8, device=recs.device)
    rec = flat.shape[1]
    n = torch.tensor([flat.shape[0]], dtype=torch.int64, device=recs.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    counts = [int(c.item()) for c in ns]
    m = max(counts)
    buf = torch.zeros((m, rec), dtype=torch.uint8, device=recs.device)
    buf[: flat.shape[0]] = flat
    bufs = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf, group=group)
    return [bufs[r][: counts[r]] for r in range(world)]


def gather_edges_timed(recs: torch.Tensor, group=None, reps: int = 3) -> dict:
    """gather_edges timed over ranks (best of reps, max over ranks): the bench's
    exchange step of emitted records, outside its timed region."""
    best = None
    for _ in range(reps):
        dist.barrier(group=group)
        if recs.is_cuda:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        parts = gather_edges(recs, group)
        if recs.is_cuda:
            torch.cuda.synchronize()
        dt = max_over_ranks(time.perf_counter() - t0, group)
        best = dt if best is None else min(best, dt)
    total = sum(int(p.shape[0]) for p in parts)
    nbytes = sum(int(p.numel()) for p in parts)
    return {"records": total, "bytes": nbytes, "ms": best * 1e3,
            "GBps": nbytes / best / 1e9 if best > 0 else None}


# ---------------------------------------------------------------------------
# C5: ONE instance split into contiguous stream slices — the
# path's one real exchange step.  is_quorum (round_votes.rs:31-33) needs the
# exact running sum at every vote, so a slice can only be tallied once the
# weights of every vote before it are known: each slice first computes its own
# partial VoteCounts, one all_gather of the K x 3 int64 slice totals gives every
# rank the sum of the ranks before it, and each slice is tallied again from its
# exact carry-in.

NIL = abi.NIL


def segment_offsets(n_votes: int, n_segments: int, align: int = 4) -> np.ndarray:
    """Boundaries (n_segments + 1, u64) of balanced contiguous slices of one
    instance's votes, multiples of `align` (a slice starts on a lane boundary)."""
    k = np.arange(n_segments + 1, dtype=np.int64)
    b = (k * n_votes // n_segments) // align * align
    b[-1] = n_votes
    return b.astype(np.uint64)


def fold_counts(w: torch.Tensor, lab: torch.Tensor):
    """Folds of consecutive VoteCount partials along dim 0 (slices in stream order):
    weights add (i64, wrapping like the reference's release build), the label is
    the last slice's that wrote a value (round_votes.rs:50-54; NIL = none).
    w int64 [S, K, 2], lab int64 [S, K] -> (exclusive w, exclusive lab, total w
    [K, 2], total lab [K])."""
    # the scans run along the innermost dimension ([K, S] layouts): torch's
    # outer-dimension scan kernels are an order of magnitude slower at S ~ 1e3
    S, K = w.shape[0], w.shape[1]
    wt = w.reshape(S, 2 * K).t().contiguous()                       # [2K, S]
    incl_t = torch.cumsum(wt, dim=1)
    excl = (incl_t - wt).t().reshape(S, K, 2)
    lt = lab.t().contiguous()                                        # [K, S]
    idx = torch.arange(S, device=w.device, dtype=torch.int64).view(1, S).expand_as(lt)
    last = torch.cummax(torch.where(lt != NIL, idx, torch.full_like(idx, -1)), dim=1).values
    prev = torch.cat([torch.full_like(last[:, :1], -1), last[:, :-1]], dim=1)

    def pick(at):
        g = torch.gather(lt, 1, at.clamp(min=0))
        return torch.where(at >= 0, g, torch.full_like(g, NIL))

    return excl, pick(prev).t(), incl_t[:, -1].reshape(K, 2), pick(last)[:, -1]


def tally_one_instance(tally_carried, n_votes: int, cfg: abi.Config, n_segments: int, device,
                       inst_id: int = 0, group=None, prior=None, offsets=None, fold=None, partials=None):
    """C5 driver.  This rank holds a contiguous slice (n_votes votes) of ONE
    instance's stream; ranks hold consecutive slices in rank order.  The slice is
    cut into n_segments segments (one wave each) and tallied twice:
      A. every segment from an empty executor -> its partial (value_w, nil_w,
         label) per (round, type), the label NIL when it wrote none;
      exchange: ONE all_gather of the slice totals (K x 3 int64 per rank; RCCL
         over xGMI, gloo in the CPU tests) -> the ranks before this one;
      B. every segment from its carry-in (prior, ranks before, segments before)
         -> per-vote codes identical to tallying the instance as one stream.
    tally_carried(cfg, offsets int64 [S + 1] on `device`, counts int64 [S, K, 3])
    runs agnes_tally_carried on the slice.  prior: the instance's (w [K, 2], label
    [K]) before this call (a stream continued across calls), None = RoundVotes::new.
    offsets: segment_offsets(n_votes, n_segments) already on `device` (lets a caller
    capture the whole step in a HIP graph).
    fold: Engine.fold_counts (agnes_fold_counts, HIP): the folds run as one kernel
    each on the device; None: torch ops (CPU tensors in the tests).
    partials(cfg, offsets, counts) (with fold): pass A as one reduction
    (agnes_tally_partials, which also keeps the votes' weights); pass B's cfg then
    carries FLAG_WEIGHTS_CACHED and tally_carried must hand it those weights.
    Returns the instance's (w, label) after every rank's votes."""
    K = 2 * cfg.max_rounds
    if offsets is None:
        S = max(1, min(n_segments, max(1, n_votes // 4)))
        off = torch.from_numpy(segment_offsets(n_votes, S).view(np.int64)).to(device)
    else:
        off = offsets
        S = off.numel() - 1
    one = abi.Config(cfg.mode, cfg.flags | abi.FLAG_ONE_INSTANCE, cfg.max_rounds, inst_id)
    if fold is not None:
        return _tally_one_instance_hip(tally_carried, fold, one, off, S, K, device, group, prior, partials)
    counts = torch.zeros((S, K, 3), dtype=torch.int64, device=device)
    counts[..., 2] = NIL
    tally_carried(one, off, counts)                                    # pass A
    ex_w, ex_lab, tot_w, tot_lab = fold_counts(counts[..., :2], counts[..., 2] & 0xFFFFFFFF)
    mine = torch.cat([tot_w, tot_lab.unsqueeze(-1)], dim=-1)           # [K, 3]
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        t = mine.to(_device_for(group))
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=group)                         # the exchange step
        ranks = torch.stack(parts).to(device)
    else:
        rank, ranks = 0, mine.unsqueeze(0)
    if prior is not None:
        pw, pl = prior
        pl = torch.where(pl == 0, torch.full_like(pl, NIL), pl)  # "no value yet" and label 0 fold alike
        ranks = torch.cat([torch.cat([pw, pl.unsqueeze(-1)], dim=-1).unsqueeze(0).to(device), ranks])
        rank += 1
    r_w, r_lab, fin_w, fin_lab = fold_counts(ranks[..., :2], ranks[..., 2])
    in_w = ex_w + r_w[rank].unsqueeze(0)
    in_lab = torch.where(ex_lab != NIL, ex_lab, r_lab[rank].unsqueeze(0).expand_as(ex_lab))
    in_lab = torch.where(in_lab == NIL, torch.zeros_like(in_lab), in_lab)  # VoteCount::new's label
    counts = torch.cat([in_w, in_lab.unsqueeze(-1)], dim=-1).contiguous()
    tally_carried(one, off, counts)                                    # pass B
    return fin_w, torch.where(fin_lab == NIL, torch.zeros_like(fin_lab), fin_lab)


def _tally_one_instance_hip(tally_carried, fold, one, off, S, K, device, group, prior, partials=None):
    """tally_one_instance with the folds as agnes_fold_counts launches (no torch
    kernels between the two carried passes on one GPU)."""
    counts = torch.empty((S, K, 3), dtype=torch.int64, device=device)
    one_b = one
    if partials is not None:
        partials(one, off, counts)                                     # pass A: one reduction
        one_b = abi.Config(one.mode, one.flags | abi.FLAG_WEIGHTS_CACHED, one.max_rounds, one.reserved)
    else:
        fold(counts, flags=abi.FOLD_RESET)                             # RoundVotes::new per slice
        tally_carried(one, off, counts)                                # pass A
    pr = None
    if prior is not None:
        pw, pl = prior
        pr = torch.cat([pw, pl.unsqueeze(-1)], dim=-1).to(device).contiguous()
    fin = torch.empty((K, 3), dtype=torch.int64, device=device)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        mine = torch.empty((K, 3), dtype=torch.int64, device=device)
        fold(counts, totals=mine)                                      # this slice's total
        t = mine.to(_device_for(group))
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=group)                         # the exchange step
        ranks = torch.stack(parts).to(device).contiguous()             # [world, K, 3]
        fold(ranks, carry=pr, totals=fin,                              # ranks before each rank
             flags=abi.FOLD_APPLY | abi.FOLD_CARRY_ZERO_NONE | abi.FOLD_TOTAL_ZERO_LABELS)
        fold(counts, carry=ranks[rank].contiguous(), flags=abi.FOLD_APPLY | abi.FOLD_ZERO_LABELS)
    else:
        fold(counts, carry=pr, totals=fin,
             flags=abi.FOLD_APPLY | abi.FOLD_ZERO_LABELS | abi.FOLD_CARRY_ZERO_NONE | abi.FOLD_TOTAL_ZERO_LABELS)
    tally_carried(one_b, off, counts)                                  # pass B
    return fin[:, :2], fin[:, 2]


INT64_MAX = (1 << 63) - 1


def new_one_sm_marks(device) -> torch.Tensor:
    """agnes_one_sm_* marks before a stream: no P1, no C, no valid candidate."""
    return torch.tensor([INT64_MAX, INT64_MAX, 0, 0], dtype=torch.int64, device=device)


def one_instance_states(sm_scan, sm_apply, sm_finish, marks: torch.Tensor, group=None):
    """C5 with the State machine: after tally_one_instance[_dedup] wrote this rank's
    slice codes, the instance's State and the votes' message nibbles
    (agnes_one_sm_*, include/agnes.h).  Without RoundSkip the vote events move the
    State only at P1 (first PolkaNil / PolkaValue at State.round in Prevote,
    state_machine.rs:197-198) and C (first PrecommitValue, :211):
      scan     every rank's first P1 / C candidates -> all_reduce MIN (2 int64);
      apply    message nibbles from each vote's position relative to P1 / C, the
               last valid candidate (:198, :202) and C's round -> all_reduce MAX;
      finish   the State, identical on every rank.
    sm_scan(marks) / sm_apply(marks) / sm_finish(marks) run this rank's passes."""
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    sm_scan(marks)
    if multi:
        t = marks[:2].to(_device_for(group))
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)        # exchange 1
        marks[:2].copy_(t.to(marks.device))
    sm_apply(marks)
    if multi:
        t = marks[2:].to(_device_for(group))
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)        # exchange 2
        marks[2:].copy_(t.to(marks.device))
    sm_finish(marks)
    return marks


def tally_one_instance_dedup(tally_carried, dedup_first, dedup_mask, dedup_reject, n_votes: int,
                             n_vals: int, cfg: abi.Config, n_segments: int, device, base: int = 0,
                             group=None, offsets=None, fold=None, partials=None, dedup_first_mask=None):
    """C5 in DEDUP mode ("DEDUP mode adds an all-reduce(min) on
    first_index").  A vote's slice cannot see whether an earlier slice (or rank)
    already counted its (round, type, validator), so the first vote of every key is
    found before the tally:
      dedup_first(base, first)  this rank's slice lowers first[key] to its global
                                vote indices (agnes_dedup_first; base = the index of
                                the slice's first vote in the whole stream);
      exchange: ONE all_reduce(MIN) of first (8 B per key: 16 MB at 1M validators,
                                one round) over RCCL, gloo in the CPU tests;
      dedup_mask(base, first)   the slice's type column with the later duplicates
                                masked (agnes_dedup_mask); tally_carried must read
                                THAT column: a masked vote counts as nothing;
      tally_one_instance        the REFERENCE split tally of the masked stream;
      dedup_reject()            the masked votes' codes -> REJECTED (None: the carried
                                tally writes REJECTED itself, FLAG_MASKED_REJECTED).
    The codes equal tallying the whole instance as one DEDUP stream (offsets: as
    tally_one_instance's, for a HIP-graph capture).  A stream
    continued across calls would also carry `first`; not offered here.
    The instance's id is cfg.reserved, for the DEDUP checks and for the carried
    tally alike (one source).  With one rank, dedup_first_mask(base, first) (the
    fused agnes_dedup_first_mask), when given, replaces the first / mask pair."""
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    if dedup_first_mask is not None and not multi:
        first = torch.empty((2 * cfg.max_rounds * n_vals,), dtype=torch.int64, device=device)  # written whole
        dedup_first_mask(base, first)
    else:
        first = torch.full((2 * cfg.max_rounds * n_vals,), INT64_MAX, dtype=torch.int64, device=device)
        dedup_first(base, first)
        if multi:
            t = first.to(_device_for(group))
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)         # the DEDUP exchange step
            first = t.to(device)
        dedup_mask(base, first)
    flags = cfg.flags | (abi.FLAG_MASKED_REJECTED if dedup_reject is None else 0)
    ref = abi.Config(abi.MODE_REFERENCE, flags, cfg.max_rounds, cfg.reserved)
    out = tally_one_instance(tally_carried, n_votes, ref, n_segments, device, cfg.reserved, group,
                             offsets=offsets, fold=fold, partials=partials)
    if dedup_reject is not None:
        dedup_reject()
    return out


__all__ = ["env", "shard_range", "Shard", "make_shard", "set_of_instances", "max_over_ranks",
           "sum_over_ranks", "decisions", "gather_decisions", "DECISION_DTYPE", "segment_offsets",
           "fold_counts", "tally_one_instance", "tally_one_instance_dedup", "INT64_MAX"]
