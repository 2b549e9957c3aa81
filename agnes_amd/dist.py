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


__all__ = ["env", "shard_range", "Shard", "make_shard", "set_of_instances", "max_over_ranks",
           "sum_over_ranks", "decisions", "gather_decisions", "DECISION_DTYPE"]
