"""Validator sets on the device: ValidatorSet::new / add /
update / remove (validators.rs:23-56, the intended behaviour -- the file does not
compile) over agnes_valset_build / agnes_valset_find.  A set is kept as its sorted,
deduplicated list; add, update and remove edit that list and rebuild, so every
state of a set is what ValidatorSet::sort (:49-55) leaves.  The built power rows
and totals feed agnes_upload_power (validator index = position in the set)."""
from __future__ import annotations

from typing import Optional

import torch


class ValidatorSets:
    def __init__(self, eng, addr: torch.Tensor, power: torch.Tensor, set_of: Optional[torch.Tensor], n_sets: int):
        """ValidatorSet::new (:28-31) for n_sets sets at once"""
        self.eng, self.n_sets = eng, n_sets
        self._build(addr, power, set_of)

    def _build(self, addr, power, set_of):
        set_of = set_of if set_of is not None else torch.zeros(addr.shape[0], dtype=torch.int32, device=addr.device)
        order, offs, pout, tot, aout = self.eng.valset_build(addr.contiguous(), power.contiguous(),
                                                             set_of.to(torch.int32).contiguous(), self.n_sets)
        self.addr, self.power, self.offsets, self.totals = aout, pout, offs, tot
        self.set_of = set_of.to(torch.int32)[order.long()]

    def find(self, addr: torch.Tensor, set_of: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.eng.valset_find(self.addr, self.offsets, addr.contiguous(),
                                    None if set_of is None else set_of.to(torch.int32).contiguous())

    def add(self, addr: torch.Tensor, power: torch.Tensor, set_of: Optional[torch.Tensor] = None):
        """ValidatorSet::add (:33-36): push, then sort (and dedup)"""
        s = set_of if set_of is not None else torch.zeros(addr.shape[0], dtype=torch.int32, device=addr.device)
        self._build(torch.cat([self.addr, addr]), torch.cat([self.power, power]),
                    torch.cat([self.set_of, s.to(torch.int32)]))

    def update(self, addr: torch.Tensor, power: torch.Tensor, set_of: Optional[torch.Tensor] = None):
        """ValidatorSet::update (:38-41): find the validator, set its voting power
        (the last update of a validator wins; an absent one is ignored)"""
        k = self.find(addr, set_of)
        hit = k >= 0
        p = self.power.clone()
        p[k[hit]] = power[hit]
        self._build(self.addr, p, self.set_of)

    def remove(self, addr: torch.Tensor, set_of: Optional[torch.Tensor] = None):
        """ValidatorSet::remove (:43-46): find the validator, drop it"""
        k = self.find(addr, set_of)
        keep = torch.ones(self.power.numel(), dtype=torch.bool, device=self.power.device)
        keep[k[k >= 0]] = False
        self._build(self.addr[keep], self.power[keep], self.set_of[keep])

    def power_table(self, n_vals: int) -> torch.Tensor:
        """[n_sets, n_vals] int64 rows (position in the set = validator index), zero
        past a set's end: the input of agnes_upload_power"""
        out = torch.zeros((self.n_sets, n_vals), dtype=torch.int64, device=self.power.device)
        offs = self.offsets.cpu().tolist()
        for s in range(self.n_sets):
            m = min(n_vals, offs[s + 1] - offs[s])
            out[s, :m] = self.power[offs[s]:offs[s] + m]
        return out
