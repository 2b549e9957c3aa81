"""Batch engine: device residency (torch tensors as HIP allocations) + the C ABI.

The hot path is `Engine.tally`: one call tallies a whole batch of instances on
the GPU (agnes_tally).  PyTorch is only plumbing here — device memory,
streams, torch.distributed — never the compute.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import abi
from .lib import AgnesError, check, load


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream_handle(stream) -> C.c_void_p:
    if stream is None:
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream)


@dataclass
class DeviceBatch:
    """Canonical 14-byte SoA vote batch resident in HBM (include/agnes.h)."""

    instance: torch.Tensor   # int32 view of u32
    round: torch.Tensor      # uint8
    type: torch.Tensor       # uint8
    value: torch.Tensor      # int32 view of u32 (AGNES_NIL = -1)
    validator: torch.Tensor  # int32 view of u32
    offsets: torch.Tensor    # int64 view of u64, n_instances + 1
    instance_set: Optional[torch.Tensor] = None
    weight: Optional[torch.Tensor] = None  # int64
    n_votes: int = 0

    @property
    def n_instances(self) -> int:
        return self.offsets.numel() - 1

    @property
    def device(self) -> torch.device:
        return self.offsets.device

    def c(self) -> abi.VoteBatch:
        return abi.VoteBatch(self.instance.data_ptr(), self.round.data_ptr(),
                             self.type.data_ptr(), self.value.data_ptr(),
                             self.validator.data_ptr(), self.offsets.data_ptr(),
                             None if self.instance_set is None else self.instance_set.data_ptr(),
                             None if self.weight is None else self.weight.data_ptr(),
                             self.n_votes, self.n_instances, 0)

    @staticmethod
    def from_host(hb, device) -> "DeviceBatch":
        """hb: any object with numpy fields instance/round/type/value/validator/offsets."""
        def t(a, dt):
            return torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(device)
        return DeviceBatch(
            t(hb.instance, np.int32), t(hb.round, np.uint8), t(hb.type, np.uint8),
            t(hb.value, np.int32), t(hb.validator, np.int32), t(hb.offsets, np.int64),
            None if getattr(hb, "instance_set", None) is None else t(hb.instance_set, np.int32),
            None if getattr(hb, "weight", None) is None else t(hb.weight, np.int64),
            int(hb.offsets[-1]))

    def to_host(self) -> dict:
        def h(x, dt):
            return x.cpu().numpy().view(dt)
        return dict(instance=h(self.instance, np.uint32), round=h(self.round, np.uint8),
                    type=h(self.type, np.uint8), value=h(self.value, np.uint32),
                    validator=h(self.validator, np.uint32), offsets=h(self.offsets, np.uint64))


def states_to_device(states: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(states, dtype=abi.STATE_DTYPE).view(np.uint8)).to(device)


def states_to_host(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(abi.STATE_DTYPE).copy()


class Engine:
    """One context per GPU (agnes_ctx)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        self.device_index = device
        self.device = torch.device("cuda", device)
        h = C.c_void_p()
        check(self.lib.agnes_ctx_create(device, C.byref(h)), "agnes_ctx_create")
        self.ctx = h
        self.n_sets = 0
        self.n_vals = 0

    def close(self):
        if self.ctx:
            self.lib.agnes_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- residency ----------------------------------------------------------
    def upload_power(self, power: np.ndarray, totals: Optional[np.ndarray] = None):
        power = np.ascontiguousarray(power, dtype=np.int64)
        if power.ndim != 2:
            raise ValueError("power must be [n_sets][n_vals]")
        tot = None if totals is None else np.ascontiguousarray(totals, dtype=np.int64)
        check(self.lib.agnes_upload_power(self.ctx, power.ctypes.data, power.shape[0],
                                          power.shape[1], None if tot is None else tot.ctypes.data),
              "agnes_upload_power")
        self.n_sets, self.n_vals = power.shape

    # -- hot path -----------------------------------------------------------
    def tally(self, cfg: abi.Config, batch: DeviceBatch, codes: torch.Tensor,
              states: Optional[torch.Tensor] = None, stream=None):
        if codes.dtype != torch.uint8 or codes.numel() < batch.n_votes:
            raise ValueError("codes must be a uint8 tensor of n_votes")
        if states is not None and states.numel() < 64 * batch.n_instances:
            raise ValueError("states must hold n_instances 64-byte records")
        b = batch.c()
        check(self.lib.agnes_tally(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(states),
                                   _stream_handle(stream)), "agnes_tally")

    def tally_states(self, cfg: abi.Config, batch: DeviceBatch, codes: torch.Tensor,
                     states_in: torch.Tensor, states_out: torch.Tensor, stream=None):
        """agnes_tally_states: the States read from states_in, written to states_out."""
        if codes.dtype != torch.uint8 or codes.numel() < batch.n_votes:
            raise ValueError("codes must be a uint8 tensor of n_votes")
        for t in (states_in, states_out):
            if t.numel() < 64 * batch.n_instances:
                raise ValueError("states must hold n_instances 64-byte records")
        b = batch.c()
        check(self.lib.agnes_tally_states(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(states_in),
                                          _ptr(states_out), _stream_handle(stream)), "agnes_tally_states")

    def tally_events(self, cfg: abi.Config, batch: DeviceBatch, codes: torch.Tensor,
                     states_in: Optional[torch.Tensor] = None, states_out: Optional[torch.Tensor] = None,
                     offsets: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, stream=None):
        """agnes_tally_events: the tally (as tally_states) and its event stream in one call.
        offsets int64 [n_instances + 1] (offsets[-1] = the record count), out uint8
        [events_capacity(cfg, batch), 24]; both allocated when None.  Returns (offsets,
        out) without reading the count back (no sync)."""
        if codes.dtype != torch.uint8 or codes.numel() < batch.n_votes:
            raise ValueError("codes must be a uint8 tensor of n_votes")
        for t in (states_in, states_out):
            if t is not None and t.numel() < 64 * batch.n_instances:
                raise ValueError("states must hold n_instances 64-byte records")
        cap = self.events_capacity(cfg, batch)
        if offsets is None:
            offsets = torch.empty(batch.n_instances + 1, dtype=torch.int64, device=self.device)
        if out is None:
            out = torch.empty((max(cap, 1), 24), dtype=torch.uint8, device=self.device)
        if offsets.numel() < batch.n_instances + 1 or out.numel() < 24 * cap:
            raise ValueError("offsets must hold n_instances + 1, out events_capacity records")
        b = batch.c()
        check(self.lib.agnes_tally_events(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(states_in),
                                          _ptr(states_out), _ptr(offsets), _ptr(out), _stream_handle(stream)),
              "agnes_tally_events")
        return offsets, out

    def tally_records(self, cfg: abi.Config, batch: DeviceBatch, codes: torch.Tensor,
                      states_in: Optional[torch.Tensor] = None, states_out: Optional[torch.Tensor] = None,
                      counts: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, stream=None):
        """agnes_tally_records: the tally (as tally_states) and its records segmented by
        instance: counts int64 [n_instances], out uint8 [events_capacity, 16] (instance i's
        records at rows seg(i) .. seg(i) + counts[i], seg(i) = offsets[i], x2 with
        RoundSkip; view a host copy as abi.SEG_EVENT_DTYPE).  Allocated when None; no sync."""
        if codes.dtype != torch.uint8 or codes.numel() < batch.n_votes:
            raise ValueError("codes must be a uint8 tensor of n_votes")
        for t in (states_in, states_out):
            if t is not None and t.numel() < 64 * batch.n_instances:
                raise ValueError("states must hold n_instances 64-byte records")
        cap = self.events_capacity(cfg, batch)
        if counts is None:
            counts = torch.empty(max(batch.n_instances, 1), dtype=torch.int64, device=self.device)
        if out is None:
            out = torch.empty((max(cap, 1), 16), dtype=torch.uint8, device=self.device)
        if counts.numel() < batch.n_instances or out.numel() < 16 * cap:
            raise ValueError("counts must hold n_instances, out events_capacity records")
        b = batch.c()
        check(self.lib.agnes_tally_records(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(states_in),
                                           _ptr(states_out), _ptr(counts), _ptr(out), _stream_handle(stream)),
              "agnes_tally_records")
        return counts, out

    def records_compact(self, cfg: abi.Config, batch: DeviceBatch, counts: torch.Tensor, seg: torch.Tensor,
                        offsets: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, stream=None):
        """agnes_records_compact: offsets int64 [n_instances + 1] (the scan of counts) and the
        dense agnes_vote_event records (uint8 [events_capacity, 24]); allocated when None."""
        if offsets is None:
            offsets = torch.empty(batch.n_instances + 1, dtype=torch.int64, device=self.device)
        if out is None:
            out = torch.empty((max(self.events_capacity(cfg, batch), 1), 24), dtype=torch.uint8, device=self.device)
        b = batch.c()
        check(self.lib.agnes_records_compact(self.ctx, C.byref(cfg), C.byref(b), _ptr(counts), _ptr(seg),
                                             _ptr(offsets), _ptr(out), out.numel() // 24 if out is not None else 0,
                                             _stream_handle(stream)),
              "agnes_records_compact")
        return offsets, out

    def tally_edges(self, cfg: abi.Config, batch: DeviceBatch, codes: torch.Tensor,
                    states_in: Optional[torch.Tensor] = None, states_out: Optional[torch.Tensor] = None,
                    counts: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, stream=None):
        """agnes_tally_edges: the tally (as tally_states) and its edge summary segmented by
        instance: counts int64 [n_instances], out uint8 [n_votes, 16] (instance i's edges
        at rows offsets[i] .. offsets[i] + counts[i]; view a host copy as abi.EDGE_DTYPE).
        Allocated when None; no sync."""
        if codes.dtype != torch.uint8 or codes.numel() < batch.n_votes:
            raise ValueError("codes must be a uint8 tensor of n_votes")
        for t in (states_in, states_out):
            if t is not None and t.numel() < 64 * batch.n_instances:
                raise ValueError("states must hold n_instances 64-byte records")
        if counts is None:
            counts = torch.empty(max(batch.n_instances, 1), dtype=torch.int64, device=self.device)
        if out is None:
            out = torch.empty((max(batch.n_votes, 1), 16), dtype=torch.uint8, device=self.device)
        if counts.numel() < batch.n_instances or out.numel() < 16 * batch.n_votes:
            raise ValueError("counts must hold n_instances, out n_votes records")
        b = batch.c()
        check(self.lib.agnes_tally_edges(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(states_in),
                                         _ptr(states_out), _ptr(counts), _ptr(out), _stream_handle(stream)),
              "agnes_tally_edges")
        return counts, out

    def edges_compact(self, cfg: abi.Config, batch: DeviceBatch, counts: torch.Tensor, seg: torch.Tensor,
                      offsets: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, stream=None):
        """agnes_edges_compact: offsets int64 [n_instances + 1] and the dense agnes_edge
        records (uint8 [n_votes, 16]); allocated when None."""
        if offsets is None:
            offsets = torch.empty(batch.n_instances + 1, dtype=torch.int64, device=self.device)
        if out is None:
            out = torch.empty((max(batch.n_votes, 1), 16), dtype=torch.uint8, device=self.device)
        b = batch.c()
        check(self.lib.agnes_edges_compact(self.ctx, C.byref(cfg), C.byref(b), _ptr(counts), _ptr(seg),
                                           _ptr(offsets), _ptr(out), out.numel() // 16 if out is not None else 0,
                                           _stream_handle(stream)), "agnes_edges_compact")
        return offsets, out

    def records_overflow(self) -> int:
        """agnes_records_overflow: records the dense writers dropped (past out's capacity or
        their segment's end) since the last query; 0 when every record fit (synchronises)."""
        n = C.c_uint64(0)
        rc = self.lib.agnes_records_overflow(self.ctx, C.byref(n))
        if rc not in (abi.OK, abi.E_OVERFLOW):
            check(rc, "agnes_records_overflow")
        return int(n.value)

    def events_capacity(self, cfg: abi.Config, batch: DeviceBatch) -> int:
        b = batch.c()
        return int(self.lib.agnes_events_capacity(C.byref(cfg), C.byref(b)))

    def tally_carried(self, cfg: abi.Config, batch: DeviceBatch, codes: torch.Tensor,
                      counts: torch.Tensor, stream=None):
        """agnes_tally_carried: counts = int64 tensor [n_instances, 2 * max_rounds, 3]
        (agnes_vote_count records: value_w, nil_w, value | reserved << 32), in/out."""
        if codes.dtype != torch.uint8 or codes.numel() < batch.n_votes:
            raise ValueError("codes must be a uint8 tensor of n_votes")
        if (counts.dtype != torch.int64 or not counts.is_contiguous()
                or counts.numel() < batch.n_instances * 2 * cfg.max_rounds * 3):
            raise ValueError("counts must be a contiguous int64 [n_instances, 2R, 3] tensor")
        b = batch.c()
        check(self.lib.agnes_tally_carried(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(counts),
                                           _stream_handle(stream)), "agnes_tally_carried")

    def tally_partials(self, cfg: abi.Config, batch: DeviceBatch, counts: torch.Tensor,
                       weights: Optional[torch.Tensor] = None, stream=None):
        """agnes_tally_partials (C5 pass A as one reduction): counts := int64 [n_instances,
        2 * max_rounds, 3] (each segment's VoteCounts from RoundVotes::new, label NIL when
        none); weights (int64 [n_votes] or None) := each vote's weight, 0 when not valid."""
        if (counts.dtype != torch.int64 or not counts.is_contiguous()
                or counts.numel() < batch.n_instances * 2 * cfg.max_rounds * 3):
            raise ValueError("counts must be a contiguous int64 [n_instances, 2R, 3] tensor")
        if weights is not None and (weights.dtype != torch.int64 or weights.numel() < batch.n_votes):
            raise ValueError("weights must be an int64 tensor of n_votes")
        b = batch.c()
        check(self.lib.agnes_tally_partials(self.ctx, C.byref(cfg), C.byref(b), _ptr(counts), _ptr(weights),
                                            _stream_handle(stream)), "agnes_tally_partials")

    def fold_counts(self, counts: torch.Tensor, carry: Optional[torch.Tensor] = None,
                    totals: Optional[torch.Tensor] = None, flags: int = 0, stream=None):
        """agnes_fold_counts on counts = contiguous int64 [S, K, 3] (agnes_vote_count
        records); carry / totals: int64 [K, 3] or None."""
        if counts.dtype != torch.int64 or not counts.is_contiguous() or counts.dim() != 3:
            raise ValueError("counts must be a contiguous int64 [S, K, 3] tensor")
        S, K = counts.shape[0], counts.shape[1]
        for t in (carry, totals):
            if t is not None and (t.dtype != torch.int64 or not t.is_contiguous() or t.numel() < 3 * K):
                raise ValueError("carry / totals must be contiguous int64 [K, 3] tensors")
        check(self.lib.agnes_fold_counts(self.ctx, _ptr(counts), S, K, _ptr(carry), _ptr(totals), flags,
                                         _stream_handle(stream)), "agnes_fold_counts")

    # -- wire format + Ed25519 ---------------------------
    def wire_ingest(self, records: torch.Tensor, pubkeys: torch.Tensor, n_sets: int, n_vals: int, height: int,
                    max_rounds: int, offsets: torch.Tensor, instance_set: Optional[torch.Tensor] = None,
                    stream=None):
        """agnes_wire_ingest: records uint8 [n, 104] (include/agnes.h agnes_wire_vote),
        pubkeys uint8 [n_sets * n_vals, 32] (the validators' keys, set-major).
        Returns (DeviceBatch over the decoded columns with the caller's instance
        offsets, verdict uint8 [n]); a record that failed has type 0xFF, so the tally
        codes it INVALID."""
        if records.dtype != torch.uint8 or records.dim() != 2 or records.shape[1] != abi.WIRE_BYTES \
                or not records.is_contiguous():
            raise ValueError("records must be a contiguous uint8 [n, 104] tensor")
        if pubkeys.dtype != torch.uint8 or not pubkeys.is_contiguous() or pubkeys.numel() < 32 * n_sets * n_vals:
            raise ValueError("pubkeys must be a contiguous uint8 tensor of n_sets * n_vals * 32 bytes")
        n = records.shape[0]
        dev = self.device
        cols = dict(instance=torch.empty(max(n, 4), dtype=torch.int32, device=dev),
                    round=torch.empty(max(n, 4), dtype=torch.uint8, device=dev),
                    type=torch.empty(max(n, 4), dtype=torch.uint8, device=dev),
                    value=torch.empty(max(n, 4), dtype=torch.int32, device=dev),
                    validator=torch.empty(max(n, 4), dtype=torch.int32, device=dev))
        verdict = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        n_inst = 0 if instance_set is None else instance_set.numel()
        check(self.lib.agnes_wire_ingest(self.ctx, _ptr(records), n, _ptr(pubkeys), n_sets, n_vals,
                                         _ptr(instance_set), n_inst, height, max_rounds,
                                         _ptr(cols["instance"]), _ptr(cols["round"]), _ptr(cols["type"]),
                                         _ptr(cols["value"]), _ptr(cols["validator"]), _ptr(verdict),
                                         _stream_handle(stream)), "agnes_wire_ingest")
        b = DeviceBatch(cols["instance"], cols["round"], cols["type"], cols["value"], cols["validator"],
                        offsets, instance_set, None, n)
        return b, verdict[:n]

    # -- validator sets ----------------------------------
    def valset_build(self, addr: torch.Tensor, power: torch.Tensor, set_of: Optional[torch.Tensor], n_sets: int,
                     stream=None):
        """agnes_valset_build: addr uint8 [n, L], power int64 [n], set_of int32 [n]
        or None.  Returns (order int32 [m], set_offsets int64 [n_sets + 1], power_out
        int64 [m], totals int64 [n_sets], addr_out uint8 [m, L])."""
        if addr.dtype != torch.uint8 or addr.dim() != 2 or not addr.is_contiguous():
            raise ValueError("addr must be a contiguous uint8 [n, addr_len] tensor")
        n, L = addr.shape
        if power.dtype != torch.int64 or power.numel() != n or (set_of is not None and set_of.numel() != n):
            raise ValueError("power int64 [n], set_of int32 [n]")
        dev = self.device
        order = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        offs = torch.empty(n_sets + 1, dtype=torch.int64, device=dev)
        pout = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
        tot = torch.empty(n_sets, dtype=torch.int64, device=dev)
        aout = torch.empty((max(n, 1), L), dtype=torch.uint8, device=dev)
        m = C.c_uint64(0)
        check(self.lib.agnes_valset_build(self.ctx, _ptr(addr), L, _ptr(power), _ptr(set_of), n, n_sets,
                                          _ptr(order), _ptr(offs), _ptr(pout), _ptr(tot), _ptr(aout), C.byref(m),
                                          _stream_handle(stream)), "agnes_valset_build")
        k = m.value
        return order[:k], offs, pout[:k], tot, aout[:k]

    def valset_find(self, sorted_addr: torch.Tensor, set_offsets: torch.Tensor, q_addr: torch.Tensor,
                    q_set: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """agnes_valset_find: int64 index per query (-1 when absent)."""
        n_q, L = q_addr.shape
        out = torch.empty(max(n_q, 1), dtype=torch.int64, device=self.device)
        check(self.lib.agnes_valset_find(self.ctx, _ptr(sorted_addr), L, _ptr(set_offsets), set_offsets.numel() - 1,
                                         _ptr(q_addr), _ptr(q_set), n_q, _ptr(out), _stream_handle(stream)),
              "agnes_valset_find")
        return out[:n_q]

    # -- the State machine of one instance split over slices (C5) -------------
    def _one_sm_check(self, batch, codes, state, marks):
        if codes.dtype != torch.uint8 or codes.numel() < batch.n_votes:
            raise ValueError("codes must be a uint8 tensor of n_votes")
        if state.numel() < 64 or marks.dtype != torch.int64 or marks.numel() < 4:
            raise ValueError("state must hold one 64-B agnes_state, marks int64 [4]")

    def one_sm_scan(self, cfg: abi.Config, batch: DeviceBatch, base: int, codes: torch.Tensor,
                    state: torch.Tensor, marks: torch.Tensor, stream=None):
        """agnes_one_sm_scan: lowers marks[0..1] to the slice's first P1 / C candidates."""
        self._one_sm_check(batch, codes, state, marks)
        b = batch.c()
        check(self.lib.agnes_one_sm_scan(self.ctx, C.byref(cfg), C.byref(b), base, _ptr(codes), _ptr(state),
                                         _ptr(marks), _stream_handle(stream)), "agnes_one_sm_scan")

    def one_sm_apply(self, cfg: abi.Config, batch: DeviceBatch, base: int, codes: torch.Tensor,
                     state: torch.Tensor, marks: torch.Tensor, stream=None):
        """agnes_one_sm_apply: message nibbles into codes; raises marks[2..3]."""
        self._one_sm_check(batch, codes, state, marks)
        b = batch.c()
        check(self.lib.agnes_one_sm_apply(self.ctx, C.byref(cfg), C.byref(b), base, _ptr(codes), _ptr(state),
                                          _ptr(marks), _stream_handle(stream)), "agnes_one_sm_apply")

    def one_sm_finish(self, marks: torch.Tensor, state: torch.Tensor, stream=None):
        """agnes_one_sm_finish: P1, the valid value and C applied to the State."""
        if state.numel() < 64 or marks.dtype != torch.int64 or marks.numel() < 4:
            raise ValueError("state must hold one 64-B agnes_state, marks int64 [4]")
        check(self.lib.agnes_one_sm_finish(self.ctx, _ptr(marks), _ptr(state), _stream_handle(stream)),
              "agnes_one_sm_finish")

    # -- DEDUP for one instance split over slices (C5) --------------------------
    def dedup_first(self, cfg: abi.Config, batch: DeviceBatch, base: int, first: torch.Tensor, stream=None):
        """agnes_dedup_first: first = int64 [2 * max_rounds * n_vals], INT64_MAX-initialised."""
        if first.dtype != torch.int64 or first.numel() < 2 * cfg.max_rounds * self.n_vals:
            raise ValueError("first must be an int64 [2 * max_rounds * n_vals] tensor")
        b = batch.c()
        check(self.lib.agnes_dedup_first(self.ctx, C.byref(cfg), C.byref(b), base, _ptr(first),
                                         _stream_handle(stream)), "agnes_dedup_first")

    def dedup_mask(self, cfg: abi.Config, batch: DeviceBatch, base: int, first: torch.Tensor,
                   type_out: torch.Tensor, stream=None):
        if type_out.dtype != torch.uint8 or type_out.numel() < batch.n_votes:
            raise ValueError("type_out must be a uint8 tensor of n_votes")
        b = batch.c()
        check(self.lib.agnes_dedup_mask(self.ctx, C.byref(cfg), C.byref(b), base, _ptr(first), _ptr(type_out),
                                        _stream_handle(stream)), "agnes_dedup_mask")

    def dedup_first_mask(self, cfg: abi.Config, batch: DeviceBatch, base: int, first: torch.Tensor,
                         type_out: torch.Tensor, stream=None):
        """agnes_dedup_first_mask: dedup_first + dedup_mask in one call, for a batch holding
        every vote of the instance (one rank)."""
        if first.dtype != torch.int64 or first.numel() < 2 * cfg.max_rounds * self.n_vals:
            raise ValueError("first must be an int64 [2 * max_rounds * n_vals] tensor")
        if type_out.dtype != torch.uint8 or type_out.numel() < batch.n_votes:
            raise ValueError("type_out must be a uint8 tensor of n_votes")
        b = batch.c()
        check(self.lib.agnes_dedup_first_mask(self.ctx, C.byref(cfg), C.byref(b), base, _ptr(first), _ptr(type_out),
                                              _stream_handle(stream)), "agnes_dedup_first_mask")

    def dedup_reject(self, type_masked: torch.Tensor, codes: torch.Tensor, n_votes: int, stream=None):
        check(self.lib.agnes_dedup_reject(self.ctx, _ptr(type_masked), n_votes, _ptr(codes),
                                          _stream_handle(stream)), "agnes_dedup_reject")

    def last_error_count(self) -> int:
        v = C.c_uint64(0)
        check(self.lib.agnes_last_error_count(self.ctx, C.byref(v)), "agnes_last_error_count")
        return int(v.value)

    # -- measurement ----------------------------------------------------------
    def kernel_timing(self, enable: bool):
        """Bracket every kernel the engine enqueues with HIP events (clears records)."""
        check(self.lib.agnes_kernel_timing(1 if enable else 0), "agnes_kernel_timing")

    def kernel_times(self) -> dict:
        """{kernel name: (launches, total ms)} of the launches since kernel_timing(True)."""
        cap = 16
        out = (abi.KernelTime * cap)()
        n = C.c_uint32(0)
        check(self.lib.agnes_kernel_times(out, cap, C.byref(n)), "agnes_kernel_times")
        return {out[i].name.decode(): (int(out[i].launches), float(out[i].total_ms))
                for i in range(min(n.value, cap))}

    def lds_bytes_per_wave(self, cfg: abi.Config) -> int:
        return int(self.lib.agnes_lds_bytes_per_wave(C.byref(cfg), self.n_vals))

    def apply_events(self, states: torch.Tensor, ev_offsets: torch.Tensor, events: torch.Tensor,
                     msgs: torch.Tensor, flags: int = 0, stream=None):
        n = ev_offsets.numel() - 1
        check(self.lib.agnes_apply_events(self.ctx, _ptr(states), n, _ptr(ev_offsets),
                                          _ptr(events), _ptr(msgs), flags,
                                          _stream_handle(stream)), "agnes_apply_events")

    def apply_msgs(self, cfg: abi.Config, batch: DeviceBatch, kinds: torch.Tensor, pol_round,
                   codes: torch.Tensor, states: torch.Tensor, msgs: torch.Tensor, stream=None):
        """Batched ConsensusExecutor::apply_msg (agnes_apply_msgs): kinds uint8
        [n_votes] (abi.IN_*), pol_round int32 [n_votes] or None, codes uint8
        [n_votes], states uint8 [n, 64] in place, msgs uint8 [n_votes, 24]."""
        n = batch.n_votes
        if kinds.dtype != torch.uint8 or kinds.numel() < n or codes.dtype != torch.uint8 or codes.numel() < n:
            raise ValueError("kinds and codes must be uint8 tensors of n_votes")
        if msgs.numel() < 24 * n or states.numel() < 64 * batch.n_instances:
            raise ValueError("msgs / states too small")
        if pol_round is not None and (pol_round.dtype != torch.int32 or pol_round.numel() < n):
            raise ValueError("pol_round must be an int32 tensor of n_votes")
        b = batch.c()
        check(self.lib.agnes_apply_msgs(self.ctx, C.byref(cfg), C.byref(b), _ptr(kinds),
                                        None if pol_round is None else _ptr(pol_round), _ptr(codes),
                                        _ptr(states), _ptr(msgs), _stream_handle(stream)),
              "agnes_apply_msgs")

    def edges(self, cfg: abi.Config, batch: DeviceBatch, codes: torch.Tensor, stream=None):
        """Edge-triggered summary of coded votes (agnes_edge_offsets + agnes_edges).
        Returns (offsets int64 [n_instances + 1], records uint8 [n_edges, 16] — view
        the host copy as abi.EDGE_DTYPE).  Reads the total back (one sync)."""
        if codes.dtype != torch.uint8 or codes.numel() < batch.n_votes:
            raise ValueError("codes must be a uint8 tensor of n_votes")
        b = batch.c()
        offs = torch.empty(batch.n_instances + 1, dtype=torch.int64, device=self.device)
        sh = _stream_handle(stream)
        check(self.lib.agnes_edge_offsets(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(offs), sh),
              "agnes_edge_offsets")
        if stream is not None:  # the total is read on torch's current stream
            stream.synchronize()
        n = int(offs[-1].item())
        out = torch.empty((max(n, 1), 16), dtype=torch.uint8, device=self.device)
        if n:
            check(self.lib.agnes_edges(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(offs),
                                       _ptr(out), n, sh), "agnes_edges")
        return offs, out[:n]

    def events(self, cfg: abi.Config, batch: DeviceBatch, codes: torch.Tensor, stream=None):
        """The event stream of coded votes (agnes_event_offsets + agnes_events).
        Returns (offsets int64 [n_instances + 1], records uint8 [n_events, 24] — view
        the host copy as abi.VOTE_EVENT_DTYPE).  Reads the total back (one sync)."""
        if codes.dtype != torch.uint8 or codes.numel() < batch.n_votes:
            raise ValueError("codes must be a uint8 tensor of n_votes")
        b = batch.c()
        offs = torch.empty(batch.n_instances + 1, dtype=torch.int64, device=self.device)
        sh = _stream_handle(stream)
        check(self.lib.agnes_event_offsets(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(offs), sh),
              "agnes_event_offsets")
        if stream is not None:  # the total is read on torch's current stream
            stream.synchronize()
        n = int(offs[-1].item())
        out = torch.empty((max(n, 1), 24), dtype=torch.uint8, device=self.device)
        if n:
            check(self.lib.agnes_events(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(offs),
                                        _ptr(out), n, sh), "agnes_events")
        return offs, out[:n]

    def events_into(self, cfg: abi.Config, batch: DeviceBatch, codes: torch.Tensor, offsets: torch.Tensor,
                    out: torch.Tensor, stream=None):
        """agnes_events with the caller's offsets and out (uint8 [cap, 24]): pass 2 alone, no
        sync -- the records past out's capacity or past an instance's end offset are
        dropped and counted (records_overflow)."""
        b = batch.c()
        check(self.lib.agnes_events(self.ctx, C.byref(cfg), C.byref(b), _ptr(codes), _ptr(offsets), _ptr(out),
                                    out.numel() // 24, _stream_handle(stream)), "agnes_events")

    # -- synthetic workloads ------------------------------------------------
    def gen_offsets(self, p: abi.GenParams) -> np.ndarray:
        off = np.zeros(p.n_instances + 1, dtype=np.uint64)
        check(self.lib.agnes_gen_offsets(C.byref(p), off.ctypes.data), "agnes_gen_offsets")
        return off

    def gen_batch(self, p: abi.GenParams, stream=None) -> DeviceBatch:
        off = self.gen_offsets(p)
        n = int(off[-1])
        dev = self.device
        b = DeviceBatch(
            torch.empty(n, dtype=torch.int32, device=dev),
            torch.empty(n, dtype=torch.uint8, device=dev),
            torch.empty(n, dtype=torch.uint8, device=dev),
            torch.empty(n, dtype=torch.int32, device=dev),
            torch.empty(n, dtype=torch.int32, device=dev),
            torch.from_numpy(off.view(np.int64)).to(dev), n_votes=n)
        check(self.lib.agnes_gen_votes_device(
            self.ctx, C.byref(p), _ptr(b.offsets), n, _ptr(b.instance), _ptr(b.round),
            _ptr(b.type), _ptr(b.value), _ptr(b.validator), _stream_handle(stream)),
            "agnes_gen_votes_device")
        return b

    def gen_power(self, seed: int, n_sets: int, n_vals: int, kind: int, lo: int,
                  hi: int) -> np.ndarray:
        pw = np.zeros((n_sets, n_vals), dtype=np.int64)
        check(self.lib.agnes_gen_power(seed, n_sets, n_vals, kind, lo, hi, pw.ctypes.data),
              "agnes_gen_power")
        return pw


__all__ = ["Engine", "DeviceBatch", "AgnesError", "states_to_device", "states_to_host"]
