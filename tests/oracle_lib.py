"""ctypes binding of the CPU checker oracle/liboracle.so (test infrastructure).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline use this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass
from typing import Optional

import numpy as np

from agnes_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None


class OrcPower(C.Structure):
    _fields_ = [("power", C.c_void_p), ("totals", C.c_void_p), ("n_sets", C.c_uint32),
                ("n_vals", C.c_uint32)]


def build(force: bool = False) -> str:
    srcs = ["agnes_oracle.c", "agnes_oracle.h"]
    newest = max(os.path.getmtime(os.path.join(ORACLE_DIR, s)) for s in srcs)
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < newest:
        if os.path.exists(os.path.join(ORACLE_DIR, "agnes_oracle.c")):
            subprocess.run(["make", "-s", "-C", ORACLE_DIR, "liboracle.so"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.orc_is_quorum.argtypes = [C.c_int64, C.c_int64]
        L.orc_is_one_third.argtypes = [C.c_int64, C.c_int64]
        L.orc_ve_apply.argtypes = [P, C.POINTER(abi.Vote), C.c_int64, C.POINTER(C.c_uint32)]
        L.orc_ve_apply.restype = C.c_uint32
        L.orc_rv_new.argtypes = [P, C.c_int64, C.c_int64, C.c_int64]
        L.orc_rv_add.argtypes = [P, C.c_uint32, C.c_uint32, C.c_int64, C.POINTER(C.c_uint32)]
        L.orc_rv_add.restype = C.c_uint32
        L.orc_state_new.argtypes = [C.c_int64, P]
        L.orc_state_apply.argtypes = [P, C.c_int64, C.POINTER(abi.Event), C.c_uint32,
                                      C.POINTER(abi.Message)]
        L.orc_tally.argtypes = [C.POINTER(abi.Config), C.POINTER(abi.VoteBatch),
                                C.POINTER(OrcPower), P, P, C.POINTER(C.c_uint64)]
        L.orc_tally_mt.argtypes = [C.POINTER(abi.Config), C.POINTER(abi.VoteBatch),
                                   C.POINTER(OrcPower), P, P, C.POINTER(C.c_uint64), C.c_int]
        L.orc_tally_labels.argtypes = [C.POINTER(abi.Config), C.POINTER(abi.VoteBatch),
                                       C.POINTER(OrcPower), P, P, C.POINTER(C.c_uint64), P, C.c_int]
        L.orc_events.argtypes = [C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, P]
        L.orc_apply_events.argtypes = [P, C.c_uint32, P, P, P, C.c_uint32]
        L.orc_valset_build.argtypes = [P, C.c_uint32, P, P, C.c_uint64, C.c_uint32, P, P, P, P,
                                       C.POINTER(C.c_uint64)]
        L.orc_apply_msgs.argtypes = [C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), C.POINTER(OrcPower),
                                     P, P, P, P, P, C.POINTER(C.c_uint64)]
        L.orc_edges.argtypes = [C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P]
        L.orc_set_totals.argtypes = [P, C.c_uint32, C.c_uint32, P]
        L.orc_gen_instance_votes.argtypes = [C.POINTER(abi.GenParams), C.c_uint32]
        L.orc_gen_instance_votes.restype = C.c_uint64
        L.orc_gen_offsets.argtypes = [C.POINTER(abi.GenParams), P]
        L.orc_gen_votes.argtypes = [C.POINTER(abi.GenParams), P, P, P, P, P, P]
        L.orc_gen_power.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int64,
                                    C.c_int64, P]
        _lib = L
    return _lib


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


# ---------------------------------------------------------------- host batches


@dataclass
class HostBatch:
    instance: np.ndarray
    round: np.ndarray
    type: np.ndarray
    value: np.ndarray
    validator: np.ndarray
    offsets: np.ndarray
    instance_set: Optional[np.ndarray] = None
    weight: Optional[np.ndarray] = None

    @property
    def n_votes(self) -> int:
        return int(self.offsets[-1])

    @property
    def n_instances(self) -> int:
        return len(self.offsets) - 1

    def c(self) -> abi.VoteBatch:
        return abi.VoteBatch(_p(self.instance), _p(self.round), _p(self.type), _p(self.value),
                             _p(self.validator), _p(self.offsets), _p(self.instance_set),
                             _p(self.weight), self.n_votes, self.n_instances, 0)


def batch_from_lists(instance, round_, type_, value, validator, offsets, instance_set=None,
                     weight=None) -> HostBatch:
    return HostBatch(
        np.ascontiguousarray(instance, dtype=np.uint32),
        np.ascontiguousarray(round_, dtype=np.uint8),
        np.ascontiguousarray(type_, dtype=np.uint8),
        np.ascontiguousarray(value, dtype=np.uint32),
        np.ascontiguousarray(validator, dtype=np.uint32),
        np.ascontiguousarray(offsets, dtype=np.uint64),
        None if instance_set is None else np.ascontiguousarray(instance_set, dtype=np.uint32),
        None if weight is None else np.ascontiguousarray(weight, dtype=np.int64),
    )


def concat_batches(*bs: HostBatch) -> HostBatch:
    """One batch holding the given batches' instances in order (instance ids and
    offsets rebased; no instance_set / weight): e.g. an aligned generated batch followed
    by a ragged one, so one call holds both kinds of flow batch."""
    inst, off, base_i, base_v = [], [np.zeros(1, np.uint64)], 0, 0
    for b in bs:
        n = len(b.offsets) - 1
        inst.append(b.instance.astype(np.uint64) + base_i)
        off.append(b.offsets[1:].astype(np.uint64) + np.uint64(base_v))
        base_i += n
        base_v += int(b.offsets[-1])
    return batch_from_lists(np.concatenate(inst).astype(np.uint32), np.concatenate([b.round for b in bs]),
                            np.concatenate([b.type for b in bs]), np.concatenate([b.value for b in bs]),
                            np.concatenate([b.validator for b in bs]), np.concatenate(off))


def gen_offsets(p: abi.GenParams) -> np.ndarray:
    off = np.zeros(p.n_instances + 1, dtype=np.uint64)
    rc = lib().orc_gen_offsets(C.byref(p), _p(off))
    assert rc == 0, rc
    return off


def gen_batch(p: abi.GenParams) -> HostBatch:
    off = gen_offsets(p)
    n = int(off[-1])
    b = HostBatch(np.zeros(n, np.uint32), np.zeros(n, np.uint8), np.zeros(n, np.uint8),
                  np.zeros(n, np.uint32), np.zeros(n, np.uint32), off)
    rc = lib().orc_gen_votes(C.byref(p), _p(off), _p(b.instance), _p(b.round), _p(b.type),
                             _p(b.value), _p(b.validator))
    assert rc == 0, rc
    return b


def gen_power(seed, n_sets, n_vals, kind, lo, hi) -> np.ndarray:
    pw = np.zeros((n_sets, n_vals), dtype=np.int64)
    rc = lib().orc_gen_power(seed, n_sets, n_vals, kind, lo, hi, _p(pw))
    assert rc == 0, rc
    return pw


def set_totals(power: np.ndarray) -> np.ndarray:
    power = np.ascontiguousarray(power, dtype=np.int64)
    t = np.zeros(power.shape[0], dtype=np.int64)
    lib().orc_set_totals(_p(power), power.shape[0], power.shape[1], _p(t))
    return t


def tally(cfg: abi.Config, b: HostBatch, power: Optional[np.ndarray], totals=None, states=None,
          threads: int = 1):
    """Returns (codes, states_out, n_invalid)."""
    codes = np.zeros(b.n_votes, dtype=np.uint8)
    pw_struct = None
    if power is not None:
        power = np.ascontiguousarray(power, dtype=np.int64)
        if totals is None:
            totals = set_totals(power)
        totals = np.ascontiguousarray(totals, dtype=np.int64)
        pw_struct = OrcPower(_p(power), _p(totals), power.shape[0], power.shape[1])
    st = None if states is None else np.array(states, dtype=abi.STATE_DTYPE, copy=True)
    nbad = C.c_uint64(0)
    cb = b.c()
    pw_ref = C.byref(pw_struct) if pw_struct is not None else None
    if threads > 1:
        rc = lib().orc_tally_mt(C.byref(cfg), C.byref(cb), pw_ref, _p(codes), _p(st),
                                C.byref(nbad), threads)
    else:
        rc = lib().orc_tally(C.byref(cfg), C.byref(cb), pw_ref, _p(codes), _p(st), C.byref(nbad))
    if rc != 0:
        raise RuntimeError(f"orc_tally rc={rc}")
    return codes, st, int(nbad.value)


def events(cfg: abi.Config, b: HostBatch, power: Optional[np.ndarray], totals=None, states=None,
           threads: int = 1):
    """The tally with the Value each VoteExecutor event carries (orc_tally_labels),
    then the event stream (orc_events).  Returns (codes, states_out, n_invalid,
    offsets u64 [n+1], records abi.VOTE_EVENT_DTYPE)."""
    codes = np.zeros(b.n_votes, dtype=np.uint8)
    labels = np.zeros(max(b.n_votes, 1), dtype=np.uint32)
    pw_struct = None
    if power is not None:
        power = np.ascontiguousarray(power, dtype=np.int64)
        if totals is None:
            totals = set_totals(power)
        totals = np.ascontiguousarray(totals, dtype=np.int64)
        pw_struct = OrcPower(_p(power), _p(totals), power.shape[0], power.shape[1])
    st = None if states is None else np.array(states, dtype=abi.STATE_DTYPE, copy=True)
    nbad = C.c_uint64(0)
    cb = b.c()
    pw_ref = C.byref(pw_struct) if pw_struct is not None else None
    rc = lib().orc_tally_labels(C.byref(cfg), C.byref(cb), pw_ref, _p(codes), _p(st), C.byref(nbad),
                                _p(labels), max(1, threads))
    if rc != 0:
        raise RuntimeError(f"orc_tally_labels rc={rc}")
    offs = np.zeros(b.n_instances + 1, dtype=np.uint64)
    rc = lib().orc_events(C.byref(cfg), C.byref(cb), _p(codes), _p(labels), _p(offs), None)
    assert rc == 0, rc
    out = np.zeros(int(offs[-1]), dtype=abi.VOTE_EVENT_DTYPE)
    rc = lib().orc_events(C.byref(cfg), C.byref(cb), _p(codes), _p(labels), _p(offs),
                          _p(out) if len(out) else None)
    assert rc == 0, rc
    return codes, st, int(nbad.value), offs, out


def edges(cfg: abi.Config, b: HostBatch, codes: np.ndarray):
    """orc_edges: (offsets u64 [n+1], records abi.EDGE_DTYPE)."""
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    offs = np.zeros(b.n_instances + 1, dtype=np.uint64)
    cb = b.c()
    rc = lib().orc_edges(C.byref(cfg), C.byref(cb), _p(codes), _p(offs), None)
    assert rc == 0, rc
    out = np.zeros(int(offs[-1]), dtype=abi.EDGE_DTYPE)
    rc = lib().orc_edges(C.byref(cfg), C.byref(cb), _p(codes), _p(offs), _p(out) if len(out) else None)
    assert rc == 0, rc
    return offs, out


def apply_events(states: np.ndarray, ev_offsets: np.ndarray, events: np.ndarray, flags: int = 0):
    st = np.array(states, dtype=abi.STATE_DTYPE, copy=True)
    ev_offsets = np.ascontiguousarray(ev_offsets, dtype=np.uint64)
    events = np.ascontiguousarray(events, dtype=abi.EVENT_DTYPE)
    msgs = np.zeros(len(events), dtype=abi.MESSAGE_DTYPE)
    rc = lib().orc_apply_events(_p(st), len(st), _p(ev_offsets), _p(events), _p(msgs), flags)
    assert rc == 0, rc
    return st, msgs


def apply_msgs(cfg: abi.Config, b, kinds: np.ndarray, pol_round: Optional[np.ndarray],
               power: Optional[np.ndarray], states: np.ndarray, totals=None):
    """orc_apply_msgs over a message script (agnes_amd.script.Script or HostBatch +
    kinds): returns (codes, states_out, msgs abi.MESSAGE_DTYPE, n_invalid)."""
    n = b.n_votes
    codes = np.zeros(max(n, 1), dtype=np.uint8)
    msgs = np.zeros(max(n, 1), dtype=abi.MESSAGE_DTYPE)
    pw_struct = None
    if power is not None:
        power = np.ascontiguousarray(power, dtype=np.int64)
        totals = set_totals(power) if totals is None else np.ascontiguousarray(totals, dtype=np.int64)
        pw_struct = OrcPower(_p(power), _p(totals), power.shape[0], power.shape[1])
    st = np.array(states, dtype=abi.STATE_DTYPE, copy=True)
    kinds = np.ascontiguousarray(kinds, dtype=np.uint8)
    pol = None if pol_round is None else np.ascontiguousarray(pol_round, dtype=np.int32)
    cb = abi.VoteBatch(_p(b.instance), _p(b.round), _p(b.type), _p(b.value), _p(b.validator), _p(b.offsets),
                       _p(getattr(b, "instance_set", None)), _p(getattr(b, "weight", None)), n, b.n_instances, 0)
    nbad = C.c_uint64(0)
    rc = lib().orc_apply_msgs(C.byref(cfg), C.byref(cb), C.byref(pw_struct) if pw_struct is not None else None,
                              _p(kinds), _p(pol), _p(codes), _p(st), _p(msgs), C.byref(nbad))
    if rc != 0:
        raise RuntimeError(f"orc_apply_msgs rc={rc}")
    return codes[:n], st, msgs[:n], int(nbad.value)


def valset_build(addr: np.ndarray, power: np.ndarray, set_of: Optional[np.ndarray], n_sets: int):
    """orc_valset_build: (order u32 [m], set_offsets u64 [n_sets + 1], power_out i64 [m], totals i64)"""
    addr = np.ascontiguousarray(addr, dtype=np.uint8)
    n, L = addr.shape
    power = np.ascontiguousarray(power, dtype=np.int64)
    so = None if set_of is None else np.ascontiguousarray(set_of, dtype=np.uint32)
    order = np.zeros(max(n, 1), np.uint32)
    offs = np.zeros(n_sets + 1, np.uint64)
    pout = np.zeros(max(n, 1), np.int64)
    tot = np.zeros(n_sets, np.int64)
    m = C.c_uint64(0)
    rc = lib().orc_valset_build(_p(addr), L, _p(power), _p(so), n, n_sets, _p(order), _p(offs), _p(pout), _p(tot),
                                C.byref(m))
    assert rc == 0, rc
    k = m.value
    return order[:k], offs, pout[:k], tot


def state_apply(state: abi.StateRec, round_: int, ev: abi.Event, flags: int = 0):
    s = abi.StateRec()
    C.memmove(C.byref(s), C.byref(state), C.sizeof(s))
    m = abi.Message()
    has = lib().orc_state_apply(C.byref(s), round_, C.byref(ev), flags, C.byref(m))
    return s, (m if has else None)


def state_new(height: int) -> abi.StateRec:
    s = abi.StateRec()
    lib().orc_state_new(height, C.byref(s))
    return s


class RoundVotes:
    """ctypes handle on orc_round_votes (opaque storage, 64 bytes is enough)."""

    def __init__(self, height: int, round_: int, total: int):
        self.buf = C.create_string_buffer(128)
        lib().orc_rv_new(self.buf, height, round_, total)

    def add_vote(self, typ: int, value: int, weight: int):
        tv = C.c_uint32(0)
        th = lib().orc_rv_add(self.buf, typ, value, weight, C.byref(tv))
        return th, tv.value

    def ve_apply(self, typ: int, value: int, weight: int):
        v = abi.Vote(0, value, typ)
        ev = C.c_uint32(0)
        e = lib().orc_ve_apply(self.buf, C.byref(v), weight, C.byref(ev))
        return e, ev.value
