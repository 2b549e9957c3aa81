"""Loader of the HIP engine library agnes_amd/libagnes_amd.so (C ABI of include/agnes.h).

There is no fallback: if the library is missing or no GPU is visible, the
engine's compute calls fail with AgnesError.
"""
from __future__ import annotations

import ctypes as C
import os
import re

from . import abi

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "libagnes_amd.so")
HEADER = os.path.join(ROOT, "include", "agnes.h")

_STATUS = {abi.E_INVALID: "AGNES_E_INVALID", abi.E_UNSUPPORTED: "AGNES_E_UNSUPPORTED",
           abi.E_DEVICE: "AGNES_E_DEVICE", abi.E_NOMEM: "AGNES_E_NOMEM",
           abi.E_NODEVICE: "AGNES_E_NODEVICE"}


class AgnesError(RuntimeError):
    def __init__(self, where: str, rc: int):
        super().__init__(f"{where} failed: {_STATUS.get(rc, rc)}")
        self.rc = rc


def check(rc: int, where: str) -> int:
    if rc < 0:
        raise AgnesError(where, rc)
    return rc


def header_functions(path: str = HEADER):
    """Names of every function include/agnes.h declares."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b(agnes_[a-z0-9_]+)\s*\(", text)
    return sorted(set(n for n in names if not n.startswith("agnes_vote_batch")))


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise AgnesError(f"loading {LIB_PATH} (not built: run `python -c "
                         f"'import __graft_entry__ as g; g.build()'`)", abi.E_NODEVICE)
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    sig = {
        "agnes_abi_version": ([], C.c_uint32),
        "agnes_kernel_timing": ([C.c_int], C.c_int),
        "agnes_kernel_times": ([C.POINTER(abi.KernelTime), C.c_uint32, C.POINTER(C.c_uint32)], C.c_int),
        "agnes_ctx_create": ([C.c_int, C.POINTER(P)], C.c_int),
        "agnes_ctx_destroy": ([P], None),
        "agnes_ctx_device": ([P], C.c_int),
        "agnes_upload_power": ([P, P, C.c_uint32, C.c_uint32, P], C.c_int),
        "agnes_tally": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P], C.c_int),
        "agnes_tally_states": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, P], C.c_int),
        "agnes_tally_carried": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P], C.c_int),
        "agnes_tally_partials": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P], C.c_int),
        "agnes_last_error_count": ([P, C.POINTER(C.c_uint64)], C.c_int),
        "agnes_lds_bytes_per_wave": ([C.POINTER(abi.Config), C.c_uint32], C.c_int64),
        "agnes_apply_events": ([P, P, C.c_uint32, P, P, P, C.c_uint32, P], C.c_int),
        "agnes_one_sm_scan": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), C.c_uint64, P, P, P, P], C.c_int),
        "agnes_one_sm_apply": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), C.c_uint64, P, P, P, P], C.c_int),
        "agnes_one_sm_finish": ([P, P, P, P], C.c_int),
        "agnes_multi_create": ([P, C.c_uint32, P], C.c_int),
        "agnes_multi_destroy": ([P], None),
        "agnes_multi_upload_power": ([P, P, C.c_uint32, C.c_uint32, P], C.c_int),
        "agnes_multi_tally": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P], C.c_int),
        "agnes_multi_tally_one": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, C.c_uint32, P],
                                  C.c_int),
        "agnes_multi_exchange": ([P, C.c_uint32], C.c_int),
        "agnes_multi_test_corrupt": ([P, C.c_uint32], C.c_int),
        "agnes_multi_edge_offsets": ([P, C.POINTER(abi.Config), P], C.c_int),
        "agnes_multi_edges": ([P, C.POINTER(abi.Config), P, P], C.c_int),
        "agnes_valset_build": ([P, P, C.c_uint32, P, P, C.c_uint64, C.c_uint32, P, P, P, P, P,
                                C.POINTER(C.c_uint64), P], C.c_int),
        "agnes_valset_find": ([P, P, C.c_uint32, P, C.c_uint32, P, P, C.c_uint64, P, P], C.c_int),
        "agnes_wire_ingest": ([P, P, C.c_uint64, P, C.c_uint32, C.c_uint32, P, C.c_uint32, C.c_int64, C.c_uint32,
                               P, P, P, P, P, P, P], C.c_int),
        "agnes_apply_msgs": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, P, P, P], C.c_int),
        "agnes_edge_offsets": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P], C.c_int),
        "agnes_edges": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, C.c_uint64, P], C.c_int),
        "agnes_fold_counts": ([P, P, C.c_uint32, C.c_uint32, P, P, C.c_uint32, P], C.c_int),
        "agnes_event_offsets": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P], C.c_int),
        "agnes_events": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, C.c_uint64, P], C.c_int),
        "agnes_tally_events": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, P, P, P], C.c_int),
        "agnes_events_capacity": ([C.POINTER(abi.Config), C.POINTER(abi.VoteBatch)], C.c_uint64),
        "agnes_tally_records": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, P, P, P], C.c_int),
        "agnes_records_compact": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, P, C.c_uint64, P],
                                  C.c_int),
        "agnes_records_overflow": ([P, C.POINTER(C.c_uint64)], C.c_int),
        "agnes_tally_edges": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, P, P, P], C.c_int),
        "agnes_edges_compact": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), P, P, P, P, C.c_uint64, P],
                                C.c_int),
        "agnes_dedup_first": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), C.c_uint64, P, P], C.c_int),
        "agnes_dedup_mask": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), C.c_uint64, P, P, P],
                             C.c_int),
        "agnes_dedup_first_mask": ([P, C.POINTER(abi.Config), C.POINTER(abi.VoteBatch), C.c_uint64, P, P, P],
                                   C.c_int),
        "agnes_dedup_reject": ([P, P, C.c_uint64, P, P], C.c_int),
        "agnes_gen_instance_votes": ([C.POINTER(abi.GenParams), C.c_uint32], C.c_uint64),
        "agnes_gen_offsets": ([C.POINTER(abi.GenParams), P], C.c_int),
        "agnes_gen_votes_device": ([P, C.POINTER(abi.GenParams), P, C.c_uint64, P, P, P, P, P,
                                    P], C.c_int),
        "agnes_gen_power": ([C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int64,
                             C.c_int64, P], C.c_int),
        "agnes_ve_new": ([C.c_int64, C.c_int64], P),
        "agnes_ve_apply": ([P, C.POINTER(abi.Vote), C.c_int64, C.POINTER(abi.Event)], C.c_int),
        "agnes_ve_free": ([P], None),
        "agnes_state_init": ([C.c_int64, C.POINTER(abi.StateRec)], None),
        "agnes_state_apply": ([C.POINTER(abi.StateRec), C.c_int64, C.POINTER(abi.Event),
                               C.c_uint32, C.POINTER(abi.StateRec), C.POINTER(abi.Message)],
                              C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    if L.agnes_abi_version() != abi.ABI_VERSION:
        raise AgnesError("ABI version check", abi.E_INVALID)
    _lib = L
    return L
