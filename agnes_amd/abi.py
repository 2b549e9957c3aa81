"""ctypes mirror of include/agnes.h (structs, constants, numpy dtypes).

Pure declarations: importing this module loads no native code.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

ABI_VERSION = 8
NIL = 0xFFFFFFFF

OK, E_INVALID, E_UNSUPPORTED, E_DEVICE, E_NOMEM, E_NODEVICE, E_OVERFLOW = 0, -1, -2, -3, -4, -5, -6

PREVOTE, PRECOMMIT = 0, 1
THRESH_INIT, THRESH_ANY, THRESH_NIL, THRESH_VALUE = 0, 1, 2, 3
STEP_NEW_ROUND, STEP_PROPOSE, STEP_PREVOTE, STEP_PRECOMMIT, STEP_COMMIT = range(5)
(EV_NEW_ROUND, EV_NEW_ROUND_PROPOSER, EV_PROPOSAL, EV_PROPOSAL_INVALID, EV_POLKA_ANY,
 EV_POLKA_NIL, EV_POLKA_VALUE, EV_PRECOMMIT_ANY, EV_PRECOMMIT_VALUE, EV_ROUND_SKIP,
 EV_TIMEOUT_PROPOSE, EV_TIMEOUT_PREVOTE, EV_TIMEOUT_PRECOMMIT) = range(13)
EV_NONE = 0xFF
MSG_NONE, MSG_NEW_ROUND, MSG_PROPOSAL, MSG_VOTE, MSG_TIMEOUT, MSG_DECISION = range(6)
TIMEOUT_PROPOSE, TIMEOUT_PREVOTE, TIMEOUT_PRECOMMIT = range(3)
# agnes_apply_msgs message kinds (agnes.h AGNES_IN_*)
IN_VOTE, IN_PROPOSAL, IN_TIMEOUT, IN_NEW_ROUND = range(4)

CODE_NONE, CODE_POLKA_ANY, CODE_POLKA_NIL, CODE_POLKA_VALUE = 0, 1, 2, 3
CODE_PRECOMMIT_ANY, CODE_PRECOMMIT_VALUE, CODE_INVALID, CODE_REJECTED = 4, 5, 6, 7
CODE_EVENT_MASK, CODE_SKIP, CODE_MSG_SHIFT = 0x07, 0x08, 4
(VMSG_NONE, VMSG_TIMEOUT_PREVOTE, VMSG_TIMEOUT_PRECOMMIT, VMSG_PRECOMMIT_NIL,
 VMSG_PRECOMMIT_VALUE, VMSG_DECISION, VMSG_NEW_ROUND, VMSG_NEW_ROUND_TIMEOUT_PRECOMMIT,
 VMSG_NEW_ROUND_DECISION) = range(9)

MODE_REFERENCE, MODE_DEDUP = 0, 1
FLAG_ROUND_SKIP, FLAG_STATE_MACHINE, FLAG_DISTINCT_VALUES = 0x1, 0x2, 0x4
FLAG_ONE_INSTANCE = 0x8  # agnes_tally_carried: segments are slices of one instance (id cfg.reserved)
FLAG_WEIGHTS_CACHED = 0x10  # agnes_tally_carried: batch.weight = agnes_tally_partials' weights (validated as without)
TYPE_MASKED = 0xFE  # agnes_dedup_mask's type byte of a later duplicate (AGNES_TYPE_MASKED)
FLAG_MASKED_REJECTED = 0x20  # agnes_tally_carried: AGNES_TYPE_MASKED votes -> REJECTED in the pass (agnes_dedup_reject inside)
# route override (agnes.h AGNES_ROUTE_*): diagnostics / route-equivalence tests
ROUTE_SHIFT, ROUTE_AUTO, ROUTE_INSTANCE, ROUTE_SPLIT, ROUTE_WIDE = 8, 0, 1, 2, 3
EPOCH_BITS_SHIFT = 16


def FLAG_ROUTE(r: int) -> int:
    return (r & 3) << ROUTE_SHIFT




def FLAG_EPOCH_BITS(b: int) -> int:
    return (b & 0x1F) << EPOCH_BITS_SHIFT

ORDER_SHUFFLED, ORDER_PHASED, ORDER_SORTED = 0, 1, 2
POWER_UNIFORM, POWER_ZIPF, POWER_EQUAL = 0, 1, 2

EVENT_NAMES = ["NewRound", "NewRoundProposer", "Proposal", "ProposalInvalid", "PolkaAny",
               "PolkaNil", "PolkaValue", "PrecommitAny", "PrecommitValue", "RoundSkip",
               "TimeoutPropose", "TimeoutPrevote", "TimeoutPrecommit"]
STEP_NAMES = ["NewRound", "Propose", "Prevote", "Precommit", "Commit"]
MSG_NAMES = ["None", "NewRound", "Proposal", "Vote", "Timeout", "Decision"]
THRESH_NAMES = ["Init", "Any", "Nil", "Value"]


class Vote(C.Structure):
    _fields_ = [("round", C.c_int64), ("value", C.c_uint32), ("typ", C.c_uint8),
                ("pad", C.c_uint8 * 3)]


class Event(C.Structure):
    _fields_ = [("round", C.c_int64), ("pol_round", C.c_int64), ("value", C.c_uint32),
                ("kind", C.c_uint8), ("pad", C.c_uint8 * 3)]


class Message(C.Structure):
    _fields_ = [("round", C.c_int64), ("pol_round", C.c_int64), ("value", C.c_uint32),
                ("kind", C.c_uint8), ("vote_type", C.c_uint8), ("timeout_step", C.c_uint8),
                ("pad", C.c_uint8)]


class StateRec(C.Structure):
    _fields_ = [("height", C.c_int64), ("round", C.c_int64), ("locked_round", C.c_int64),
                ("valid_round", C.c_int64), ("decision_round", C.c_int64),
                ("locked_value", C.c_uint32), ("valid_value", C.c_uint32),
                ("decision_value", C.c_uint32), ("step", C.c_uint8),
                ("locked_present", C.c_uint8), ("valid_present", C.c_uint8),
                ("decided", C.c_uint8), ("pad", C.c_uint8 * 8)]


class KernelTime(C.Structure):
    """agnes_kernel_time (include/agnes.h): per-kernel launch count and total ms."""
    _fields_ = [("name", C.c_char * 40), ("launches", C.c_uint32), ("pad", C.c_uint32),
                ("total_ms", C.c_double)]


class Config(C.Structure):
    _fields_ = [("mode", C.c_uint32), ("flags", C.c_uint32), ("max_rounds", C.c_uint32),
                ("reserved", C.c_uint32)]


class VoteBatch(C.Structure):
    _fields_ = [("instance", C.c_void_p), ("round", C.c_void_p), ("type", C.c_void_p),
                ("value", C.c_void_p), ("validator", C.c_void_p), ("offsets", C.c_void_p),
                ("instance_set", C.c_void_p), ("weight", C.c_void_p),
                ("n_votes", C.c_uint64), ("n_instances", C.c_uint32), ("reserved", C.c_uint32)]


class GenParams(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_instances", C.c_uint32), ("n_vals", C.c_uint32),
                ("rounds_min", C.c_uint32), ("rounds_max", C.c_uint32),
                ("nil_permille", C.c_uint32), ("dup_permille", C.c_uint32),
                ("equiv_permille", C.c_uint32), ("higher_permille", C.c_uint32),
                ("order", C.c_uint32), ("instance_base", C.c_uint32),
                ("absent_permille", C.c_uint32), ("reserved", C.c_uint32)]


assert C.sizeof(Vote) == 16
assert C.sizeof(Event) == 24
assert C.sizeof(Message) == 24
assert C.sizeof(StateRec) == 64
assert C.sizeof(Config) == 16
assert C.sizeof(VoteBatch) == 80
assert C.sizeof(GenParams) == 56

# numpy views of the same records (for device<->host copies of state arrays)
STATE_DTYPE = np.dtype([
    ("height", "<i8"), ("round", "<i8"), ("locked_round", "<i8"), ("valid_round", "<i8"),
    ("decision_round", "<i8"), ("locked_value", "<u4"), ("valid_value", "<u4"),
    ("decision_value", "<u4"), ("step", "u1"), ("locked_present", "u1"),
    ("valid_present", "u1"), ("decided", "u1"), ("pad", "u1", (8,))])
EVENT_DTYPE = np.dtype([("round", "<i8"), ("pol_round", "<i8"), ("value", "<u4"),
                        ("kind", "u1"), ("pad", "u1", (3,))])
MESSAGE_DTYPE = np.dtype([("round", "<i8"), ("pol_round", "<i8"), ("value", "<u4"),
                          ("kind", "u1"), ("vote_type", "u1"), ("timeout_step", "u1"),
                          ("pad", "u1")])
# agnes_edge (include/agnes.h): one 16-B record per edge-triggered vote
EDGE_DTYPE = np.dtype([("vote", "<u8"), ("instance", "<u4"), ("round", "u1"), ("type", "u1"),
                       ("code", "u1"), ("prev", "u1")])
assert EDGE_DTYPE.itemsize == 16
FOLD_RESET, FOLD_APPLY, FOLD_CARRY_ZERO_NONE, FOLD_ZERO_LABELS, FOLD_TOTAL_ZERO_LABELS = 0x1, 0x2, 0x4, 0x8, 0x10
VOTE_EVENT_DTYPE = np.dtype([("vote", "<u8"), ("instance", "<u4"), ("value", "<u4"), ("round", "u1"),
                             ("kind", "u1"), ("message", "u1"), ("pad", "u1", (5,))])  # agnes_vote_event
assert VOTE_EVENT_DTYPE.itemsize == 24
SEG_EVENT_DTYPE = np.dtype([("vote", "<u8"), ("value", "<u4"), ("round", "u1"), ("kind", "u1"),
                            ("message", "u1"), ("pad", "u1")])  # agnes_seg_event
assert SEG_EVENT_DTYPE.itemsize == 16
# agnes_multi_exchange modes (include/agnes.h)
MULTI_EXCHANGE_AUTO, MULTI_EXCHANGE_HOST, MULTI_EXCHANGE_RCCL = 0, 1, 2
# agnes_multi_stats.exchange bits
MULTI_X_RCCL, MULTI_X_FALLBACK, MULTI_X_HOST = 1, 2, 4
VOTE_COUNT_DTYPE = np.dtype([("value_w", "<i8"), ("nil_w", "<i8"), ("value", "<u4"),
                             ("reserved", "<u4")])  # agnes_vote_count
MULTI_STATS_DTYPE = np.dtype([("device", "<u4"), ("i0", "<u4"), ("i1", "<u4"), ("exchange", "<u4"),
                              ("n_votes", "<u8"), ("n_invalid", "<u8"), ("h2d_ms", "<f8"), ("tally_ms", "<f8"),
                              ("d2h_ms", "<f8")])
assert STATE_DTYPE.itemsize == 64 and EVENT_DTYPE.itemsize == 24 and MESSAGE_DTYPE.itemsize == 24
assert VOTE_COUNT_DTYPE.itemsize == 24


def gen_params(seed=0xA6E5, n_instances=1, n_vals=4, rounds_min=1, rounds_max=1, nil_permille=0,
               dup_permille=0, equiv_permille=0, higher_permille=0, order=ORDER_SHUFFLED,
               instance_base=0, absent_permille=0) -> GenParams:
    return GenParams(seed, n_instances, n_vals, rounds_min, rounds_max, nil_permille,
                     dup_permille, equiv_permille, higher_permille, order, instance_base,
                     absent_permille, 0)


def config(mode=MODE_REFERENCE, flags=0, max_rounds=1, reserved=0) -> Config:
    return Config(mode, flags, max_rounds, reserved)


def new_states(n: int, height: int = 1, step: int = STEP_NEW_ROUND, round_: int = 0) -> np.ndarray:
    s = np.zeros(n, dtype=STATE_DTYPE)
    s["height"] = height
    s["round"] = round_
    s["step"] = step
    return s


# wire format (include/agnes.h agnes_wire_vote)
WIRE_BYTES = 104
WIRE_MAGIC = 0x31564741
WIRE_OK, WIRE_BAD_FORMAT, WIRE_BAD_VALIDATOR, WIRE_BAD_SIGNATURE, WIRE_BAD_HEIGHT = 0, 1, 2, 3, 4
