"""Multi-round consensus message scripts for agnes_apply_msgs (synthetic input).

A script is, per instance, the stream of messages one ConsensusExecutor sees over
a height (consensus_executor.rs:54-79): for every round r the executor's own
NewRound input (execute, :31-33; NewRoundProposer with the instance's value when
it proposes r), the round's Proposal (pol_round -1, an earlier round, or an
invalid one), TimeoutPropose, the prevotes of every validator (value, another
value, or nil), TimeoutPrevote, the precommits and TimeoutPrecommit.  Rounds
before the last carry nil-heavy precommits so that TimeoutPrecommit moves the
State to round r + 1 (round_skip, state_machine.rs:209); the last round is
value-heavy and usually decides (:211).  Within a round the messages arrive in a
random order that keeps the phases roughly ordered (prevotes mostly before
precommits); a fraction of votes arrive late, inside the next round's window, so
votes for an earlier round interleave with the next round's messages.  A small
fraction of votes carry an out-of-range validator and a few messages an unknown
kind (both INVALID).

Vectorised numpy: a fixed number of messages per (instance, round), sorted per
instance by a random arrival key.  Laid out as the engine's vote batch (SoA,
instance-contiguous) plus the kind and pol_round columns.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import abi

NIL = abi.NIL


@dataclass
class Script:
    instance: np.ndarray   # u32
    round: np.ndarray      # u8
    type: np.ndarray       # u8: vote type / timeout step
    value: np.ndarray      # u32 (NIL = None)
    validator: np.ndarray  # u32
    offsets: np.ndarray    # u64 [n_instances + 1]
    kinds: np.ndarray      # u8 abi.IN_*
    pol_round: np.ndarray  # i32
    instance_set = None
    weight = None

    @property
    def n_votes(self) -> int:
        return int(self.offsets[-1])

    @property
    def n_instances(self) -> int:
        return len(self.offsets) - 1


def gen_script(seed: int, n_instances: int, n_vals: int, rounds: int, *, n_labels: int = 3,
               nil_permille: int = 150, other_permille: int = 100, late_permille: int = 50,
               invalid_permille: int = 10, proposer_permille: int = 250) -> Script:
    """Messages of `rounds` rounds for n_instances executors over n_vals validators
    (power set: the engine's, instance % n_sets).  Per (instance, round): 1 NewRound,
    1 Proposal, 1 TimeoutPropose, n_vals prevotes, 1 TimeoutPrevote, n_vals
    precommits, 1 TimeoutPrecommit."""
    if not (1 <= rounds <= 16) or n_vals < 1 or n_instances < 0:
        raise ValueError("rounds in 1..16, n_vals >= 1")
    rng = np.random.default_rng(seed)
    V = n_vals
    M = 5 + 2 * V  # messages per (instance, round)
    N, R = n_instances, rounds
    shape = (N, R, M)
    # message slots of one round: 0 NewRound, 1 Proposal, 2 TimeoutPropose,
    # 3..3+V prevotes, 3+V TimeoutPrevote, 4+V..4+2V precommits, 4+2V TimeoutPrecommit
    slot = np.arange(M)
    is_pv = (slot >= 3) & (slot < 3 + V)
    is_pc = (slot >= 4 + V) & (slot < 4 + 2 * V)
    kind = np.full(M, abi.IN_VOTE, np.uint8)
    kind[0] = abi.IN_NEW_ROUND
    kind[1] = abi.IN_PROPOSAL
    kind[[2, 3 + V, 4 + 2 * V]] = abi.IN_TIMEOUT
    typ = np.zeros(M, np.uint8)
    typ[2] = abi.TIMEOUT_PROPOSE
    typ[3 + V] = abi.TIMEOUT_PREVOTE
    typ[4 + 2 * V] = abi.TIMEOUT_PRECOMMIT
    typ[is_pc] = abi.PRECOMMIT
    val_of_slot = np.zeros(M, np.uint32)
    val_of_slot[is_pv] = np.arange(V)
    val_of_slot[is_pc] = np.arange(V)

    kinds = np.broadcast_to(kind, shape).copy()
    types = np.broadcast_to(typ, shape).copy()
    validator = np.broadcast_to(val_of_slot, shape).copy()
    rnd = np.broadcast_to(np.arange(R, dtype=np.uint8)[None, :, None], shape).copy()

    # the round's proposed value (labels 1..n_labels) and another value
    prop = rng.integers(1, n_labels + 1, size=(N, R), dtype=np.uint32)
    other = (prop % np.uint32(n_labels)) + np.uint32(1)
    value = np.full(shape, NIL, np.uint32)
    proposer = rng.integers(0, 1000, size=(N, R)) < proposer_permille
    value[:, :, 0] = np.where(proposer, prop, NIL)
    value[:, :, 1] = prop
    u = rng.integers(0, 1000, size=shape)
    last = (np.arange(R) == R - 1)[None, :, None]
    # prevotes: nil / other / proposed value
    pv_val = np.where(u < nil_permille, NIL, np.where(u < nil_permille + other_permille, other[:, :, None],
                                                      prop[:, :, None]))
    # precommits: value-heavy in the last round, nil-heavy before it
    pc_nil = np.where(last, nil_permille, 1000 - nil_permille)
    pc_val = np.where(u < pc_nil, NIL, np.where(u < pc_nil + other_permille // 2, other[:, :, None],
                                                prop[:, :, None]))
    value = np.where(is_pv[None, None, :], pv_val, value)
    value = np.where(is_pc[None, None, :], pc_val, value).astype(np.uint32)

    # pol_round of the Proposal: -1 (70 %), an earlier round (20 %), the round itself (10 %, ignored)
    pu = rng.integers(0, 10, size=(N, R))
    r_of = np.arange(R)[None, :]
    earlier = np.where(r_of > 0, rng.integers(0, np.maximum(r_of, 1), size=(N, R)), -1)
    pol = np.where(pu < 7, -1, np.where(pu < 9, earlier, r_of)).astype(np.int32)
    pol_round = np.zeros(shape, np.int32)
    pol_round[:, :, 1] = pol

    # invalid votes: validator out of range; a few unknown kinds
    iv = rng.integers(0, 1000, size=shape)
    validator = np.where((iv < invalid_permille) & (is_pv | is_pc)[None, None, :], np.uint32(V), validator)
    kinds = np.where((iv >= 1000 - max(1, invalid_permille // 5)) & (slot == 2)[None, None, :], np.uint8(7),
                     kinds).astype(np.uint8)

    # arrival order: NewRound first, then the phases with overlap; some votes late
    phase = np.zeros(M)
    phase[1:3] = 0.1
    phase[is_pv] = 0.2
    phase[3 + V] = 0.55
    phase[is_pc] = 0.45
    phase[4 + 2 * V] = 0.9
    key = 2.0 * rnd + phase[None, None, :] + (slot > 0)[None, None, :] * rng.random(shape) * 0.5
    late = (rng.integers(0, 1000, size=shape) < late_permille) & (is_pv | is_pc)[None, None, :]
    key = np.where(late, key + 1.5, key)
    key[:, :, 0] = 2.0 * np.arange(R)[None, :]
    order = np.argsort(key.reshape(N, R * M), axis=1, kind="stable")

    def col(a):
        return np.take_along_axis(a.reshape(N, R * M), order, axis=1).reshape(-1)

    n_msgs = N * R * M
    return Script(
        instance=np.repeat(np.arange(N, dtype=np.uint32), R * M),
        round=col(rnd).astype(np.uint8),
        type=col(types).astype(np.uint8),
        value=col(value).astype(np.uint32),
        validator=col(validator).astype(np.uint32),
        offsets=np.arange(0, n_msgs + 1, R * M, dtype=np.uint64) if N else np.zeros(1, np.uint64),
        kinds=col(kinds).astype(np.uint8),
        pol_round=col(pol_round).astype(np.int32),
    )
