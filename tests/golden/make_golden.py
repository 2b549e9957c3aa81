"""Writes tests/golden/*.json.

reference_tests.json — the ONLY golden vectors the reference ships, transcribed
from its two unit tests' inputs and assert_eq! expectations, plus the C1
known-answer traces derived by hand from the cited code:

  round_votes::tests::add_votes     /root/reference/src/round_votes.rs:107-132
  state_machine::tests::happy_case  /root/reference/src/state_machine.rs:331-345

regress_small.json — small synthetic batches whose expected codes/states come
from the independent Python restatement (tests/pyref.py).  These pin the
engine's extensions (multi-round, DEDUP, RoundSkip, power weights) against
regressions; the reference has no test for them ("parity unpinned" beyond the
vectors above).

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import pyref  # noqa: E402

V = 7  # any label: Value is a ZST in the reference (lib.rs:3-4)


def reference_tests():
    return {
        "add_votes": {
            "source": "src/round_votes.rs:107-132",
            "total": 4, "weight": 1,
            # (type, value) — prevote(val) x2, prevote(nil), prevote(val)
            "votes": [[0, V], [0, V], [0, None], [0, V]],
            "thresh": ["Init", "Init", "Any", "Value"],
        },
        "happy_case": {
            "source": "src/state_machine.rs:331-345",
            "height": 1,
            "events": [
                {"round": 0, "kind": "NewRoundProposer", "value": V},
                {"round": 0, "kind": "Proposal", "pol_round": -1, "value": V},
                {"round": 0, "kind": "PolkaValue", "value": V},
                {"round": 0, "kind": "PrecommitValue", "value": V},
            ],
            "messages": [
                {"kind": "Proposal", "round": 0, "value": V, "pol_round": -1},
                {"kind": "Vote", "vote_type": "Prevote", "round": 0, "value": V},
                {"kind": "Vote", "vote_type": "Precommit", "round": 0, "value": V},
                {"kind": "Decision", "round": 0, "value": V},
            ],
            "final_step": "Commit",
        },
        # hand-derived from vote_executor.rs:26-36 + round_votes.rs:31-67, SURVEY.md §8(c)
        "c1_value": {
            "source": "derived: VoteExecutor::new(1,4), w=1",
            "total": 4, "weight": 1,
            "votes": [[0, V]] * 4 + [[1, V]] * 4,
            "events": [None, None, "PolkaValue", "PolkaValue", None, None, "PrecommitValue",
                       "PrecommitValue"],
            # composed with State::new(1) + NewRoundProposer(v) + Proposal(-1, v)
            # (consensus_executor.rs:61-69, state_machine.rs:198,202,205,211)
            "messages": [None, None, {"kind": "Vote", "vote_type": "Precommit", "round": 0,
                                      "value": V}, None, None, None,
                         {"kind": "Decision", "round": 0, "value": V}, None],
            "final_step": "Commit",
        },
        "c1_nil": {
            "source": "derived: vote_executor.rs:30,33",
            "total": 4, "weight": 1,
            "votes": [[0, None]] * 4 + [[1, None]] * 4,
            "events": [None, None, "PolkaNil", "PolkaNil", None, None, None, None],
        },
        "c1_mixed": {
            "source": "derived: round_votes.rs:62-63",
            "total": 4, "weight": 1,
            "votes": [[0, V], [0, None], [0, V], [0, None]],
            "events": [None, None, "PolkaAny", "PolkaAny"],
        },
    }


def regress_cases():
    """Small hand-shaped batches (pure Python generator, independent of agnes_gen.h)."""
    import random
    cases = []
    configs = [
        ("ref_single_round", pyref.MODE_REFERENCE, 0, 1, False),
        ("ref_multi_round_sm", pyref.MODE_REFERENCE, pyref.FLAG_STATE_MACHINE, 4, False),
        ("dedup_skip_sm", pyref.MODE_DEDUP,
         pyref.FLAG_STATE_MACHINE | pyref.FLAG_ROUND_SKIP, 5, True),
        ("ref_skip", pyref.MODE_REFERENCE, pyref.FLAG_ROUND_SKIP, 5, True),
    ]
    for ci, (name, mode, flags, max_rounds, adversarial) in enumerate(configs):
        rng = random.Random(1000 + ci)
        n_inst, n_vals, n_sets = 6, 7, 3
        power = [[rng.randint(1, 9) for _ in range(n_vals)] for _ in range(n_sets)]
        totals = [sum(p) for p in power]
        inst, rnd, typ, val, vidx, offs = [], [], [], [], [], [0]
        for i in range(n_inst):
            n_rounds = rng.randint(1, max(1, max_rounds - (1 if adversarial else 0)))
            for r in range(n_rounds):
                votes = [(r, t, v) for t in (0, 1) for v in range(n_vals)]
                if adversarial:
                    votes += [rng.choice(votes) for _ in range(4)]
                    votes += [(min(r + 1, max_rounds - 1), rng.randint(0, 1),
                               rng.randrange(n_vals)) for _ in range(3)]
                rng.shuffle(votes)
                for (rr, t, v) in votes:
                    inst.append(i)
                    rnd.append(rr)
                    typ.append(t)
                    vidx.append(v)
                    x = rng.random()
                    val.append(pyref.NIL if x < 0.25 else (100 + rr if x < 0.9 else 200 + rr))
            offs.append(len(rnd))
        # a few invalid votes
        if adversarial:
            vidx[3] = n_vals + 1
            rnd[5] = max_rounds
        states = None
        if flags & pyref.FLAG_STATE_MACHINE:
            states = []
            for i in range(n_inst):
                s = pyref.State(height=1)
                s, _ = pyref.apply(s, 0, pyref.EV_NEW_ROUND_PROPOSER, 100)
                s, _ = pyref.apply(s, 0, pyref.EV_PROPOSAL, 100, pol_round=-1)
                states.append(s)
        b = pyref.Batch(inst, rnd, typ, val, vidx, offs)
        codes, out_states = pyref.tally(b, power, totals, mode, flags, max_rounds, states)
        case = {
            "name": name, "mode": mode, "flags": flags, "max_rounds": max_rounds,
            "power": power, "totals": totals,
            "instance": inst, "round": rnd, "type": typ, "value": val, "validator": vidx,
            "offsets": offs, "codes": codes,
        }
        if states is not None:
            case["states_in"] = [state_json(s) for s in states]
            case["states_out"] = [state_json(s) for s in out_states]
        cases.append(case)
    return cases


def state_json(s):
    return {
        "height": s.height, "round": s.round, "step": s.step,
        "locked": list(s.locked) if s.locked else None,
        "valid": list(s.valid) if s.valid else None,
        "decision": list(s.decision) if s.decision else None,
    }


def main():
    with open(os.path.join(HERE, "reference_tests.json"), "w") as f:
        json.dump(reference_tests(), f, indent=1)
    with open(os.path.join(HERE, "regress_small.json"), "w") as f:
        json.dump(regress_cases(), f)
    print("wrote reference_tests.json, regress_small.json")


if __name__ == "__main__":
    main()
