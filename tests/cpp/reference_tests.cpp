// The reference's own unit tests, restated over the C++ mirror of its API
// (include/agnes.hpp) — every call runs on the GPU engine.
//
//   round_votes::tests::add_votes      /root/reference/src/round_votes.rs:107-132
//   state_machine::tests::happy_case   /root/reference/src/state_machine.rs:331-345
//
// plus the C1 VoteExecutor traces derived from vote_executor.rs:26-36.
#include <cstdio>
#include <cstdlib>

#include "agnes.hpp"

using namespace agnes;

static int failures = 0;
#define ASSERT_EQ(a, b)                                                      \
    do {                                                                     \
        if (!((a) == (b))) {                                                 \
            std::fprintf(stderr, "%s:%d: assert_eq!(%s, %s) failed\n",       \
                         __FILE__, __LINE__, #a, #b);                        \
            ++failures;                                                      \
        }                                                                    \
    } while (0)

// Golden vector of round_votes.rs:107-132: four unit-weight prevotes against a
// total of 4 give the threshold sequence Init, Init, Any, Value.
static void add_votes() {
    const Value label{};
    const std::optional<Value> some_label = label;
    RoundVotes counts(/*height*/ 1, /*round*/ 0, /*total*/ 4);
    const Vote for_label = Vote::new_prevote(0, some_label);
    const Vote for_nil = Vote::new_prevote(0, std::nullopt);
    const Thresh expected[4] = {Thresh::Init(), Thresh::Init(), Thresh::Any(), Thresh::Value_(label)};
    const Vote* sequence[4] = {&for_label, &for_label, &for_nil, &for_label};
    for (int k = 0; k < 4; ++k) ASSERT_EQ(counts.add_vote(*sequence[k], 1), expected[k]);
}

// Golden vector of state_machine.rs:331-345: one height through the four
// events of a proposer's round 0 ends in Commit with each expected message.
static void happy_case() {
    const Value label{};
    const std::optional<Value> some_label = label;
    const State start = State::new_(1);
    auto [proposed, msg_a] = start.apply(0, Event::NewRoundProposer(label));
    ASSERT_EQ(*msg_a, Message::proposal_(0, label, -1));
    auto [prevoted, msg_b] = proposed.apply(0, Event::Proposal(-1, label));
    ASSERT_EQ(*msg_b, Message::prevote(0, some_label));
    auto [precommitted, msg_c] = prevoted.apply(0, Event::PolkaValue(label));
    ASSERT_EQ(*msg_c, Message::precommit(0, some_label));
    auto [committed, msg_d] = precommitted.apply(0, Event::PrecommitValue(label));
    ASSERT_EQ(*msg_d, Message::decision_(0, label));
    ASSERT_EQ(committed.step(), Step::Commit);
}

// C1: VoteExecutor::new(1, 4), weight 1 — vote_executor.rs:26-36
static void c1_vote_executor() {
    Value val{7};
    VoteExecutor ve(1, 4);
    const EventKind pv = EventKind::PolkaValue, cv = EventKind::PrecommitValue;
    std::optional<EventKind> want[8] = {std::nullopt, std::nullopt, pv, pv,
                                        std::nullopt, std::nullopt, cv, cv};
    for (int k = 0; k < 8; ++k) {
        Vote vote = k < 4 ? Vote::new_prevote(0, val) : Vote::new_precommit(0, val);
        std::optional<Event> e = ve.apply(vote, 1);
        ASSERT_EQ(e.has_value(), want[k].has_value());
        if (e && want[k]) {
            ASSERT_EQ(e->kind, *want[k]);
            ASSERT_EQ(e->value, val);
        }
    }
    // precommit nil quorum produces no event (vote_executor.rs:33)
    VoteExecutor nil(1, 4);
    for (int k = 0; k < 4; ++k) ASSERT_EQ(nil.apply(Vote::new_precommit(0, std::nullopt), 1).has_value(), false);
}

int main() {
    try {
        add_votes();
        happy_case();
        c1_vote_executor();
    } catch (const Error& e) {
        std::fprintf(stderr, "engine error: %s\n", e.what());
        return 2;
    }
    if (failures) {
        std::fprintf(stderr, "%d assertion(s) failed\n", failures);
        return 1;
    }
    std::puts("reference tests: ok");
    return 0;
}
