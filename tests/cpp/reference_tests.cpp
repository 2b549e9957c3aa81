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

// round_votes.rs:107-132
static void add_votes() {
    Value v{};
    std::optional<Value> val = v;
    int64_t total = 4;
    RoundVotes round_votes(1, 0, total);
    int64_t weight = 1;

    // add a vote. nothing changes.
    Vote vote = Vote::new_prevote(0, val);
    Thresh thresh = round_votes.add_vote(vote, weight);
    ASSERT_EQ(thresh, Thresh::Init());

    // add it again, nothing changes.
    thresh = round_votes.add_vote(vote, weight);
    ASSERT_EQ(thresh, Thresh::Init());

    // add a vote for nil, get Thresh::Any
    Vote vote_nil = Vote::new_prevote(0, std::nullopt);
    thresh = round_votes.add_vote(vote_nil, weight);
    ASSERT_EQ(thresh, Thresh::Any());

    // add vote for value, get Thresh::Value
    thresh = round_votes.add_vote(vote, weight);
    ASSERT_EQ(thresh, Thresh::Value_(v));
}

// state_machine.rs:331-345
static void happy_case() {
    Value val{};
    std::optional<Value> v = val;
    State s = State::new_(1);
    auto [s1, m1] = s.apply(0, Event::NewRoundProposer(val));
    ASSERT_EQ(*m1, Message::proposal_(0, val, -1));
    auto [s2, m2] = s1.apply(0, Event::Proposal(-1, val));
    ASSERT_EQ(*m2, Message::prevote(0, v));
    auto [s3, m3] = s2.apply(0, Event::PolkaValue(val));
    ASSERT_EQ(*m3, Message::precommit(0, v));
    auto [s4, m4] = s3.apply(0, Event::PrecommitValue(val));
    ASSERT_EQ(*m4, Message::decision_(0, val));
    ASSERT_EQ(s4.step(), Step::Commit);
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
