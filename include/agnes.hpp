/*
 * agnes.hpp — C++ mirror of the reference's public Rust API for the vote path,
 * over the C ABI of agnes.h (every call runs on the GPU engine).
 *
 *   Rust (Liamsi/agnes)                          C++ here
 *   lib.rs:3-4      Value {}                     agnes::Value{id}      (label; ZST in Rust)
 *   lib.rs:15-39    VoteType, Vote::new_*        agnes::VoteType, agnes::Vote::new_prevote/new_precommit
 *   round_votes.rs:22-28  Thresh                 agnes::Thresh
 *   round_votes.rs:83,92  RoundVotes::new/add_vote  agnes::RoundVotes
 *   vote_executor.rs:13,20 VoteExecutor::new/apply  agnes::VoteExecutor
 *   state_machine.rs:14-163 Step/Event/Message/Timeout  agnes::Step/Event/Message/Timeout
 *   state_machine.rs:35,174 State::new/apply     agnes::State::new_/apply
 *
 * Error behaviour: the reference never fails; here the only failures are
 * engine failures (no GPU, device error), reported as agnes::Error.
 */
#ifndef AGNES_HPP
#define AGNES_HPP

#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>

#include "agnes.h"

namespace agnes {

class Error : public std::runtime_error {
  public:
    Error(const char* where, int rc)
        : std::runtime_error(std::string(where) + " failed: " + std::to_string(rc)), rc(rc) {}
    int rc;
};

inline int check(int rc, const char* where) {
    if (rc < 0) throw Error(where, rc);
    return rc;
}

struct Value {
    uint32_t id = 0;
    bool operator==(const Value& o) const { return id == o.id; }
    bool operator!=(const Value& o) const { return id != o.id; }
};

inline uint32_t to_raw(const std::optional<Value>& v) { return v ? v->id : AGNES_NIL; }
inline std::optional<Value> from_raw(uint32_t x) {
    return x == AGNES_NIL ? std::nullopt : std::optional<Value>(Value{x});
}

enum class VoteType : uint8_t { Prevote = AGNES_PREVOTE, Precommit = AGNES_PRECOMMIT };

struct Vote {
    VoteType typ = VoteType::Prevote;
    int64_t round = 0;
    std::optional<Value> value;
    static Vote new_prevote(int64_t round, std::optional<Value> value) {
        return Vote{VoteType::Prevote, round, value};
    }
    static Vote new_precommit(int64_t round, std::optional<Value> value) {
        return Vote{VoteType::Precommit, round, value};
    }
    bool operator==(const Vote& o) const {
        return typ == o.typ && round == o.round && value == o.value;
    }
    agnes_vote raw() const {
        agnes_vote v{};
        v.round = round;
        v.value = to_raw(value);
        v.typ = (uint8_t)typ;
        return v;
    }
};

enum class ThreshKind : uint32_t {
    Init = AGNES_THRESH_INIT,
    Any = AGNES_THRESH_ANY,
    Nil = AGNES_THRESH_NIL,
    Value = AGNES_THRESH_VALUE
};

struct Thresh {
    ThreshKind kind = ThreshKind::Init;
    agnes::Value value{};
    static Thresh Init() { return {ThreshKind::Init, {}}; }
    static Thresh Any() { return {ThreshKind::Any, {}}; }
    static Thresh Nil() { return {ThreshKind::Nil, {}}; }
    static Thresh Value_(agnes::Value v) { return {ThreshKind::Value, v}; }
    bool operator==(const Thresh& o) const {
        return kind == o.kind && (kind != ThreshKind::Value || value == o.value);
    }
};

/* RoundVotes (round_votes.rs:74-97): move-only handle on a GPU-resident tally */
class RoundVotes {
  public:
    RoundVotes(int64_t height, int64_t round, int64_t total) : h_(agnes_rv_new(height, round, total)) {
        if (!h_) throw Error("agnes_rv_new", AGNES_E_NODEVICE);
    }
    RoundVotes(RoundVotes&& o) noexcept : h_(std::exchange(o.h_, nullptr)) {}
    RoundVotes(const RoundVotes&) = delete;
    RoundVotes& operator=(const RoundVotes&) = delete;
    ~RoundVotes() { agnes_rv_free(h_); }
    Thresh add_vote(const Vote& vote, int64_t weight) {
        const agnes_vote v = vote.raw();
        uint32_t tv = 0;
        const int th = check(agnes_rv_add_vote(h_, &v, weight, &tv), "agnes_rv_add_vote");
        return Thresh{(ThreshKind)th, agnes::Value{tv}};
    }

  private:
    agnes_rv* h_;
};

enum class EventKind : uint8_t {
    NewRound = AGNES_EV_NEW_ROUND,
    NewRoundProposer = AGNES_EV_NEW_ROUND_PROPOSER,
    Proposal = AGNES_EV_PROPOSAL,
    ProposalInvalid = AGNES_EV_PROPOSAL_INVALID,
    PolkaAny = AGNES_EV_POLKA_ANY,
    PolkaNil = AGNES_EV_POLKA_NIL,
    PolkaValue = AGNES_EV_POLKA_VALUE,
    PrecommitAny = AGNES_EV_PRECOMMIT_ANY,
    PrecommitValue = AGNES_EV_PRECOMMIT_VALUE,
    RoundSkip = AGNES_EV_ROUND_SKIP,
    TimeoutPropose = AGNES_EV_TIMEOUT_PROPOSE,
    TimeoutPrevote = AGNES_EV_TIMEOUT_PREVOTE,
    TimeoutPrecommit = AGNES_EV_TIMEOUT_PRECOMMIT,
};

/* Event (state_machine.rs:96-110) */
struct Event {
    EventKind kind = EventKind::NewRound;
    int64_t pol_round = 0;   /* Proposal(pol_round, _) */
    agnes::Value value{};    /* NewRoundProposer / Proposal / PolkaValue / PrecommitValue */
    static Event NewRound() { return {EventKind::NewRound}; }
    static Event NewRoundProposer(agnes::Value v) { return {EventKind::NewRoundProposer, 0, v}; }
    static Event Proposal(int64_t pol_round, agnes::Value v) { return {EventKind::Proposal, pol_round, v}; }
    static Event ProposalInvalid() { return {EventKind::ProposalInvalid}; }
    static Event PolkaAny() { return {EventKind::PolkaAny}; }
    static Event PolkaNil() { return {EventKind::PolkaNil}; }
    static Event PolkaValue(agnes::Value v) { return {EventKind::PolkaValue, 0, v}; }
    static Event PrecommitAny() { return {EventKind::PrecommitAny}; }
    static Event PrecommitValue(agnes::Value v) { return {EventKind::PrecommitValue, 0, v}; }
    static Event RoundSkip() { return {EventKind::RoundSkip}; }
    static Event TimeoutPropose() { return {EventKind::TimeoutPropose}; }
    static Event TimeoutPrevote() { return {EventKind::TimeoutPrevote}; }
    static Event TimeoutPrecommit() { return {EventKind::TimeoutPrecommit}; }
    agnes_event raw(int64_t round) const {
        agnes_event e{};
        e.round = round;
        e.pol_round = pol_round;
        e.value = value.id;
        e.kind = (uint8_t)kind;
        return e;
    }
};

/* VoteExecutor (vote_executor.rs:8-36) */
class VoteExecutor {
  public:
    VoteExecutor(int64_t height, int64_t total_weight) : h_(agnes_ve_new(height, total_weight)) {
        if (!h_) throw Error("agnes_ve_new", AGNES_E_NODEVICE);
    }
    VoteExecutor(VoteExecutor&& o) noexcept : h_(std::exchange(o.h_, nullptr)) {}
    VoteExecutor(const VoteExecutor&) = delete;
    VoteExecutor& operator=(const VoteExecutor&) = delete;
    ~VoteExecutor() { agnes_ve_free(h_); }
    std::optional<Event> apply(const Vote& vote, int64_t weight) {
        const agnes_vote v = vote.raw();
        agnes_event e{};
        if (check(agnes_ve_apply(h_, &v, weight, &e), "agnes_ve_apply") == 0) return std::nullopt;
        return Event{(EventKind)e.kind, e.pol_round, agnes::Value{e.value}};
    }

  private:
    agnes_ve* h_;
};

enum class Step : uint8_t {
    NewRound = AGNES_STEP_NEW_ROUND,
    Propose = AGNES_STEP_PROPOSE,
    Prevote = AGNES_STEP_PREVOTE,
    Precommit = AGNES_STEP_PRECOMMIT,
    Commit = AGNES_STEP_COMMIT
};
enum class TimeoutStep : uint8_t {
    Propose = AGNES_TIMEOUT_PROPOSE,
    Prevote = AGNES_TIMEOUT_PREVOTE,
    Precommit = AGNES_TIMEOUT_PRECOMMIT
};

struct RoundValue {
    int64_t round = 0;
    agnes::Value value{};
    bool operator==(const RoundValue& o) const { return round == o.round && value == o.value; }
};
struct Timeout {
    int64_t round = 0;
    TimeoutStep step = TimeoutStep::Propose;
    bool operator==(const Timeout& o) const { return round == o.round && step == o.step; }
};
struct Proposal {
    int64_t round = 0;
    agnes::Value value{};
    int64_t pol_round = 0;
    bool operator==(const Proposal& o) const {
        return round == o.round && value == o.value && pol_round == o.pol_round;
    }
};

enum class MessageKind : uint8_t {
    NewRound = AGNES_MSG_NEW_ROUND,
    Proposal = AGNES_MSG_PROPOSAL,
    Vote = AGNES_MSG_VOTE,
    Timeout = AGNES_MSG_TIMEOUT,
    Decision = AGNES_MSG_DECISION
};

/* Message (state_machine.rs:118-148) */
struct Message {
    MessageKind kind = MessageKind::NewRound;
    int64_t round = 0;
    agnes::Proposal proposal{};
    agnes::Vote vote{};
    agnes::Timeout timeout{};
    RoundValue decision{};
    static Message new_round(int64_t r) { Message m; m.kind = MessageKind::NewRound; m.round = r; return m; }
    static Message proposal_(int64_t round, agnes::Value v, int64_t pol_round) {
        Message m;
        m.kind = MessageKind::Proposal;
        m.proposal = {round, v, pol_round};
        return m;
    }
    static Message prevote(int64_t round, std::optional<agnes::Value> v) {
        Message m;
        m.kind = MessageKind::Vote;
        m.vote = Vote::new_prevote(round, v);
        return m;
    }
    static Message precommit(int64_t round, std::optional<agnes::Value> v) {
        Message m;
        m.kind = MessageKind::Vote;
        m.vote = Vote::new_precommit(round, v);
        return m;
    }
    static Message timeout_(int64_t round, TimeoutStep s) {
        Message m;
        m.kind = MessageKind::Timeout;
        m.timeout = {round, s};
        return m;
    }
    static Message decision_(int64_t round, agnes::Value v) {
        Message m;
        m.kind = MessageKind::Decision;
        m.decision = {round, v};
        return m;
    }
    static Message from_raw(const agnes_message& r) {
        switch (r.kind) {
        case AGNES_MSG_NEW_ROUND: return new_round(r.round);
        case AGNES_MSG_PROPOSAL: return proposal_(r.round, agnes::Value{r.value}, r.pol_round);
        case AGNES_MSG_VOTE:
            return r.vote_type == AGNES_PREVOTE ? prevote(r.round, agnes::from_raw(r.value))
                                                : precommit(r.round, agnes::from_raw(r.value));
        case AGNES_MSG_TIMEOUT: return timeout_(r.round, (TimeoutStep)r.timeout_step);
        default: return decision_(r.round, agnes::Value{r.value});
        }
    }
    bool operator==(const Message& o) const {
        if (kind != o.kind) return false;
        switch (kind) {
        case MessageKind::NewRound: return round == o.round;
        case MessageKind::Proposal: return proposal == o.proposal;
        case MessageKind::Vote: return vote == o.vote;
        case MessageKind::Timeout: return timeout == o.timeout;
        default: return decision == o.decision;
        }
    }
};

/* State (state_machine.rs:24-31): Copy in Rust, a value type here */
struct State {
    agnes_state raw{};
    static State new_(int64_t height) { /* State::new, :35-43 */
        State s;
        agnes_state_init(height, &s.raw);
        return s;
    }
    int64_t height() const { return raw.height; }
    int64_t round() const { return raw.round; }
    Step step() const { return (Step)raw.step; }
    std::optional<RoundValue> locked() const {
        if (!raw.locked_present) return std::nullopt;
        return RoundValue{raw.locked_round, agnes::Value{raw.locked_value}};
    }
    std::optional<RoundValue> valid() const {
        if (!raw.valid_present) return std::nullopt;
        return RoundValue{raw.valid_round, agnes::Value{raw.valid_value}};
    }
    /* State::apply(self, round, event) -> (State, Option<Message>), :174 */
    std::pair<State, std::optional<Message>> apply(int64_t round, const Event& ev,
                                                   uint32_t flags = 0) const {
        const agnes_event e = ev.raw(round);
        State out;
        agnes_message m{};
        const int has = check(agnes_state_apply(&raw, round, &e, flags, &out.raw, &m), "agnes_state_apply");
        if (!has) return {out, std::nullopt};
        return {out, Message::from_raw(m)};
    }
};

} // namespace agnes

#endif
