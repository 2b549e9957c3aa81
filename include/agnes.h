/*
 * agnes.h — C ABI of the MI355X-native Agnes vote-tally engine.
 *
 * This header is the drop-in boundary for ONE hot path of Liamsi/agnes
 * (reference mounted read-only at /root/reference, Rust, GPL-3.0, clean-room):
 *
 *   ConsensusExecutor::apply_msg, Vote arm      src/consensus_executor.rs:61-69
 *     -> VoteExecutor::apply(vote, weight)       src/vote_executor.rs:20-23
 *        -> RoundVotes::add_vote                 src/round_votes.rs:92-97
 *           -> VoteCount::add_vote / is_quorum   src/round_votes.rs:31-33,48-67
 *        -> VoteExecutor::to_event               src/vote_executor.rs:26-36
 *     -> State::apply(round, event)              src/state_machine.rs:174-214
 *
 * batched one instance (height x validator-set x round set) per wave on the GPU.
 * Plain C: POD structs, pointers and sizes, integer status codes.  No torch,
 * no C++ types, nothing unwinds across the boundary.
 *
 * Integer semantics: every weight / total is int64 with two's-complement
 * WRAPPING arithmetic (the reference's release-build behaviour of i64 `+`/`*`,
 * round_votes.rs:32,52,55,62).  Results are bit-exact with the reference on
 * every input, including overflowing ones.
 */
#ifndef AGNES_H
#define AGNES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AGNES_ABI_VERSION 8u

/* ---------------------------------------------------------------------------
 * Status codes (reference never fails, state_machine.rs:212; these report
 * boundary misuse only).
 * ------------------------------------------------------------------------- */
#define AGNES_OK 0
#define AGNES_E_INVALID (-1)     /* bad argument / null pointer / size mismatch   */
#define AGNES_E_UNSUPPORTED (-2) /* configuration outside what the engine handles */
#define AGNES_E_DEVICE (-3)      /* HIP runtime error                            */
#define AGNES_E_NOMEM (-4)       /* allocation failed                            */
#define AGNES_E_NODEVICE (-5)    /* no GPU visible: the engine has NO CPU fallback */
#define AGNES_E_OVERFLOW (-6)    /* agnes_records_overflow: records that did not fit were dropped */

/* ---------------------------------------------------------------------------
 * Value / vote vocabulary (src/lib.rs:3-39)
 *
 * `Value` is a zero-sized struct in the reference (lib.rs:3-4).  Here it is a
 * 32-bit label `value_id`; `Option<Value>::None` (a nil vote) is AGNES_NIL.
 * ------------------------------------------------------------------------- */
#define AGNES_NIL 0xFFFFFFFFu

#define AGNES_PREVOTE 0u   /* VoteType::Prevote   lib.rs:17 */
#define AGNES_PRECOMMIT 1u /* VoteType::Precommit lib.rs:18 */

/* Thresh, round_votes.rs:22-28 */
#define AGNES_THRESH_INIT 0u
#define AGNES_THRESH_ANY 1u
#define AGNES_THRESH_NIL 2u
#define AGNES_THRESH_VALUE 3u

/* Step, state_machine.rs:14-21 */
#define AGNES_STEP_NEW_ROUND 0u
#define AGNES_STEP_PROPOSE 1u
#define AGNES_STEP_PREVOTE 2u
#define AGNES_STEP_PRECOMMIT 3u
#define AGNES_STEP_COMMIT 4u

/* Event, state_machine.rs:96-110 (same order as the Rust enum) */
#define AGNES_EV_NEW_ROUND 0u
#define AGNES_EV_NEW_ROUND_PROPOSER 1u
#define AGNES_EV_PROPOSAL 2u
#define AGNES_EV_PROPOSAL_INVALID 3u
#define AGNES_EV_POLKA_ANY 4u
#define AGNES_EV_POLKA_NIL 5u
#define AGNES_EV_POLKA_VALUE 6u
#define AGNES_EV_PRECOMMIT_ANY 7u
#define AGNES_EV_PRECOMMIT_VALUE 8u
#define AGNES_EV_ROUND_SKIP 9u
#define AGNES_EV_TIMEOUT_PROPOSE 10u
#define AGNES_EV_TIMEOUT_PREVOTE 11u
#define AGNES_EV_TIMEOUT_PRECOMMIT 12u
#define AGNES_EV_NONE 0xFFu /* Option<Event>::None */

/* Message, state_machine.rs:118-124 */
#define AGNES_MSG_NONE 0u
#define AGNES_MSG_NEW_ROUND 1u
#define AGNES_MSG_PROPOSAL 2u
#define AGNES_MSG_VOTE 3u
#define AGNES_MSG_TIMEOUT 4u
#define AGNES_MSG_DECISION 5u

/* TimeoutStep, state_machine.rs:159-163 */
#define AGNES_TIMEOUT_PROPOSE 0u
#define AGNES_TIMEOUT_PREVOTE 1u
#define AGNES_TIMEOUT_PRECOMMIT 2u

/* ---------------------------------------------------------------------------
 * POD mirrors of the reference types
 * ------------------------------------------------------------------------- */

/* Vote, lib.rs:22-27 (+ value label).  Copy in the reference; passed by pointer. */
typedef struct agnes_vote {
    int64_t round;     /* Vote.round (i64)                    */
    uint32_t value;    /* Vote.value: label or AGNES_NIL      */
    uint8_t typ;       /* AGNES_PREVOTE / AGNES_PRECOMMIT     */
    uint8_t pad[3];
} agnes_vote;

/* Event, state_machine.rs:96-110 */
typedef struct agnes_event {
    int64_t round;     /* round argument of State::apply (state_machine.rs:174)   */
    int64_t pol_round; /* Event::Proposal(pol_round, _) only                     */
    uint32_t value;    /* NewRoundProposer / Proposal / PolkaValue / PrecommitValue */
    uint8_t kind;      /* AGNES_EV_*                                              */
    uint8_t pad[3];
} agnes_event;

/* Message, state_machine.rs:118-163 (Proposal lib.rs:8-13, Timeout :152-155) */
typedef struct agnes_message {
    int64_t round;        /* NewRound(r) / Proposal.round / Vote.round / Timeout.round / Decision.round */
    int64_t pol_round;    /* Proposal.pol_round                                     */
    uint32_t value;       /* Proposal / Vote (AGNES_NIL = None) / Decision value    */
    uint8_t kind;         /* AGNES_MSG_*                                            */
    uint8_t vote_type;    /* Vote.typ                                               */
    uint8_t timeout_step; /* Timeout.step                                           */
    uint8_t pad;
} agnes_message;

/* State, state_machine.rs:24-31 (Copy).  64-byte device/host record.
 * `decided`/`decision_*` are an extension recording Message::Decision
 * (the reference leaves that to the consumer, consensus_executor.rs:46-48). */
typedef struct agnes_state {
    int64_t height;         /* State.height                      */
    int64_t round;          /* State.round                       */
    int64_t locked_round;   /* State.locked: Option<RoundValue>  */
    int64_t valid_round;    /* State.valid:  Option<RoundValue>  */
    int64_t decision_round; /* extension                         */
    uint32_t locked_value;
    uint32_t valid_value;
    uint32_t decision_value; /* extension */
    uint8_t step;            /* AGNES_STEP_*                     */
    uint8_t locked_present;  /* Option::is_some                  */
    uint8_t valid_present;
    uint8_t decided; /* extension */
    uint8_t pad[8];
} agnes_state;

/* ---------------------------------------------------------------------------
 * Per-vote result code (1 byte per input vote; the dense hot-path output)
 *
 *   bits 0..2  tally event  (VoteExecutor::apply -> Option<Event>, vote_executor.rs:20-36)
 *   bit  3     RoundSkip    (+1/3 distinct validators of the vote's round; extension)
 *   bits 4..7  message(s) State::apply produced for this vote (state machine on)
 * ------------------------------------------------------------------------- */
#define AGNES_CODE_NONE 0u
#define AGNES_CODE_POLKA_ANY 1u       /* (Prevote, Thresh::Any)     */
#define AGNES_CODE_POLKA_NIL 2u       /* (Prevote, Thresh::Nil)     */
#define AGNES_CODE_POLKA_VALUE 3u     /* (Prevote, Thresh::Value)   */
#define AGNES_CODE_PRECOMMIT_ANY 4u   /* (Precommit, Thresh::Any)   */
#define AGNES_CODE_PRECOMMIT_VALUE 5u /* (Precommit, Thresh::Value) */
#define AGNES_CODE_INVALID 6u  /* field out of range / wrong instance: vote ignored        */
#define AGNES_CODE_REJECTED 7u /* DEDUP mode: not the first vote of (round,type,validator) */
#define AGNES_CODE_EVENT_MASK 0x07u
#define AGNES_CODE_SKIP 0x08u
#define AGNES_CODE_MSG_SHIFT 4

/* message nibble (all carry round = the vote's round; value = the event's value) */
#define AGNES_VMSG_NONE 0u
#define AGNES_VMSG_TIMEOUT_PREVOTE 1u   /* Timeout{r, Prevote}   (arm 6, :196)  */
#define AGNES_VMSG_TIMEOUT_PRECOMMIT 2u /* Timeout{r, Precommit} (arm 12, :208) */
#define AGNES_VMSG_PRECOMMIT_NIL 3u     /* Vote precommit(r, None)   (:197)     */
#define AGNES_VMSG_PRECOMMIT_VALUE 4u   /* Vote precommit(r, Some v) (:198)     */
#define AGNES_VMSG_DECISION 5u          /* Decision{r, v}            (:211)     */
#define AGNES_VMSG_NEW_ROUND 6u         /* NewRound(r)               (:210)     */
#define AGNES_VMSG_NEW_ROUND_TIMEOUT_PRECOMMIT 7u /* RoundSkip then PrecommitAny   */
#define AGNES_VMSG_NEW_ROUND_DECISION 8u          /* RoundSkip then PrecommitValue */

/* ---------------------------------------------------------------------------
 * Batch configuration
 * ------------------------------------------------------------------------- */
#define AGNES_MODE_REFERENCE 0u /* every vote counts (round_votes.rs:48-56; test :120-122 relies on it) */
#define AGNES_MODE_DEDUP 1u     /* first vote of (instance, round, type, validator) wins; rest REJECTED */

#define AGNES_FLAG_ROUND_SKIP 0x1u      /* emit RoundSkip (+1/3) — producer absent in the reference */
#define AGNES_FLAG_STATE_MACHINE 0x2u   /* apply events to per-instance State (apply_msg :61-69)     */
#define AGNES_FLAG_DISTINCT_VALUES 0x4u /* compare value labels in prevote() (:241); default: ZST, all equal */
#define AGNES_FLAG_ONE_INSTANCE 0x8u    /* agnes_tally_carried only: the batch's segments are consecutive
                                           slices of ONE instance whose votes carry instance id
                                           agnes_config.reserved (C5: one huge instance split over
                                           waves and GPUs) */
#define AGNES_FLAG_WEIGHTS_CACHED 0x10u /* agnes_tally_carried only: batch->weight holds the weights
                                           agnes_tally_partials wrote for this batch; the votes are
                                           validated (set, validator index) as without it and the
                                           power table is not gathered again (C5 pass B) */
#define AGNES_FLAG_MASKED_REJECTED 0x20u /* agnes_tally_carried only: a vote whose type byte is
                                           AGNES_TYPE_MASKED gets AGNES_CODE_REJECTED instead of
                                           INVALID (still counted by agnes_last_error_count) —
                                           agnes_dedup_reject's rewrite inside the pass (C5 DEDUP) */

/* Route override, bits 8..9 of agnes_config.flags (diagnostics and the
 * route-equivalence tests: every route gives identical codes and States).
 *   AUTO      the engine's choice: the fused flow kernel for REFERENCE without
 *             RoundSkip, the per-instance kernel + apply pass otherwise, the i64
 *             kernel for instances outside the u32 domain
 *   INSTANCE  the per-instance u32 kernel with the State machine fused
 *   SPLIT     the per-instance u32 kernel, then the one-instance-per-lane apply pass
 *   WIDE      the i64 kernel for every instance */
#define AGNES_ROUTE_SHIFT 8
#define AGNES_ROUTE_MASK 0x3u
#define AGNES_ROUTE_AUTO 0u
#define AGNES_ROUTE_INSTANCE 1u
#define AGNES_ROUTE_SPLIT 2u
#define AGNES_ROUTE_WIDE 3u
#define AGNES_FLAG_ROUTE(r) ((uint32_t)(r) << AGNES_ROUTE_SHIFT)
/* Bits 16..20 of agnes_config.flags: minimum bits the DEDUP / RoundSkip first-vote
 * tables spend on a vote's index inside its instance (0 = just enough for the
 * batch).  More index bits leave fewer epochs per table fill, so the tables are
 * recycled more often (testing the recycling; results are identical). */
#define AGNES_EPOCH_BITS_SHIFT 16
#define AGNES_FLAG_EPOCH_BITS(b) (((uint32_t)(b) & 0x1Fu) << AGNES_EPOCH_BITS_SHIFT)

typedef struct agnes_config {
    uint32_t mode;       /* AGNES_MODE_*                                            */
    uint32_t flags;      /* AGNES_FLAG_*                                            */
    uint32_t max_rounds; /* votes with round >= max_rounds are INVALID (1..256)      */
    uint32_t reserved;
} agnes_config;

/* Canonical structure-of-arrays vote batch: 14 bytes per vote.
 * Votes of one instance are CONTIGUOUS and in arrival order:
 *   instance i owns votes [offsets[i], offsets[i+1]).
 * Each instance is the reference's per-height executor pair (VoteExecutor +
 * State), one independent VoteExecutor per (instance, round).
 * Alignment (device columns): instance/value/validator 16 B, round/type and the
 * codes output 4 B, weight 8 B — any hipMalloc / torch allocation qualifies;
 * otherwise agnes_tally returns AGNES_E_INVALID. */
typedef struct agnes_vote_batch {
    const uint32_t* instance;  /* n_votes — must equal the owning segment's index  */
    const uint8_t* round;      /* n_votes — Vote.round                             */
    const uint8_t* type;       /* n_votes — Vote.typ                               */
    const uint32_t* value;     /* n_votes — Vote.value (AGNES_NIL = None)          */
    const uint32_t* validator; /* n_votes — index into the instance's power set    */
    const uint64_t* offsets;   /* n_instances + 1                                  */
    const uint32_t* instance_set; /* optional n_instances; NULL -> instance % n_sets */
    const int64_t* weight;     /* optional n_votes: caller-supplied weight (vote_executor.rs:20)
                                   instead of the power-table gather                */
    uint64_t n_votes;
    uint32_t n_instances;
    uint32_t reserved;
} agnes_vote_batch;

/* ---------------------------------------------------------------------------
 * Scalar mirror of the reference API (the shape a Rust FFI binds; runs on the
 * GPU through the batch engine — there is no CPU implementation behind it).
 * ------------------------------------------------------------------------- */
typedef struct agnes_ve agnes_ve;

/* VoteExecutor::new(height, total_weight)            vote_executor.rs:13-16 */
agnes_ve* agnes_ve_new(int64_t height, int64_t total_weight);
/* VoteExecutor::apply(&mut self, vote, weight) -> Option<Event>
 * vote_executor.rs:20-23.  Returns 1 and fills *out on Some(event), 0 on None,
 * <0 on error.  Exactly the reference executor: ONE RoundVotes for every vote,
 * vote->round is not consulted by the tally (vote_executor.rs:9,14
 * "TODO: more rounds"); out->round is set to vote->round, the round
 * apply_msg passes to State::apply (consensus_executor.rs:68).  The batch
 * engine (agnes_tally) keeps one executor per (instance, round) instead. */
int agnes_ve_apply(agnes_ve* ve, const agnes_vote* vote, int64_t weight, agnes_event* out);
void agnes_ve_free(agnes_ve* ve);

/* RoundVotes (round_votes.rs:74-97): the tally layer below VoteExecutor.
 * agnes_rv_add_vote returns the Thresh (AGNES_THRESH_*) of RoundVotes::add_vote
 * (round_votes.rs:92-97) and, for Thresh::Value, its value in *value; <0 on error. */
typedef struct agnes_rv agnes_rv;
agnes_rv* agnes_rv_new(int64_t height, int64_t round, int64_t total);
int agnes_rv_add_vote(agnes_rv* rv, const agnes_vote* vote, int64_t weight, uint32_t* value);
void agnes_rv_free(agnes_rv* rv);

/* State::new(height)                                  state_machine.rs:35-43 */
void agnes_state_init(int64_t height, agnes_state* out);
/* State::apply(self, round, event) -> (State, Option<Message>)
 * state_machine.rs:174-214.  Returns 1 when a message was produced, 0 if
 * None, <0 on error.  Runs on the GPU. */
int agnes_state_apply(const agnes_state* in, int64_t round, const agnes_event* ev, uint32_t flags,
                      agnes_state* out, agnes_message* msg);

/* ---------------------------------------------------------------------------
 * Batch engine (the hot path).  All array pointers passed to agnes_tally /
 * agnes_apply_events are DEVICE pointers on the context's device.
 *
 * Streams: every call is asynchronous on its `stream` (NULL: the default stream).
 * A context's scratch is shared by its calls, so a call on a different stream
 * than the context's previous call first waits for that stream (an event): the
 * calls of one context never overlap.  Use one context per concurrent stream for
 * overlap; while capturing a HIP graph, make the call before the capture on the
 * capture stream too (a wait on another stream's event cannot be captured).
 * ------------------------------------------------------------------------- */
typedef struct agnes_ctx agnes_ctx;

int agnes_ctx_create(int device, agnes_ctx** out);
void agnes_ctx_destroy(agnes_ctx* ctx);
int agnes_ctx_device(const agnes_ctx* ctx);

/* Upload the validator power table (Validator.voting_power, validators.rs:5-8)
 * as int64 power[n_sets][n_vals] (HOST pointer).  totals (HOST, optional,
 * n_sets) is the total_weight of VoteExecutor::new (vote_executor.rs:13); NULL
 * means the wrapping sum of the set's powers. */
int agnes_upload_power(agnes_ctx* ctx, const int64_t* power, uint32_t n_sets, uint32_t n_vals,
                       const int64_t* totals);

/* Tally a batch: per-vote codes (device, n_votes bytes); optional per-instance
 * State array (device, n_instances, read and written in place) used when
 * AGNES_FLAG_STATE_MACHINE is set.  `stream` is a hipStream_t (NULL = default).
 * Asynchronous: returns after enqueueing.  Bad votes never fail the call; they
 * get AGNES_CODE_INVALID and are counted by agnes_last_error_count. */
int agnes_tally(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch,
                uint8_t* codes, agnes_state* states, void* stream);
/* agnes_tally with the States read from states_in and written to states_out
 * (State::apply takes self by value and returns the new State,
 * state_machine.rs:174: a batch of heights can start from one template of
 * States::new without copying it first).  states_in == NULL or == states_out:
 * in place, as agnes_tally.  The two arrays must not overlap otherwise. */
int agnes_tally_states(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch,
                       uint8_t* codes, const agnes_state* states_in, agnes_state* states_out, void* stream);

/* VoteCount of one (round, type) bucket (round_votes.rs:15-19): the executor state
 * a stream carries between calls.  value = the bucket's label, the last non-nil
 * value written (:50-54; 0 = VoteCount::new).  24-byte device record. */
typedef struct agnes_vote_count {
    int64_t value_w;
    int64_t nil_w;
    uint32_t value;
    uint32_t reserved;
} agnes_vote_count;

/* agnes_tally continuing carried executors: counts (DEVICE, [n_instances][2 *
 * max_rounds], index round * 2 + type) holds each segment's RoundVotes state
 * before its first vote and is overwritten with the state after its last.  With
 * AGNES_FLAG_ONE_INSTANCE every segment is a consecutive slice of one instance
 * (id cfg->reserved): a segment's counts are then the fold of the slices before it
 * (weights summed, the latest label) and the codes equal one stream's (C5: one
 * instance split over waves and GPUs, agnes_amd/dist.py tally_one_instance).
 * REFERENCE mode without RoundSkip or State machine; runs the i64 kernel. */
int agnes_tally_carried(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch,
                        uint8_t* codes, agnes_vote_count* counts, void* stream);

/* Pass A of the split-instance protocol as one reduction (C5, agnes_amd/dist.py
 * tally_one_instance): counts (DEVICE, [n_instances][2 * max_rounds]) := each
 * segment's VoteCounts from RoundVotes::new (round_votes.rs:48-56: the weights of
 * its valid votes summed per side, value = its last non-nil value, AGNES_NIL when
 * none): what AGNES_FOLD_RESET + agnes_tally_carried leave in counts, without the
 * thresholds and the codes.  weights (DEVICE, i64 [n_votes], or NULL): each vote's
 * weight, 0 for a vote that is not valid; pass B then runs agnes_tally_carried with
 * batch->weight = weights and AGNES_FLAG_WEIGHTS_CACHED.  The configurations, the
 * validity rules and AGNES_FLAG_ONE_INSTANCE are agnes_tally_carried's, except that
 * the weights always come from the power table: a batch with caller weights
 * (batch->weight != NULL) is AGNES_E_UNSUPPORTED.  The batch's columns need no
 * alignment; n_votes < 2^32 - 1.  Asynchronous on `stream`. */
int agnes_tally_partials(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch,
                         agnes_vote_count* counts, int64_t* weights, void* stream);

/* The fold of one instance's slices (C5, agnes_amd/dist.py tally_one_instance):
 * counts (DEVICE, [n_slices][keys]) hold each slice's partial VoteCounts (value
 * AGNES_NIL: no value written); partials fold like consecutive add_vote calls
 * (round_votes.rs:48-56: weights add, wrapping; the later value slot wins).
 *   AGNES_FOLD_RESET   every record := VoteCount::new with no value (AGNES_NIL)
 *   AGNES_FOLD_APPLY   every slice := carry (or zero) + the slices before it: the
 *                      carry-in of the next agnes_tally_carried pass
 *   totals (or NULL)   [keys] := carry + every slice
 * carry (DEVICE [keys] or NULL); flags also choose the label conventions:
 * AGNES_FOLD_CARRY_ZERO_NONE reads a carry label 0 as "none", _ZERO_LABELS /
 * _TOTAL_ZERO_LABELS write "none" as 0 (VoteCount::new's Value{}). */
#define AGNES_FOLD_RESET 0x1u
#define AGNES_FOLD_APPLY 0x2u
#define AGNES_FOLD_CARRY_ZERO_NONE 0x4u
#define AGNES_FOLD_ZERO_LABELS 0x8u
#define AGNES_FOLD_TOTAL_ZERO_LABELS 0x10u
int agnes_fold_counts(agnes_ctx* ctx, agnes_vote_count* counts, uint32_t n_slices, uint32_t keys,
                      const agnes_vote_count* carry, agnes_vote_count* totals, uint32_t flags, void* stream);

/* DEDUP for one instance split over slices (C5; agnes_amd/dist.py
 * tally_one_instance_dedup).  The carried tally is REFERENCE only, so the first
 * vote of each (round, type, validator) is found up front:
 *   agnes_dedup_first  lowers first[(round * 2 + type) * n_vals + validator] (DEVICE,
 *                      u64 [2 * max_rounds * n_vals], caller-initialised to
 *                      INT64_MAX) to base + j for every valid vote j of the batch,
 *                      base = the index of the batch's first vote in the whole
 *                      stream; the caller then min-combines `first` over the ranks;
 *   agnes_dedup_mask   writes type_out (DEVICE, n_votes): the batch's type column
 *                      with every valid vote that is not its key's first set to
 *                      AGNES_TYPE_MASKED — tallied with it, such a vote counts as
 *                      nothing (round_votes.rs:48-56 never runs for it);
 *   agnes_dedup_reject after the carried tally: the codes of the masked votes
 *                      INVALID -> AGNES_CODE_REJECTED (the DEDUP codes of the
 *                      whole instance; agnes_last_error_count still counts them);
 *                      or the carried tally with AGNES_FLAG_MASKED_REJECTED writes
 *                      REJECTED for them in the pass (one launch fewer).
 * Validity is the tally's: instance id == cfg->reserved, round < max_rounds,
 * type <= 1, validator < n_vals (set reserved % n_sets; batch->instance_set must be
 * NULL, else AGNES_E_UNSUPPORTED).
 * Asynchronous on `stream`. */
#define AGNES_TYPE_MASKED 0xFEu
int agnes_dedup_first(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch, uint64_t base,
                      uint64_t* first, void* stream);
int agnes_dedup_mask(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch, uint64_t base,
                     const uint64_t* first, uint8_t* type_out, void* stream);
/* agnes_dedup_first + agnes_dedup_mask in one call (round 4), for a batch that holds
 * every vote of the instance (one rank: no other slice's table is min-combined into
 * `first` between the two): `type_out` as the two calls give it; `first` is an output
 * here, written whole (INT64_MAX for a key without a valid vote), so it needs no
 * caller initialisation — the two calls' table on an INT64_MAX-filled `first`. */
int agnes_dedup_first_mask(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch, uint64_t base,
                           uint64_t* first, uint8_t* type_out, void* stream);
int agnes_dedup_reject(agnes_ctx* ctx, const uint8_t* type_masked, uint64_t n_votes, uint8_t* codes,
                       void* stream);

/* The State machine of ONE instance split into slices (C5 with
 * AGNES_FLAG_STATE_MACHINE; agnes_amd/dist.py one_instance_states), after the
 * carried tally wrote the slice's codes.  Without RoundSkip the vote events move
 * the State only at P1 (the first PolkaNil / PolkaValue at State.round while in
 * Prevote, state_machine.rs:197-198) and at C (the first PrecommitValue,
 * :211); every message follows from a vote's position relative to them.
 *   agnes_one_sm_scan    lowers marks[0] / marks[1] to the slice's first P1 / C
 *                        candidate (position << 32 | value)
 *   (the caller min-combines marks[0..1] over the ranks)
 *   agnes_one_sm_apply   ORs each vote's message nibble into its code; raises
 *                        marks[2] to the last valid candidate ((position + 1) << 32
 *                        | value) and marks[3] to C's round + 1
 *   (the caller max-combines marks[2..3] over the ranks)
 *   agnes_one_sm_finish  applies P1, the valid value and C to *state.
 * marks: DEVICE int64[4], initialised to {INT64_MAX, INT64_MAX, 0, 0}; state:
 * DEVICE, the instance's State before the slice's votes (read by scan / apply,
 * written by finish).  batch: the slice (round and value columns, n_votes; its
 * other columns are not read), base = the global index of its first vote;
 * base + n_votes <= 2^31.  REFERENCE or DEDUP mode, no RoundSkip
 * (AGNES_E_UNSUPPORTED). */
int agnes_one_sm_scan(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch, uint64_t base,
                      const uint8_t* codes, const agnes_state* state, int64_t* marks, void* stream);
int agnes_one_sm_apply(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch, uint64_t base,
                       uint8_t* codes, const agnes_state* state, int64_t* marks, void* stream);
int agnes_one_sm_finish(agnes_ctx* ctx, const int64_t* marks, agnes_state* state, void* stream);

/* Number of votes coded AGNES_CODE_INVALID by the most recent agnes_tally on
 * this context (synchronises the context's stream). */
int agnes_last_error_count(agnes_ctx* ctx, uint64_t* out);

/* Bytes of dynamic LDS one wave needs for cfg with n_vals validators per set;
 * > 0 on success, < 0 when the configuration is unsupported. */
int64_t agnes_lds_bytes_per_wave(const agnes_config* cfg, uint32_t n_vals);

/* Batched State::apply over explicit event lists (state_machine.rs:183-322):
 * instance i applies events [ev_offsets[i], ev_offsets[i+1]) in order to
 * states[i]; msgs[k] receives the Option<Message> of event k (kind 0 = None).
 * All pointers DEVICE.  One instance per lane. */
int agnes_apply_events(agnes_ctx* ctx, agnes_state* states, uint32_t n_instances,
                       const uint64_t* ev_offsets, const agnes_event* events, agnes_message* msgs,
                       uint32_t flags, void* stream);

/* Batched ConsensusExecutor::apply_msg (consensus_executor.rs:54-86) over
 * per-instance message streams: instance i applies messages [offsets[i],
 * offsets[i+1]) of `batch` in order, against its own VoteCounts (one executor per
 * (round, type), starting at VoteCount::new) and states[i] (in place).  The
 * batch's columns are read per message kind (kinds[j], AGNES_IN_*):
 *   VOTE       Message::Vote (:61-69): instance, round, type, value, validator
 *              (or weight) as agnes_tally, then State::apply(round, event)
 *   PROPOSAL   Message::Proposal (:56-60): Event::Proposal(pol_round[j], value)
 *              at round (pol_round NULL: -1 for every proposal)
 *   TIMEOUT    Message::Timeout (:70-77): type = AGNES_TIMEOUT_* -> TimeoutX at round
 *   NEW_ROUND  the executor's own NewRound (execute, :31-33): Event::NewRound at
 *              round, or NewRoundProposer(value) when value != AGNES_NIL
 * msgs[j] receives the Option<Message> of message j (kind AGNES_MSG_NONE = None),
 * codes[j] the vote's tally code (bits 0..2; INVALID for a bad vote or kind, NONE
 * for the other kinds; agnes_last_error_count counts the INVALIDs).  REFERENCE mode without RoundSkip (else
 * AGNES_E_UNSUPPORTED); cfg->flags AGNES_FLAG_DISTINCT_VALUES applies; the State
 * machine is implied; max_rounds <= 16.  All pointers DEVICE; one instance per
 * lane (latency bound: messages of one instance are sequential). */
#define AGNES_IN_VOTE 0u
#define AGNES_IN_PROPOSAL 1u
#define AGNES_IN_TIMEOUT 2u
#define AGNES_IN_NEW_ROUND 3u
int agnes_apply_msgs(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch, const uint8_t* kinds,
                     const int32_t* pol_round, uint8_t* codes, agnes_state* states, agnes_message* msgs,
                     void* stream);

/* ---------------------------------------------------------------------------
 * Validator sets: ValidatorSet, validators.rs:23-56 -- the
 * intended behaviour; the file does not compile, so no reference output pins it.
 * A set keeps its validators sorted by address (ValidatorSet::sort, :49-55;
 * Validator::address = the public key, :15-17) without exact duplicates
 * (Vec::dedup, a derived PartialEq: same address and power).
 *
 * agnes_valset_build builds n_sets sets at once from one flat list: validator i has
 * address addr[i * addr_len ..] (fixed length, 1..64 B), power power[i] and set
 * set_of[i] (NULL: set 0; a set id >= n_sets drops the validator).  Outputs, sets
 * consecutive:
 *   order[k]        the input index of output validator k (sorted by address; equal
 *                   addresses by power -- sort_unstable_by leaves them in any order,
 *                   this is one -- then by input index; a duplicate keeps its first)
 *   power_out[k]    power[order[k]]: the power row agnes_upload_power takes
 *   addr_out[k]     (optional) the sorted addresses, for agnes_valset_find
 *   set_offsets[s]  [n_sets + 1]: set s is outputs [set_offsets[s], set_offsets[s+1])
 *   totals[s]       the wrapping sum of set s's powers (VoteExecutor::new's
 *                   total_weight, vote_executor.rs:13)
 *   *n_out (HOST)   the number of outputs.
 * DEVICE pointers except n_out; n <= 2^30; synchronous.
 * agnes_valset_find: for query q (address q_addr[q * addr_len ..], set q_set[q] or 0)
 * the index of its validator in the built set (ValidatorSet::update / remove: "find
 * val in list", :39, :44), UINT64_MAX when absent. */
int agnes_valset_build(agnes_ctx* ctx, const uint8_t* addr, uint32_t addr_len, const int64_t* power,
                       const uint32_t* set_of, uint64_t n, uint32_t n_sets, uint32_t* order, uint64_t* set_offsets,
                       int64_t* power_out, int64_t* totals, uint8_t* addr_out, uint64_t* n_out, void* stream);
int agnes_valset_find(agnes_ctx* ctx, const uint8_t* sorted_addr, uint32_t addr_len, const uint64_t* set_offsets,
                      uint32_t n_sets, const uint8_t* q_addr, const uint32_t* q_set, uint64_t n_q, uint64_t* out,
                      void* stream);

/* ---------------------------------------------------------------------------
 * Wire format and signature verification.  The reference has
 * neither: its README (README.md:8-14, 36-41) leaves the wire format and the
 * signature check to the consumer, and Validator carries the public key the
 * votes are checked against (validators.rs:4-8, 15-17: address() = public_key).
 * A signed vote is one 104-byte little-endian record: the 40 sign-bytes
 * (magic .. pad) followed by the Ed25519 signature R || S over them (RFC 8032).
 * ------------------------------------------------------------------------- */
#define AGNES_WIRE_MAGIC 0x31564741u /* "AGV1" */
#define AGNES_WIRE_SIGNED_BYTES 40u
typedef struct agnes_wire_vote {
    uint32_t magic;     /* AGNES_WIRE_MAGIC                                   */
    uint32_t instance;  /* the instance id of the batch the vote belongs to  */
    int64_t height;     /* State.height (state_machine.rs:8)                  */
    int64_t round;      /* Vote.round (lib.rs:24)                             */
    uint32_t validator; /* index into the instance's validator set           */
    uint32_t value;     /* value_id, AGNES_NIL = nil (Vote.value: Option<Value>) */
    uint8_t type;       /* 0 prevote, 1 precommit (VoteType, lib.rs:15-19)    */
    uint8_t pad[7];     /* zero                                               */
    uint8_t sig[64];    /* Ed25519 R || S over bytes 0 .. 39                  */
} agnes_wire_vote;
enum {
    AGNES_WIRE_OK = 0,
    AGNES_WIRE_BAD_FORMAT = 1,    /* magic, type > 1, pad != 0, round outside [0, max_rounds) */
    AGNES_WIRE_BAD_VALIDATOR = 2, /* no such set / validator for the instance                */
    AGNES_WIRE_BAD_SIGNATURE = 3, /* S >= L, the key decodes to no point, or [S]B - [k]A != R */
    AGNES_WIRE_BAD_HEIGHT = 4     /* height != the batch's height                             */
};
/* agnes_wire_ingest: decode and verify n records into the tally's SoA columns, one
 * record per lane.  The key of record i is pubkeys[(set * n_vals + validator) * 32 ..]
 * with set = instance_set[instance] (instance < n_instances, else BAD_VALIDATOR) or,
 * without instance_set, instance % n_sets.  Signature check: RFC 8032 §5.1.7 in the
 * cofactorless form of OpenSSL 3.0 (reject S >= L; decode A per §5.1.3; accept iff
 * encode([S]B - [k]A) == R, k = SHA-512(R || A || sign-bytes) mod L).  Out, in record
 * order: instance, value, validator as decoded; round (low byte) and type for an
 * accepted record, round 0 and type 0xFF (coded INVALID by agnes_tally) for any
 * other; verdict[i] = AGNES_WIRE_*.  All pointers DEVICE; records 8-B and pubkeys
 * 16-B aligned (else AGNES_E_INVALID); n <= 2^36.  Asynchronous on `stream`. */
int agnes_wire_ingest(agnes_ctx* ctx, const agnes_wire_vote* records, uint64_t n, const uint8_t* pubkeys,
                      uint32_t n_sets, uint32_t n_vals, const uint32_t* instance_set, uint32_t n_instances,
                      int64_t height, uint32_t max_rounds, uint32_t* instance, uint8_t* round, uint8_t* type,
                      uint32_t* value, uint32_t* validator, uint8_t* verdict, void* stream);

/* ---------------------------------------------------------------------------
 * Native multi-GPU driver: one context, stream and host thread
 * per device; a HOST batch is cut into contiguous instance ranges balanced by
 * votes (instances are independent: no collective on the data path), each range
 * is copied to its device, tallied (agnes_tally) and its codes / States copied
 * back into the HOST arrays.  The entry a consumer without torch.distributed binds
 * (agnes_amd/dist.py is the one-process-per-GPU Python equivalent).  A device may
 * be listed more than once (several contexts on one GPU).
 * ------------------------------------------------------------------------- */
typedef struct agnes_multi agnes_multi;
typedef struct agnes_multi_stats {
    uint32_t device, i0, i1; /* the range [i0, i1) this device tallied */
    uint32_t exchange;       /* agnes_multi_tally_one: AGNES_MULTI_X_* bits of how it exchanged */
    uint64_t n_votes, n_invalid;
    double h2d_ms, tally_ms, d2h_ms; /* host wall-clock of the three phases */
} agnes_multi_stats;
int agnes_multi_create(const int* devices, uint32_t n_devices, agnes_multi** out);
void agnes_multi_destroy(agnes_multi* m);
/* agnes_upload_power on every device */
int agnes_multi_upload_power(agnes_multi* m, const int64_t* power, uint32_t n_sets, uint32_t n_vals,
                             const int64_t* totals);
/* batch, codes, states (optional, in/out with AGNES_FLAG_STATE_MACHINE) are HOST
 * pointers; stats (optional) receives one record per device.  Synchronous. */
int agnes_multi_tally(agnes_multi* m, const agnes_config* cfg, const agnes_vote_batch* batch, uint8_t* codes,
                      agnes_state* states, agnes_multi_stats* stats);

/* C5 through the native driver: ONE instance's stream (batch: HOST, n_instances ==
 * 1, instance ids 0, the power table's set 0) cut into consecutive slices, one per
 * device in device order, and tallied with codes identical to one stream's
 * (VoteExecutor::apply vote by vote, vote_executor.rs:20-36, over the running
 * VoteCount of round_votes.rs:48-67).  Each device tallies its slice twice around
 * the path's exchange step: pass A partials -> ALL-GATHER of the
 * slice totals -> each device's carry-in (the fold of the slices before it) -> pass
 * B.  DEDUP mode adds an ALL-REDUCE(MIN) of the first-vote table (the first vote of
 * each (round, type, validator) wins); AGNES_FLAG_STATE_MACHINE with `state` (HOST,
 * one record, in/out) an ALL-REDUCE(MIN) of the P1 / C positions and an
 * ALL-REDUCE(MAX) of the valid candidate and the decision round (agnes_one_sm_*).
 * counts (HOST [2 * max_rounds], optional) receives the instance's executors after
 * its last vote.  segments_per_device: waves per slice (0: 2048).  No RoundSkip,
 * DISTINCT_VALUES, caller weights or instance sets (AGNES_E_UNSUPPORTED).
 * Synchronous; stats (optional) one record per device (i0 = 0, i1 = 1). */
int agnes_multi_tally_one(agnes_multi* m, const agnes_config* cfg, const agnes_vote_batch* batch, uint8_t* codes,
                          agnes_state* state, agnes_vote_count* counts, uint32_t segments_per_device,
                          agnes_multi_stats* stats);
/* How agnes_multi_tally_one exchanges: AUTO = RCCL (ncclCommInitAll, one rank per
 * device, xGMI between MI355X) when the devices are distinct and more than one, else
 * pinned host memory; HOST; RCCL (AGNES_E_UNSUPPORTED when a device is listed twice). */
#define AGNES_MULTI_EXCHANGE_AUTO 0u
#define AGNES_MULTI_EXCHANGE_HOST 1u
#define AGNES_MULTI_EXCHANGE_RCCL 2u
int agnes_multi_exchange(agnes_multi* m, uint32_t mode);
/* agnes_multi_stats.exchange: RCCL carried the call's collectives; FALLBACK: the
 * handle's RCCL self-check failed (the first collective of each kind -- all-gather,
 * MIN on u64 / i64, MAX -- is compared with the host exchange of the same data; on a
 * mismatch the call's results come from the host exchange and the handle uses it from
 * then on); HOST: pinned host memory carried them. */
#define AGNES_MULTI_X_RCCL 1u
#define AGNES_MULTI_X_FALLBACK 2u
#define AGNES_MULTI_X_HOST 4u
/* Test hook (not for production): bit k of ops re-arms the self-check of kind k (0 MIN
 * u64, 1 MIN i64, 2 MAX i64, 3 all-gather) and flips the first received byte of its next
 * RCCL collective before the check; bit 4 + k flips it in EVERY RCCL collective of kind
 * k, checked or not (an RCCL that is really broken: once a check fails, the call's later
 * collectives must take the host exchange), so tests can drive the fallback path. */
int agnes_multi_test_corrupt(agnes_multi* m, uint32_t ops);

/* ---------------------------------------------------------------------------
 * Edge-triggered summary of a coded batch.
 *
 * VoteExecutor::apply is level-triggered (vote_executor.rs:20-36): once a
 * threshold holds, every later vote of the executor repeats its event.  The
 * summary keeps the votes a consumer acts on.  Per instance, the executor of a
 * valid vote (event not INVALID / REJECTED) is its (round, type) — the
 * HeightVotes the reference leaves as a stub (consensus_executor.rs:5,
 * vote_executor.rs:9,14) — and its LEVEL is the vote's code bits 0..3 (tally
 * event + RoundSkip), 0 before its first vote (VoteCount::new,
 * round_votes.rs:36-45).  A vote is an EDGE when its level differs from the
 * level its executor's previous valid vote left, or when it carries a message
 * (code bits 4..7) other than the last message of its executor (State::apply
 * repeats Timeouts the same way, state_machine.rs:196,208).  Records are ordered
 * by instance, then vote index.
 * ------------------------------------------------------------------------- */
typedef struct agnes_edge {
    uint64_t vote;     /* index of the vote in the batch                    */
    uint32_t instance; /* the vote's segment (instance) index               */
    uint8_t round;     /* Vote.round                                        */
    uint8_t type;      /* Vote.typ                                          */
    uint8_t code;      /* the vote's code byte: new level | message << 4     */
    uint8_t prev;      /* the executor before this vote: level | last message << 4 */
} agnes_edge;

/* The tally and its edge summary in ONE call (round 5), SEGMENTED by instance: instance
 * i's edges at out[offsets[i] + k], k < counts[i] (a vote is at most one edge), in vote
 * order -- the records agnes_edges gives, at segment offsets.  On the flow route
 * (REFERENCE without RoundSkip, max_rounds <= 15, u32 sums; any offsets) the tally
 * kernel finds and writes them while the votes are in registers, each executor's state
 * carried in LDS: no pass over the codes; on the split per-instance route (DEDUP or
 * RoundSkip with the State machine, max_rounds <= 8) the State machine's pass writes
 * them.  counts (DEVICE, n_instances u64); out
 * (DEVICE, 16-B aligned, n_votes records; offsets must not go back); max_rounds <= 128.  agnes_edges_compact
 * gives the dense layout (offsets[n_instances + 1] from the counts; out, when not
 * null, exactly agnes_edges'). */
int agnes_tally_edges(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch, uint8_t* codes,
                      const agnes_state* states_in, agnes_state* states_out, uint64_t* counts, agnes_edge* out,
                      void* stream);
/* out_cap: the records out holds (see agnes_records_overflow) */
int agnes_edges_compact(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch, const uint64_t* counts,
                        const agnes_edge* seg, uint64_t* offsets, agnes_edge* out, uint64_t out_cap, void* stream);
/* Pass 1: offsets (DEVICE, n_instances + 1): exclusive offsets of each instance's
 * edges, offsets[n_instances] = the total.  codes as agnes_tally left them
 * (DEVICE); votes with round >= cfg->max_rounds or type > 1 are never edges.
 * Asynchronous on `stream`. */
int agnes_edge_offsets(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch,
                       const uint8_t* codes, uint64_t* offsets, void* stream);
/* Pass 2: the records into out (DEVICE, out_cap records: offsets[n_instances] of them),
 * instance i's at [offsets[i], offsets[i+1]).  offsets from agnes_edge_offsets on the
 * same batch and codes; an edge past out_cap or past its instance's end offset is
 * dropped, never written (agnes_records_overflow reports it). */
int agnes_edges(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch,
                const uint8_t* codes, const uint64_t* offsets, agnes_edge* out, uint64_t out_cap, void* stream);
/* The same summary of the LAST agnes_multi_tally's batch (the native multi-GPU
 * driver), gathered from every device into HOST arrays in the batch's own numbering:
 * offsets [n_instances + 1] first, then out [offsets[n_instances]] records. */
int agnes_multi_edge_offsets(agnes_multi* m, const agnes_config* cfg, uint64_t* offsets);
int agnes_multi_edges(agnes_multi* m, const agnes_config* cfg, const uint64_t* offsets, agnes_edge* out);

/* ---------------------------------------------------------------------------
 * Event stream: every Some(Event) the batch's votes produced, stream-compacted
 * (instance then vote order) with the Event's payload — what a caller of
 * VoteExecutor::apply (vote_executor.rs:20-23, via ConsensusExecutor::apply_vote,
 * consensus_executor.rs:61-69) collects vote by vote.  A vote gives at most two
 * records: a RoundSkip (code bit AGNES_CODE_SKIP, applied first) and its
 * VoteExecutor event (code bits 0..2 = 1..5).  The Value a PolkaValue /
 * PrecommitValue carries is its VoteCount's value slot after the vote (the last
 * non-nil value added, round_votes.rs:50-54, 58-59): the walk follows the value
 * column over the votes the tally added (every code but INVALID and REJECTED),
 * from VoteCount::new's Value{} (0) — executors carried from an earlier call
 * (agnes_tally_carried) are not followed.
 * ------------------------------------------------------------------------- */
typedef struct agnes_vote_event {
    uint64_t vote;     /* index of the vote in the batch                             */
    uint32_t instance; /* the vote's segment (instance) index                        */
    uint32_t value;    /* PolkaValue / PrecommitValue: the Value; else AGNES_NIL      */
    uint8_t round;     /* Vote.round                                                 */
    uint8_t kind;      /* AGNES_EV_POLKA_ANY .. AGNES_EV_PRECOMMIT_VALUE, _ROUND_SKIP */
    uint8_t message;   /* the vote's State machine message nibble (code >> 4)        */
    uint8_t pad[5];
} agnes_vote_event;

/* Pass 1: offsets (DEVICE, n_instances + 1): exclusive offsets of each instance's
 * records, offsets[n_instances] = the total.  codes as agnes_tally left them. */
int agnes_event_offsets(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch,
                        const uint8_t* codes, uint64_t* offsets, void* stream);
/* Pass 2: the records into out (DEVICE, 8-B aligned, out_cap records: offsets[n_instances]
 * of them); reads codes, round, type and value.  max_rounds <= 64.  A record past out_cap
 * or past its instance's (its emit batch's) end offset -- offsets that are not this
 * batch's, an undersized out -- is dropped, never written (agnes_records_overflow). */
int agnes_events(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch,
                 const uint8_t* codes, const uint64_t* offsets, agnes_vote_event* out, uint64_t out_cap,
                 void* stream);

/* The tally and its event stream in ONE call (agnes_tally with
 * d_out / d_n_out): agnes_tally_states, then the records of every Some(Event) as
 * agnes_event_offsets + agnes_events would give them.  offsets (DEVICE,
 * n_instances + 1) receives the exclusive record offsets, offsets[n_instances] the
 * number of records (d_n_out); out (DEVICE, 8-B aligned) must hold
 * agnes_events_capacity(cfg, batch) records (the most a batch can produce: one per
 * vote, two with RoundSkip).  On the fused route (REFERENCE without RoundSkip,
 * max_rounds <= 15) the tally kernel counts each instance's records itself, so no
 * count pass re-reads the codes.  batch->value 4-B aligned; max_rounds <= 64. */
int agnes_tally_events(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch, uint8_t* codes,
                       const agnes_state* states_in, agnes_state* states_out, uint64_t* offsets,
                       agnes_vote_event* out, void* stream);
uint64_t agnes_events_capacity(const agnes_config* cfg, const agnes_vote_batch* batch);

/* The same records SEGMENTED by instance (round 5): no scan between the tally and the
 * records, so on the flow route (REFERENCE without RoundSkip, max_rounds <= 15, every
 * and max_rounds <= 15: the C2 / C3 streams and their ragged variants) the
 * tally kernel writes them itself while the votes are in registers: the records cost no
 * second pass over the votes.
 * Instance i's records are out[seg(i) + k], k < counts[i], in vote order, with
 * seg(i) = batch->offsets[i] (2 * offsets[i] with AGNES_FLAG_ROUND_SKIP); the slots
 * between an instance's last record and the next segment are left as they were.  Every
 * other route writes the segments and the counts with the event stream's emit pass (no
 * count pass; a lane-per-instance walk for the flow route's walk-list instances,
 * columns off 16-B alignment, or max_rounds > 32).
 * counts (DEVICE, n_instances u64); out (DEVICE, 16-B aligned) must hold
 * agnes_events_capacity(cfg, batch) records; the segments are the instances' vote
 * ranges, so offsets must not go back (overlapping ranges overlap their segments).
 * The record is agnes_vote_event without the instance (the segment names it) and the
 * padding. */
typedef struct agnes_seg_event {
    uint64_t vote;    /* index of the vote in the batch                             */
    uint32_t value;   /* PolkaValue / PrecommitValue: the Value; else AGNES_NIL      */
    uint8_t round;    /* Vote.round                                                 */
    uint8_t kind;     /* AGNES_EV_POLKA_ANY .. AGNES_EV_PRECOMMIT_VALUE, _ROUND_SKIP */
    uint8_t message;  /* the vote's State machine message nibble (code >> 4)        */
    uint8_t pad;
} agnes_seg_event;
int agnes_tally_records(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch, uint8_t* codes,
                        const agnes_state* states_in, agnes_state* states_out, uint64_t* counts, agnes_seg_event* out,
                        void* stream);
/* The dense layout from the segmented one (one pass over the records, none over the
 * votes): offsets (DEVICE, n_instances + 1) := the exclusive scan of counts
 * (offsets[n_instances] = the total), then (out not null, 8-B aligned) the
 * agnes_vote_event records in instance then vote order -- exactly agnes_tally_events'. */
int agnes_records_compact(agnes_ctx* ctx, const agnes_config* cfg, const agnes_vote_batch* batch,
                          const uint64_t* counts, const agnes_seg_event* seg, uint64_t* offsets, agnes_vote_event* out,
                          uint64_t out_cap, void* stream);

/* Records the dense writers (agnes_events, agnes_edges, agnes_tally_events, the two
 * compactions) dropped on this context since the last query, because they fell past
 * out_cap (agnes_tally_events: agnes_events_capacity) or past their segment's end
 * offset: the calls are asynchronous, so a bad size surfaces here, as a status, and
 * never as a write outside `out`.  Synchronises the context's stream; resets the count.
 * Returns AGNES_OK (nothing dropped) or AGNES_E_OVERFLOW with the count in *dropped.
 * The segmented writers (agnes_tally_records / agnes_tally_edges) place instance i's
 * records at most at its own votes' positions (a vote gives at most `mult` records),
 * inside agnes_events_capacity() for any offsets, so they cannot overflow. */
int agnes_records_overflow(agnes_ctx* ctx, uint64_t* dropped);

/* ---------------------------------------------------------------------------
 * Synthetic workload generator (counter-based splitmix64; identical on host
 * and device, see agnes_amd/csrc/agnes_gen.h).  Not part of the hot path.
 * ------------------------------------------------------------------------- */
typedef struct agnes_gen_params {
    uint64_t seed;
    uint32_t n_instances;
    uint32_t n_vals;          /* validators per set                             */
    uint32_t rounds_min;      /* rounds per instance ~ U[rounds_min, rounds_max] */
    uint32_t rounds_max;
    uint32_t nil_permille;    /* base votes that are nil                         */
    uint32_t dup_permille;    /* extra exact duplicates per round (of 2*n_vals)  */
    uint32_t equiv_permille;  /* extra equivocating votes per round              */
    uint32_t higher_permille; /* extra votes tagged round+1 per round            */
    uint32_t order;           /* AGNES_ORDER_*                                   */
    uint32_t instance_base;   /* global id of local instance 0 (sharding)        */
    uint32_t absent_permille; /* abstention (<= 500): round r keeps M - A_r votes, A_r ~
                                 U[0, 2 M absent / 1000] -- instance lengths take any value */
    uint32_t reserved;
} agnes_gen_params;

#define AGNES_ORDER_SHUFFLED 0u /* random permutation of each round's votes       */
#define AGNES_ORDER_PHASED 1u   /* each round: shuffled prevotes, then precommits */
#define AGNES_ORDER_SORTED 2u   /* each round: prevotes by validator, then precommits */

/* votes per instance (without abstention every round of one params has the same count) */
uint64_t agnes_gen_instance_votes(const agnes_gen_params* p, uint32_t local_instance);
/* host: offsets[n_instances+1] */
int agnes_gen_offsets(const agnes_gen_params* p, uint64_t* offsets);
/* device: fill the SoA columns of a batch whose offsets are already on device */
int agnes_gen_votes_device(agnes_ctx* ctx, const agnes_gen_params* p, const uint64_t* d_offsets,
                           uint64_t n_votes, uint32_t* instance, uint8_t* round, uint8_t* type,
                           uint32_t* value, uint32_t* validator, void* stream);

#define AGNES_POWER_UNIFORM 0u /* U[lo, hi]                                   */
#define AGNES_POWER_ZIPF 1u    /* floor(hi / (rank+1)^1.1), rank a hashed permutation */
#define AGNES_POWER_EQUAL 2u   /* all == lo                                   */
/* host: power[n_sets][n_vals] */
int agnes_gen_power(uint64_t seed, uint32_t n_sets, uint32_t n_vals, uint32_t kind, int64_t lo,
                    int64_t hi, int64_t* power);

/* Per-kernel timing of the engine's own launches (measurement; off by default).
 * agnes_kernel_timing(1) clears the records and brackets every kernel the engine
 * enqueues from then on with HIP events on the caller's stream; (0) stops.
 * agnes_kernel_times synchronises on the recorded events and writes, per kernel
 * name in first-launch order, the launch count and total milliseconds. */
typedef struct agnes_kernel_time {
    char name[40];
    uint32_t launches;
    uint32_t pad;
    double total_ms;
} agnes_kernel_time;
int agnes_kernel_timing(int enable);
int agnes_kernel_times(agnes_kernel_time* out, uint32_t cap, uint32_t* n);

/* ABI probe */
uint32_t agnes_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* AGNES_H */
