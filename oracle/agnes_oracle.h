/*
 * agnes_oracle.h — CPU restatement of Liamsi/agnes's vote-tally / state-machine
 * path.  TEST INFRASTRUCTURE ONLY: it is the checker for the HIP engine and the
 * `cpu_baseline` leg of bench.py.  Product code (agnes_amd/, include/) never
 * links, loads or calls it.
 *
 * Parity pinning: the two unit tests the reference ships
 *   round_votes::tests::add_votes   (src/round_votes.rs:107-132)
 *   state_machine::tests::happy_case (src/state_machine.rs:331-345)
 * are replayed against this oracle (tests/golden/reference_tests.json,
 * tests/test_oracle_golden.py), together with traces derived by hand from the
 * cited code.  The reference itself cannot be built here (Rust,
 * no toolchain; validators.rs does not type-check), so there is no oracle/_ref.
 * Extensions (per-round executors, DEDUP, RoundSkip producer, power-table
 * weights) are specified in DESIGN.md §2 and cross-checked against an
 * independent pure-Python restatement (tests/pyref.py).
 */
#ifndef AGNES_ORACLE_H
#define AGNES_ORACLE_H

#include <stdint.h>

#include "../include/agnes.h"

#ifdef __cplusplus
extern "C" {
#endif

/* VoteCount, round_votes.rs:15-19 */
typedef struct orc_vote_count {
    int64_t nil;
    int64_t value_w;
    int64_t total;
    uint32_t value; /* last value written (label of Value{}; initial label 0) */
    uint32_t pad;
} orc_vote_count;

/* RoundVotes, round_votes.rs:74-80 */
typedef struct orc_round_votes {
    int64_t height;
    int64_t round;
    orc_vote_count prevotes;
    orc_vote_count precommits;
} orc_round_votes;

int orc_is_quorum(int64_t value, int64_t total);   /* round_votes.rs:31-33       */
int orc_is_one_third(int64_t value, int64_t total); /* RoundSkip producer (ext.)  */
void orc_vc_new(orc_vote_count* c, int64_t total); /* round_votes.rs:36-45       */
/* round_votes.rs:48-67; returns AGNES_THRESH_*, *tvalue = Thresh::Value payload */
uint32_t orc_vc_add(orc_vote_count* c, uint32_t value, int64_t weight, uint32_t* tvalue);
void orc_rv_new(orc_round_votes* rv, int64_t height, int64_t round, int64_t total); /* :83-90 */
uint32_t orc_rv_add(orc_round_votes* rv, uint32_t typ, uint32_t value, int64_t weight,
                    uint32_t* tvalue); /* :92-97 */
/* vote_executor.rs:26-36: returns AGNES_EV_* or AGNES_EV_NONE */
uint32_t orc_to_event(uint32_t typ, uint32_t thresh);
/* VoteExecutor::apply, vote_executor.rs:20-23 (one RoundVotes, round 0) */
uint32_t orc_ve_apply(orc_round_votes* rv, const agnes_vote* v, int64_t weight, uint32_t* evalue);

void orc_state_new(int64_t height, agnes_state* s); /* state_machine.rs:35-43 */
/* state_machine.rs:183-322; returns 1 when *msg holds Some(message) */
int orc_state_apply(agnes_state* s, int64_t round, const agnes_event* ev, uint32_t flags,
                    agnes_message* msg);

/* Batch restatement of the engine contract: one executor per
 * (instance, round), weights from power[set][validator] or batch->weight.
 * Host pointers.  states may be NULL when the state-machine flag is clear. */
typedef struct orc_power {
    const int64_t* power; /* [n_sets][n_vals] */
    const int64_t* totals; /* [n_sets] */
    uint32_t n_sets;
    uint32_t n_vals;
} orc_power;

int orc_tally(const agnes_config* cfg, const agnes_vote_batch* batch, const orc_power* pw,
              uint8_t* codes, agnes_state* states, uint64_t* n_invalid);
/* same, instances split over `threads` pthreads (CPU baseline) */
int orc_tally_mt(const agnes_config* cfg, const agnes_vote_batch* batch, const orc_power* pw,
                 uint8_t* codes, agnes_state* states, uint64_t* n_invalid, int threads);
/* orc_tally_mt that also writes, per vote, the Value its VoteExecutor event
 * carries (labels[j]: the VoteCount's value slot for PolkaValue / PrecommitValue,
 * AGNES_NIL otherwise) */
int orc_tally_labels(const agnes_config* cfg, const agnes_vote_batch* batch, const orc_power* pw,
                     uint8_t* codes, agnes_state* states, uint64_t* n_invalid, uint32_t* labels,
                     int threads);
/* the event stream (agnes_event_offsets + agnes_events) from the tally's codes and
 * labels: offsets[n_instances + 1]; out NULL = count only */
int orc_events(const agnes_config* cfg, const agnes_vote_batch* batch, const uint8_t* codes,
               const uint32_t* labels, uint64_t* offsets, agnes_vote_event* out);
/* batched State::apply over explicit event lists */
int orc_apply_events(agnes_state* states, uint32_t n_instances, const uint64_t* ev_offsets,
                     const agnes_event* events, agnes_message* msgs, uint32_t flags);

/* batched ConsensusExecutor::apply_msg over per-instance message streams
 * (agnes_apply_msgs): kinds AGNES_IN_*, pol_round per message (NULL: -1) */
int orc_apply_msgs(const agnes_config* cfg, const agnes_vote_batch* batch, const orc_power* pw, const uint8_t* kinds,
                   const int32_t* pol_round, uint8_t* codes, agnes_state* states, agnes_message* msgs,
                   uint64_t* n_invalid);

/* validator sets (agnes_valset_build's contract, host pointers) */
int orc_valset_build(const uint8_t* addr, uint32_t addr_len, const int64_t* power, const uint32_t* set_of,
                     uint64_t n, uint32_t n_sets, uint32_t* order, uint64_t* set_offsets, int64_t* power_out,
                     int64_t* totals, uint64_t* n_out);

/* edge-triggered summary of coded votes (agnes_edge_offsets + agnes_edges):
 * offsets[n_instances + 1]; out NULL = count only */
int orc_edges(const agnes_config* cfg, const agnes_vote_batch* batch, const uint8_t* codes,
              uint64_t* offsets, agnes_edge* out);

/* wrapping totals of each set (VoteExecutor::new's total_weight default) */
void orc_set_totals(const int64_t* power, uint32_t n_sets, uint32_t n_vals, int64_t* totals);

/* host generator (same header as the device generator) */
uint64_t orc_gen_instance_votes(const agnes_gen_params* p, uint32_t i);
int orc_gen_offsets(const agnes_gen_params* p, uint64_t* offsets);
int orc_gen_votes(const agnes_gen_params* p, const uint64_t* offsets, uint32_t* instance,
                  uint8_t* round, uint8_t* type, uint32_t* value, uint32_t* validator);
int orc_gen_power(uint64_t seed, uint32_t n_sets, uint32_t n_vals, uint32_t kind, int64_t lo,
                  int64_t hi, int64_t* power);

#ifdef __cplusplus
}
#endif

#endif
