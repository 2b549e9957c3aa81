/*
 * agnes_internal.h — engine-internal declarations shared by the kernels
 * (agnes_kernels.hip) and the host C ABI (agnes_api.cpp).
 */
#ifndef AGNES_INTERNAL_H
#define AGNES_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/agnes.h"

/* Per power set, precomputed on the host at upload (agnes_upload_power).
 * fast == 1 when every power is in [0, 2^31) and 0 <= total <= i64::MAX/2:
 * then, for sums s < 2^31, `3*s > 2*total` (round_votes.rs:32) is exactly
 * `s > q2` with q2 = min(floor(2*total/3), 2^32-1), and the +1/3 RoundSkip test
 * `3*s > total` is `s > q1`, q1 = min(floor(total/3), 2^32-1). */
typedef struct agnes_set_info {
    int64_t total;
    uint32_t q2;
    uint32_t q1;
    uint32_t maxpow;
    uint32_t fast;
    /* the u64 domain (w64 == 1): every power >= 0 and 0 <= total < 2^61.  For sums
     * s < 2^61 `3*s > 2*total` is `s > q2w` (q2w = floor(2*total/3)) and `3*s > total`
     * is `s > q1w`, without the i64 wrap (round_votes.rs:31-33) */
    uint32_t w64;
    uint32_t pad;
    uint64_t q2w;
    uint64_t q1w;
    uint64_t maxw;
} agnes_set_info;

/* Carried VoteCount of one (instance, round, type): round_votes.rs:15-19 */
typedef struct agnes_carry_rec {
    int64_t value_w;
    int64_t nil_w;
    uint32_t value;
    uint32_t pad;
} agnes_carry_rec;

typedef struct agnes_tally_args {
    agnes_vote_batch vb;
    const int64_t* power;       /* [n_sets][n_vals] */
    const uint32_t* power32;    /* low 32 bits, used by fast instances */
    const agnes_set_info* sets; /* [n_sets] */
    uint32_t n_sets;
    uint32_t n_vals;
    uint32_t max_rounds;
    uint32_t flags;
    uint8_t* codes;
    agnes_state* states;          /* out (and in, when states_in is null) */
    const agnes_state* states_in; /* optional: the States before the call (the sweep route reads them here) */
    agnes_carry_rec* carry; /* optional [n_instances][2*max_rounds], in/out */
    unsigned long long* n_invalid;
    uint32_t* list;       /* deferred instances (fast kernel -> wide kernel), n_instances */
    uint32_t* walk;       /* sweep: instances of batches that are not one vote stream, n_instances */
    uint32_t* list_count;
    uint32_t epoch_shift; /* bits of a vote's index inside its instance (DEDUP/SKIP tables) */
    uint32_t set_cache;   /* bytes of block LDS caching the set constants (0: read them from HBM);
                             set by the launcher only when it costs no occupancy */
    uint32_t power_cache; /* bytes of block LDS holding the u32 power table (0: gather from HBM) */
    uint32_t one_inst;    /* AGNES_FLAG_ONE_INSTANCE: every segment is a slice of instance one_id */
    uint32_t one_id;
    uint32_t batch;       /* flow: instances per work-queue batch (0: the kernel's FB) */
    uint32_t tail_batch;  /* flow: instances per batch of the queue's tail (0: the SMALLB tail) */
    uint32_t tail_n;      /* flow: instances in the tail (the last ones)                        */
    uint32_t w64;         /* the u64 fast domain (agnes_set_info.w64 sets outside the u32 one):
                             tally_fast with u64 sums, the apply pass tests the same deferral */
    uint32_t edges;       /* agnes_tally_edges: ev_counts / rec_out are the edge summary's (EDG) */
    uint32_t gate;        /* flow: 0 runs; 1 returns at once when flow_prep found an unaligned
                             instance offset, 2 when it found none */
    uint32_t prep_zero;   /* flow_prep zeroes the counters (the caller skipped their memset) */
    uint64_t* edge_counts; /* optional (agnes_tally_edges on the split per-instance route): apply_codes
                              also writes each instance's edges to edge_out's segments and their
                              counts here (the instances it defers to the LIST kernel excepted) */
    void* edge_out;
    void* rec_out;        /* optional (agnes_tally_records): agnes_seg_event [n_votes], instance i's
                             records at [offsets[i], offsets[i] + ev_counts[i]) -- the flow
                             kernel writes them (REC); every other route's emit pass does */
    uint64_t* ev_counts;  /* optional [n_instances]: the flow kernel writes each instance's event
                             record count (agnes_tally_events); instances it hands to the walk
                             list are left to agnes_launch_event_count_list */
} agnes_tally_args;

/* agnes_kernel_timing: HIP events around each launch while enabled (agnes_api.cpp) */
extern "C" void agnes_kt_mark(const char* name, hipStream_t st, bool begin);
struct AgnesKt {
    const char* name;
    hipStream_t st;
    AgnesKt(const char* n, hipStream_t s) : name(n), st(s) { agnes_kt_mark(name, st, true); }
    ~AgnesKt() { agnes_kt_mark(name, st, false); }
};

/* bytes of dynamic LDS one wave uses */
int64_t agnes_lds_per_wave(uint32_t mode, uint32_t flags, uint32_t max_rounds, uint32_t n_vals);

/* launchers (agnes_kernels.hip) — enqueue only */
/* wide_all: every instance on the i64 path (caller weights, carried executors or
 * a power set outside the fast domain); else the u32 kernel runs first and
 * defers the instances it cannot prove to the i64 list kernel */
hipError_t agnes_launch_tally(const agnes_tally_args* a, uint32_t mode, int num_cus, bool wide_all,
                              hipStream_t stream);
/* the u32 fast-path kernel (agnes_fast.hip): every instance it can prove stays
 * below 2^31, the rest appended to a->list for the i64 LIST kernel */
hipError_t agnes_launch_tally_fast(const agnes_tally_args* a, uint32_t mode, int num_cus,
                                   hipStream_t stream);
/* the fused sweep kernel (agnes_sweep.hip): REFERENCE mode without RoundSkip, tally
 * and State machine in one pass; same deferral protocol */
bool agnes_sweep_supported(const agnes_tally_args* a);
hipError_t agnes_launch_sweep(const agnes_tally_args* a, int num_cus, hipStream_t stream);
/* the 8-votes-per-lane flow kernel (agnes_flow.hip) for the sweep route's streams */
bool agnes_flow_supported(const agnes_tally_args* a);
/* rg: the kernel that also holds the unaligned-stream loop -- a batch whose offsets are
 * not all multiples of 4 is walked by it unless one of its instances holds 1 .. 7 votes
 * (then: the walk list; without rg every such batch goes there); the u64 kernel's holds
 * that loop only */
hipError_t agnes_launch_flow(const agnes_tally_args* a, int num_cus, hipStream_t stream, bool rg);
/* flow_prep: the gate words (AGNES_PREP_SLOT0) for a.gate, and (a.prep_zero) the counters
 * zeroed in the same launch */
hipError_t agnes_launch_flow_prep(const agnes_tally_args* a, hipStream_t stream);
bool agnes_flow_rg_build();
/* the u32 flow route has the unaligned-stream kernel (AGNES_FLOW_RG builds) */
bool agnes_flow_rg(const agnes_tally_args* a);
/* the segmented records (agnes_tally_records) of every instance, or of the ones on a
 * list (the flow route's walk list; list_n on the device), one lane per instance; and
 * the dense stream from them (offs: the exclusive scan of the counts) */
/* (agnes_tally_records, routes without the fused records) the emit pass writing the
 * segmented records and the counts (no count pass); the columns 16-B aligned and
 * 2 * max_rounds <= 64 (agnes_seg_emit_ok), else the walk */
bool agnes_seg_emit_ok(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds);
hipError_t agnes_launch_seg_emit(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds, uint32_t mult,
                                 uint64_t* counts, void* seg, hipStream_t st);
hipError_t agnes_launch_seg_walk(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds, uint32_t mult,
                                 const uint32_t* list, const uint32_t* list_n, uint64_t* counts, void* seg,
                                 hipStream_t stream);
/* (the dense writers: out holds cap records; the ones past cap or past their segment's end
 * offset are dropped and counted in *ovf -- agnes_records_overflow) */
hipError_t agnes_launch_seg_compact(const agnes_vote_batch* vb, uint32_t mult, const void* seg, const uint64_t* offs,
                                    agnes_vote_event* out, hipStream_t stream, uint64_t cap, unsigned long long* ovf);
/* the same for the edge summary (agnes_tally_edges / agnes_edges_compact) */
hipError_t agnes_launch_edge_seg_walk(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds,
                                      const uint32_t* list, const uint32_t* list_n, uint64_t* counts, agnes_edge* seg,
                                      hipStream_t stream);
hipError_t agnes_launch_edge_compact(const agnes_vote_batch* vb, const agnes_edge* seg, const uint64_t* offs,
                                     agnes_edge* out, hipStream_t stream, uint64_t cap, unsigned long long* ovf);
/* the flow kernel can count event records (agnes_tally_events) in this configuration */
bool agnes_flow_counts_events(uint32_t flags, uint32_t max_rounds, bool edges = false, bool rec = false);
/* the batched State::apply pass over the codes a tally kernel left (agnes_apply.hip):
 * one instance per lane, skipping the instances deferred to the LIST kernel */
bool agnes_apply_codes_supported(const agnes_tally_args* a);
/* apply_codes can write the edges too (keys = 2 * max_rounds <= 16: the executor bytes in
 * two registers) */
bool agnes_apply_edges_supported(uint32_t max_rounds);
hipError_t agnes_launch_apply_codes(const agnes_tally_args* a, hipStream_t stream);
int64_t agnes_fast_lds_per_wave(uint32_t mode, uint32_t flags, uint32_t max_rounds, uint32_t n_vals);
hipError_t agnes_launch_apply_events(agnes_state* states, uint32_t n, const uint64_t* off,
                                     const agnes_event* ev, agnes_message* msgs, uint32_t flags,
                                     hipStream_t stream);
hipError_t agnes_launch_apply_msgs(const agnes_vote_batch* vb, const uint8_t* kind, const int32_t* pol,
                                  const int64_t* power, const agnes_set_info* sets, uint32_t n_sets, uint32_t n_vals,
                                  uint32_t max_rounds, uint32_t flags, agnes_state* states, agnes_message* msgs,
                                  uint8_t* codes, unsigned long long* n_invalid, hipStream_t stream);
/* pass 0 scan, 1 apply, 2 finish (agnes_onesm.hip) */
hipError_t agnes_launch_one_sm(int pass, const uint8_t* codes, const uint8_t* round, const uint32_t* value, uint64_t n,
                               uint64_t base, agnes_state* state, int64_t* marks, int num_cus, hipStream_t stream);
/* validator sets (agnes_valset.hip) */
hipError_t agnes_launch_valset_build(const uint8_t* addr, uint32_t addr_len, const int64_t* power, const uint32_t* set_of,
                                     uint32_t n, uint32_t n_sets, uint32_t* idx, uint32_t N, uint64_t* pos,
                                     uint64_t* scan_scratch, uint32_t* set_out, uint32_t* order, int64_t* power_out,
                                     uint8_t* addr_out, uint64_t* set_offsets, int64_t* totals, hipStream_t st);
hipError_t agnes_launch_valset_find(const uint8_t* sorted_addr, uint32_t addr_len, const uint64_t* set_offsets,
                                    uint32_t n_sets, const uint8_t* q_addr, const uint32_t* q_set, uint64_t n_q,
                                    uint64_t* out, hipStream_t st);
struct agnes_wire_args {
    const agnes_wire_vote* records;
    uint64_t n;
    const uint8_t* pubkeys;
    uint32_t n_sets, n_vals;
    const uint32_t* instance_set;
    uint32_t n_instances, max_rounds;
    int64_t height;
    uint32_t *instance, *value, *validator;
    uint8_t *round, *type, *verdict;
    const int32_t* base_table; /* agnes_launch_wire_table's output */
};
hipError_t agnes_launch_wire_ingest(const agnes_wire_args* a, hipStream_t st);
size_t agnes_wire_table_bytes(void);
hipError_t agnes_launch_wire_table(int32_t* table, hipStream_t st);
hipError_t agnes_launch_gen(const agnes_gen_params* p, const uint64_t* d_offsets, uint64_t n_votes,
                            uint32_t* instance, uint8_t* round, uint8_t* type, uint32_t* value,
                            uint32_t* validator, hipStream_t stream);

/* the edge summary (agnes_edges.hip): out == nullptr -> count pass + exclusive scan of
 * offs (scratch: agnes_edges_scratch_words u64); else the emit pass */
uint64_t agnes_edges_scratch_words(uint32_t n_instances);
/* offs[1..n] := inclusive scan of the per-instance counts (offs[0] = 0 left as is) */
hipError_t agnes_launch_offsets_scan(uint64_t* offs, uint32_t n, uint64_t* scratch, hipStream_t stream);
/* the fold of one instance's slices' VoteCounts (agnes_fold.hip) */
hipError_t agnes_launch_fold(agnes_vote_count* counts, uint32_t n_slices, uint32_t keys,
                             const agnes_vote_count* carry, agnes_vote_count* totals, uint32_t flags,
                             hipStream_t stream);
/* the event stream (agnes_events.hip): out == nullptr -> count pass + scan, else emit */
hipError_t agnes_launch_partials(const agnes_vote_batch* vb, const int64_t* power, const uint32_t* power32,
                                 const agnes_set_info* sets, uint32_t n_sets, uint32_t n_vals,
                                 uint32_t max_rounds, uint32_t one_inst, uint32_t one_id, agnes_carry_rec* counts,
                                 int64_t* weights, hipStream_t st);
hipError_t agnes_launch_events(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds,
                               uint64_t* offs, agnes_vote_event* out, uint64_t* scratch, hipStream_t stream,
                               uint64_t cap = 0, unsigned long long* ovf = nullptr);
/* the event-record counts of the instances on a tally's walk list (walk[0 .. *walk_n)),
 * into offs[1 + instance]: the ones the flow kernel did not count */
hipError_t agnes_launch_event_count_list(const agnes_vote_batch* vb, const uint8_t* codes, const uint32_t* walk,
                                         const uint32_t* walk_n, uint64_t* offs, int num_cus, hipStream_t stream);
hipError_t agnes_launch_edges(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds,
                              uint64_t* offs, agnes_edge* out, uint64_t* scratch, hipStream_t stream,
                              uint64_t cap = 0, unsigned long long* ovf = nullptr);

/* DEDUP for a split instance (agnes_dedup.hip): type_out == nullptr -> the first-seen
 * pass into first[], else the mask pass; reject rewrites the masked votes' codes */
hipError_t agnes_launch_dedup(const agnes_vote_batch* vb, uint32_t inst_id, uint32_t max_rounds,
                              uint32_t n_vals, bool set_ok, uint64_t base, uint64_t* first,
                              uint8_t* type_out, hipStream_t stream);
/* the same first-index table without global atomics (a counting sort by key bucket and
 * LDS minima): when agnes_dedup_bucketed; scratch: agnes_dedup_scratch_bytes */
bool agnes_dedup_bucketed(uint64_t n_votes, uint32_t max_rounds, uint32_t n_vals);
uint64_t agnes_dedup_scratch_bytes(uint64_t n_votes, uint32_t max_rounds, uint32_t n_vals);
/* type_out != nullptr (agnes_dedup_first_mask): also the mask, for a batch that is the
 * whole stream (no other slice's votes min-combined into first afterwards) */
hipError_t agnes_launch_dedup_first_bucketed(const agnes_vote_batch* vb, uint32_t inst_id, uint32_t max_rounds,
                                             uint32_t n_vals, bool set_ok, uint64_t base, uint64_t* first,
                                             uint8_t* type_out, void* scratch, hipStream_t stream);
/* first[0 .. n) := INT64_MAX */
hipError_t agnes_launch_dedup_fill(uint64_t* first, uint64_t n, hipStream_t stream);
hipError_t agnes_launch_dedup_reject(const uint8_t* type_masked, uint64_t n, uint8_t* codes, hipStream_t stream);

#define AGNES_WAVES_PER_BLOCK 4
/* list_count[0] counts the deferred (i64 LIST) list; list_count[1 .. AGNES_QUEUE_N] are
 * the u32 kernels' work-queue counters; list_count[AGNES_WALK_COUNT] counts the sweep's
 * walk list and list_count[AGNES_WALK_QUEUE] is the walk kernel's queue counter; they
 * follow the invalid-vote count in one device block, zeroed by one memset per call.
 * The invalid-vote count is AGNES_ERR_STRIPES u64 stripes AGNES_ERR_STRIDE bytes
 * apart: a wave adds its count to its block's stripe (add_invalid) — a thousand waves
 * adding to ONE address serialize at the memory side (10 us of C5d's 45-us pass B,
 * measured) — and agnes_last_error_count sums the stripes. */
#define AGNES_QUEUE_N 256
#define AGNES_WALK_COUNT (AGNES_QUEUE_N + 1)
#define AGNES_WALK_QUEUE (AGNES_QUEUE_N + 2)
/* flow_prep's words, one per block of it (every one written on every call): whether
 * its share of the instance offsets holds one off a multiple of 4 */
#define AGNES_PREP_SLOT0 (AGNES_QUEUE_N + 4)
#define AGNES_PREP_SLOTS 256
#define AGNES_QUEUE_WORDS (AGNES_QUEUE_N + 4 + AGNES_PREP_SLOTS)
#define AGNES_ERR_STRIPES 32
#define AGNES_ERR_STRIDE 512
#define AGNES_ERR_BYTES (AGNES_ERR_STRIPES * AGNES_ERR_STRIDE)
#define AGNES_COUNTER_BYTES (AGNES_ERR_BYTES + AGNES_QUEUE_WORDS * 4)
/* one wave's invalid votes into its block's stripe of the count */
__device__ __forceinline__ void add_invalid(unsigned long long* n_invalid, unsigned long long n) {
    atomicAdd(n_invalid + (blockIdx.x % AGNES_ERR_STRIPES) * (AGNES_ERR_STRIDE / 8u), n);
}
#define AGNES_MAX_LDS_PER_WAVE (36 * 1024)

#endif
