/*
 * agnes_flow.hip — the hot path for REFERENCE batches without RoundSkip (BASELINE
 * C2/C3): ingest -> weight gather -> ordered tally -> quorum -> event ->
 * State::apply, ONE pass over the votes (consensus_executor.rs:61-69).
 *
 * A work queue hands out batches of up to FB consecutive instances.  A batch whose
 * offsets are multiples of 4 and whose instances are in the flow domain (u32 power
 * set, maxpow < 4096, len * maxpow < 2^30) is walked as ONE vote stream in 512-vote
 * chunks: lane l holds votes 8l .. 8l+7, as two 4-vote UNITS (A, B).  Instance
 * starts are multiples of 4, so a unit never straddles an instance; a lane can
 * (the instance of its unit B started inside the lane: a SPLIT lane).  Any other
 * batch goes to the walk list (agnes_sweep.hip) with its States copied through.
 *
 * Per chunk (VALU per vote is what bounds the kernel, so the per-vote work is
 * lane-serial with transient masks and every wave-level step is shared by 512
 * votes):
 *   K1   validation (bit tests per unit, SWAR on the round/type bytes), weight
 *        gather from the power table (block LDS copy when it fits, else L2);
 *   K2   per round present: one lane-serial prefix of the four buckets of the
 *        round's RoundVotes (prevote / precommit x value / nil, round_votes.rs:
 *        48-56), packed as 16-bit fields of one 64-bit accumulator (a vote adds
 *        w << (32 * precommit + 16 * nil): one shift and one add); four DPP wave
 *        scans of the lanes' last-segment totals; a segment's running sum is
 *        scan - base + carry;
 *   K3   per vote is_quorum on its own type's sums (round_votes.rs:31-33) with
 *        precedence Value > Nil > Any > Init (:58-66) as a level 0..3, and
 *        to_event (vote_executor.rs:26-36) as one byte lookup by (type, level);
 *   K4   State::apply for the vote events (state_machine.rs:196-211).  Without
 *        RoundSkip the step moves only at P1 (the first PolkaNil / PolkaValue at
 *        State.round while in Prevote, :197-198) and at C (the first
 *        PrecommitValue, any round, :211).  Every unit lowers its instance's P1 and
 *        C positions by an LDS atomic min, reads them back, and derives every
 *        message from the vote's position relative to them: TimeoutPrevote before
 *        P1 in Prevote (:196), TimeoutPrecommit before C (:208), the precommit at
 *        P1, the Decision at C.  valid (:198, :202) is the last PolkaValue at
 *        State.round at or after P1 (or from the start, entering in Precommit)
 *        before C: an LDS atomic max of (position, value) over the non-nil ones
 *        (in this domain a nil PolkaValue's label is the last non-nil one's,
 *        round_votes.rs:50-54, and P1 / C are crossed by non-nil votes).
 */
#include <type_traits>

#include "agnes_fast.h"

namespace agnes {
namespace flow {
using namespace agnes::fast;

constexpr uint32_t LV = 8u, CH = 64u * LV; /* votes per lane, per chunk */

/* Diagnostics build only (AGNES_FLOW_DIAG, tools/flowdiag.py): per wave, 64 u64 words --
 * [0] s_memrealtime at the start (100 MHz), [1] at the end, [2] batches, [3] chunks, then
 * per batch k < 30: [4 + 2k] its start time, [5 + 2k] instances | chunks << 16 | votes << 32. */
#ifdef AGNES_FLOW_DIAG
__device__ unsigned long long* flow_diag_buf;
#define FDIAG(...) __VA_ARGS__
#else
#define FDIAG(...)
#endif
/* DMA slot: each column of the chunk as a contiguous image */
constexpr uint32_t F_INST = 0, F_VALUE = 2048, F_VAL = 4096, F_ROUND = 6144, F_TYPE = 6656, F_BYTES = 7168;
/* instances per batch: header offsets in lanes 0..FB, per-instance data in lane k.  A
 * batch's stream ends in a partial chunk, so the bigger the batch the fewer idle lanes
 * (C2: 16 instances = 3,200 votes in 7 chunks, 32 = 6,400 in 13) */
#ifndef AGNES_FLOW_TAIL_DIV
#define AGNES_FLOW_TAIL_DIV 16 /* the queue's tail: 1/16 of the instances in SMALLB batches */
#endif
#ifndef AGNES_FLOW_BATCHES_PER_WAVE
#define AGNES_FLOW_BATCHES_PER_WAVE 4 /* batches per wave the batch size leaves (0: always FB); c3shard A/B 4 vs FB: flow 0.362 vs 0.444 ms */
#endif
#ifndef AGNES_FLOW_TAIL_VOTES
#define AGNES_FLOW_TAIL_VOTES 0 /* votes per batch of the queue's tail (0: the SMALLB tail; 1024 measured 2 % slower on C3 / c3shard) */
#endif
#ifndef AGNES_FLOW_TAIL_PER_WAVE
#define AGNES_FLOW_TAIL_PER_WAVE 2
#endif
#ifndef AGNES_FLOW_AHEAD
#define AGNES_FLOW_AHEAD 1 /* batches a wave holds claimed beyond the current one (1 or 2) */
#endif
#ifndef AGNES_FLOW_FAST_START
#define AGNES_FLOW_FAST_START 1 /* static first batches, the first chunk's DMA before the set constants */
#endif
#ifndef AGNES_FLOW_QN
#define AGNES_FLOW_QN AGNES_QUEUE_N /* work-queue counters (the blocks of one share its batches) */
#endif
static_assert(AGNES_FLOW_QN >= 1 && AGNES_FLOW_QN <= AGNES_QUEUE_N, "flow queue counters");
#ifndef AGNES_FLOW_SMALLB
#define AGNES_FLOW_SMALLB 4
#endif
constexpr uint32_t FB = 32u;
constexpr uint32_t SMALLB = AGNES_FLOW_SMALLB; /* batch size of the work queue's tail       */
/* instance record, 12 words: quorum threshold, power-row base, validators of its set
 * (0: no such set); the State machine's view: the roles its step keeps (one byte per
 * vote, 0 without the State machine), State.round in every byte, 0xFF bytes when it
 * enters in Precommit (valid from the start); the P1 and C positions (stream-relative,
 * ~0: none); decision round | F_LOCK (P1 was a PolkaValue); step.  The last valid
 * candidate is kept beside (vtab: position + 1 << 32 | its value, an LDS u64 max); the
 * locked and decision values go straight into the staged States when P1 / C are
 * found (the vote's value is still in registers). */
constexpr uint32_t R_Q2 = 0, R_PBASE = 1, R_NV = 2, R_EQ8 = 3, R_SMASK = 4, R_EQ = 5, R_VALL = 6, R_STEP = 7, R_P1 = 8,
                   R_C = 9, R_DF = 10, R_DR = 11, RECW = 12;
/* (W64) the threshold's high word; 16-word records */
constexpr uint32_t R_Q2H = 12, RECW64 = 16;
constexpr uint32_t F_LOCK = 0x100u;
constexpr uint32_t NONE = 0xFFFFFFFFu;

/* K4 roles of a vote event (byte lookup by v_perm, index = event code 0..7) */
constexpr uint32_t X_P1 = 0x01u, X_C = 0x02u, X_TP = 0x04u, X_TC = 0x08u, X_PV = 0x10u;
constexpr uint32_t XT_LO = (0u) | (X_TP << 8) | (X_P1 << 16) | ((X_P1 | X_PV) << 24); /* None, PolkaAny, PolkaNil, PolkaValue */
constexpr uint32_t XT_HI = (X_TC) | (X_C << 8);                                      /* PrecommitAny, PrecommitValue */
/* roles kept per step (byte lookup by step 0..7): NewRound / Propose: TimeoutPrecommit
 * and commit only (:208, :211); Prevote: all; Precommit: no P1 / TimeoutPrevote; Commit: none (:205) */
constexpr uint32_t SM_LO = (X_C | X_TC) | ((X_C | X_TC) << 8) | (0x1Fu << 16) | ((X_C | X_TC | X_PV) << 24);
constexpr uint32_t SM_HI = 0u;
/* to_event by index type * 4 + level (Init, Any, Nil, Value): vote_executor.rs:26-36 */
constexpr uint32_t EV_LO = AGNES_CODE_NONE | (AGNES_CODE_POLKA_ANY << 8) | (AGNES_CODE_POLKA_NIL << 16) |
                           (AGNES_CODE_POLKA_VALUE << 24);
constexpr uint32_t EV_HI = AGNES_CODE_NONE | (AGNES_CODE_PRECOMMIT_ANY << 8) | (AGNES_CODE_NONE << 16) |
                           (AGNES_CODE_PRECOMMIT_VALUE << 24);

/* (REC) each carried row also holds the executors' value slots vl[2R] (u32): the last
 * non-nil value an executor took, round_votes.rs:50-54 */
__host__ __device__ inline uint32_t carry_bytes(uint32_t R, bool w64 = false, bool rec = false) {
    return (uint32_t)align16((w64 ? 64ull : (rec ? 48ull : 32ull)) * R);
}
/* per-wave LDS: DMA slot | carried executors (2 copies x (vw[2R], vn[2R]) u32, or u64
 * for W64) | instance records | (State machine) valid candidates, two batches' staged States */
__host__ __device__ inline uint32_t lds_bytes(bool sm, uint32_t R, bool evc = false, bool w64 = false, bool edg = false,
                                              bool rec = false) {
    return F_BYTES + carry_bytes(R, w64, rec) + FB * (w64 ? RECW64 : RECW) * 4u + (sm ? FB * 8u + 2u * FB * 64u : 0u) +
           (evc ? FB * 4u : 0u) + (edg ? (uint32_t)align16(FB * 2ull * R) : 0u) + (rec ? (uint32_t)align16(16ull * R) : 0u);
}

/* a State out (plain stores: non-temporal ones measured slower on C2) */
__device__ __forceinline__ void st_out(uint4* p, uint4 v) { *p = v; }
__device__ __forceinline__ uint32_t zero_marks(uint32_t x) { /* 0x80 in the bytes of x that are zero */
    const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    return ((t | x) & 0x80808080u) ^ 0x80808080u;
}
__device__ __forceinline__ uint32_t nz_marks(uint32_t x) { /* 0x80 in the bytes of x that are not zero */
    return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
__device__ __forceinline__ uint32_t mark_bytes(uint32_t m) { /* 0x80 marks -> 0xFF bytes (no multiply) */
    return (m << 1) - (m >> 7);
}
__device__ __forceinline__ uint32_t rep4(uint32_t b) { /* byte 0 of b in every byte */
    return __builtin_amdgcn_perm(0u, b, 0u);
}
__device__ __forceinline__ uint32_t below_bytes(int32_t i) { /* 0xFF in the bytes below byte i, i clamped to 0..4 */
    return i <= 0 ? 0u : (i >= 4 ? 0xFFFFFFFFu : (1u << (8u * (uint32_t)i)) - 1u);
}
__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t wave_or(uint32_t x) { /* every lane active */
    x |= dpp<0x111, 0xf>(x);
    x |= dpp<0x112, 0xf>(x);
    x |= dpp<0x114, 0xf>(x);
    x |= dpp<0x118, 0xf>(x);
    x |= dpp<0x142, 0xa>(x);
    x |= dpp<0x143, 0xc>(x);
    return rdl(x, 63u);
}
/* saddr forms: address = uniform 64-bit base + 32-bit lane offset; the vote
 * columns are read once (non-temporal) */
/* (a stream's first or last chunk: the base goes through readfirstlane, so the "s" operand
 * stays an SGPR pair whatever the compiler's uniformity analysis concludes about it) */
__device__ __forceinline__ void sdma16(const void* base, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    const uint64_t b = rfl64((uint64_t)(uintptr_t)base);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(b), "s"(lds)
                 : "memory");
}
__device__ __forceinline__ void sdma4(const void* base, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    const uint64_t b = rfl64((uint64_t)(uintptr_t)base);
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(b), "s"(lds)
                 : "memory");
}
/* a whole chunk: the five columns, each column's two 256-vote halves under ONE m0 (the
 * instruction offset moves the global and the LDS address alike), m0 saved once */
__device__ __forceinline__ void sdma_chunk(const void* bi, const void* bv, const void* bd, const void* br,
                                           const void* bt, uint32_t o16, uint32_t o4, uint32_t slotl) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\t"
                 "s_mov_b32 m0, %8\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %3 nt\n\tglobal_load_lds_dwordx4 %1, %3 offset:1024 nt\n\t"
                 "s_mov_b32 m0, %9\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %4 nt\n\tglobal_load_lds_dwordx4 %1, %4 offset:1024 nt\n\t"
                 "s_mov_b32 m0, %10\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, %5 nt\n\tglobal_load_lds_dwordx4 %1, %5 offset:1024 nt\n\t"
                 "s_mov_b32 m0, %11\n\ts_nop 0\n\t"
                 "global_load_lds_dword %2, %6 nt\n\tglobal_load_lds_dword %2, %6 offset:256 nt\n\t"
                 "s_mov_b32 m0, %12\n\ts_nop 0\n\t"
                 "global_load_lds_dword %2, %7 nt\n\tglobal_load_lds_dword %2, %7 offset:256 nt\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(o16), "v"(o4), "s"(bi), "s"(bv), "s"(bd), "s"(br), "s"(bt), "s"(slotl + F_INST),
                   "s"(slotl + F_VALUE), "s"(slotl + F_VAL), "s"(slotl + F_ROUND), "s"(slotl + F_TYPE)
                 : "memory");
}
/* the codes are written once and not read again by the step: non-temporal stores
 * (same-box A/B: C2 flow 0.643 -> 0.613 ms, C3 -1..3 %) */
__device__ __forceinline__ void sstore4(void* base, uint32_t voff, uint32_t d) {
    asm volatile("global_store_dword %0, %1, %2 nt" ::"v"(voff), "v"(d), "s"(base) : "memory");
}
__device__ __forceinline__ void sstore8(void* base, uint32_t voff, uint32_t d0, uint32_t d1) {
    asm volatile("global_store_dwordx2 %0, %1, %2 nt" ::"v"(voff), "v"(u64of(d0, d1)), "s"(base) : "memory");
}

/* a batch: instances [s0, e0).  Its header is built in three stages, each one
 * chunk apart so that its loads land behind the chunk DMA's wait: (1) offsets
 * (lanes 0..m, clamped to n_votes) and sets (lanes k < m) requested; (2) lengths
 * and the checks on the offsets, the sets' constants requested; (3) the quorum
 * thresholds and whether the batch is one flow stream. */
struct Hdr {
    uint32_t s0, e0;
    uint32_t olo, ohi;  /* lanes 0..m: offset                                     */
    uint32_t hs;        /* lane k < m: the power set of instance k                */
    uint32_t q2, mp;    /* lane k: set q2, maxpow; after stage 3 q2 = threshold   */
    uint32_t q2h, mph;  /* (W64) their high words                                */
    uint32_t fa, ln;    /* lane k: set fast flag (W64: w64 flag; 2: no such set), length */
    uint32_t stage;     /* 1, 2, 3 (ready)                                       */
    uint32_t stream;    /* stage 2: the offsets pass; stage 3: walked by this kernel */
    uint32_t rag;       /* stage 2: some offset is not a multiple of 4 (the U kernel's batch);
                           (U) 2: it also holds an instance of 1 .. 7 votes (the walk list) */
    uint32_t go;        /* stage 3: this kernel walks it as one stream                        */
};

/* EVC: also the number of event records of each instance of a flow batch (votes whose
 * code is Some(Event), 1..5: this route never sets the RoundSkip bit) into
 * a.ev_counts[instance] -- the count pass of the event stream (agnes_events.hip) */
/* W64 (one round, round 4): the u64 domain (agnes_fast.h defer_si) — weights from the
 * i64 power table and the four buckets of K2 as u64 sums instead of 16-bit fields */
#ifndef AGNES_FLOW_W64_WPE
#define AGNES_FLOW_W64_WPE 2
#endif
#ifndef AGNES_FLOW_WPE
#define AGNES_FLOW_WPE 3
#endif
#ifndef AGNES_FLOW_RG
#define AGNES_FLOW_RG 1 /* the u32 kernels also walk unaligned streams (0, A/B builds: they go to the walk list) */
#endif
#ifndef AGNES_FLOW_FORCE_U
#define AGNES_FLOW_FORCE_U 0 /* A/B builds only: every stream through the unaligned-stream loop */
#endif
#ifndef AGNES_FLOW_CODE_VMCNT
#define AGNES_FLOW_CODE_VMCNT 1
#endif
#ifndef AGNES_FLOW_XWPE
#define AGNES_FLOW_XWPE 3 /* the records / edges variants, one round */
#endif
#ifndef AGNES_FLOW_XWPE_R
#define AGNES_FLOW_XWPE_R 3 /* ... several rounds: a few spills at 3 waves per SIMD cost less than
                             * 2 waves (C3 records 4.89 -> 4.11 ms, its shard 0.75 -> 0.64) */
#endif
#ifndef AGNES_FLOW_EWPE_R
#define AGNES_FLOW_EWPE_R 2 /* the edges, several rounds: at 3 waves their spills cost more
                             * (C3 edges 3.85 -> 4.30 ms) */
#endif
/* REC (agnes_tally_records): the event records themselves, segmented by instance.
 * EDG (agnes_tally_edges): the edge summary instead -- etab counts each instance's
 * edges and the 16-B agnes_edge records go to the instance's segment (agnes_edges.hip's
 * definition, orc_edges: a valid vote is an edge when its executor's state, level |
 * last message << 4, changes). */
/* RG (round 6): the kernel also walks the batches whose instance offsets are NOT all
 * multiples of 4 -- the ragged streams of validator sets with absent validators -- in a
 * second copy of the chunk loop (U), chosen per batch.  Its lane's eight votes split at any
 * position: the instance (or, in runs mode, the round run) starting inside the lane owns
 * votes sp .. 7 (its PART B), the one running into the lane votes 0 .. sp - 1 (PART A);
 * the per-vote choices the aligned loop makes by the unit (vote < 4) it makes by the part
 * (vote < sp).  Every instance of such a batch holds 0 or at least 8 votes, so a lane holds
 * at most one instance start (else the batch goes to the walk list).  The aligned loop's
 * code is the same whether the kernel holds the other one or not; the two share the queue,
 * so a batch costs nothing in the loop that does not walk it. */
template <bool PC, bool SM, bool R1, bool EVC, bool W64, bool REC = false, bool EDG = false, bool RG = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W64 ? AGNES_FLOW_W64_WPE : ((REC || EDG) ? (R1 ? AGNES_FLOW_XWPE : (EDG ? AGNES_FLOW_EWPE_R : AGNES_FLOW_XWPE_R)) : AGNES_FLOW_WPE)))) void flow(agnes_tally_args a, uint32_t lds_per_wave) {
    static_assert(!REC || (EVC && !W64), "records: with the record counts, u32 sums");
    static_assert(!EDG || (EVC && !W64 && !REC), "edges: the counts are the edges', u32 sums");
    static_assert(!RG || !W64, "unaligned streams: u32 sums");
    /* the gate (flow_prep's words, 4 per lane): the aligned kernel runs when every instance
     * offset is a multiple of 4, the RG one (its register allocation holds both loops, which
     * costs the aligned loop ~2-5 %) when some is not */
    if (a.gate) {
        static_assert(AGNES_PREP_SLOTS == 256 && AGNES_PREP_SLOT0 % 4 == 0, "the gate: one uint4 per lane");
        const uint4 f = reinterpret_cast<const uint4*>(a.list_count + AGNES_PREP_SLOT0)[lane_id()];
        if ((ballot((f.x | f.y | f.z | f.w) != 0u) != 0ull) != (a.gate == 2u)) return;
    }
    constexpr uint32_t RW = W64 ? RECW64 : RECW; /* record words */

    const uint32_t lane = lane_id();
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint32_t R = R1 ? 1u : a.max_rounds, nv = a.n_vals, ns = a.n_sets, n = a.vb.n_instances;
    const uint64_t NV = a.vb.n_votes;
    const uint32_t o32 = 32u * lane, o16 = 16u * lane, o8 = 8u * lane, o4 = 4u * lane;

    /* block-shared power table, u32 (W64: the i64 one) — launcher-staged only when it
     * costs no occupancy */
    if (PC) {
        const uint32_t np = ns * nv;
        if (W64) {
            uint64_t* pc = reinterpret_cast<uint64_t*>(agnes_smem);
            for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) pc[k] = (uint64_t)a.power[k];
        } else {
            uint32_t* pc = reinterpret_cast<uint32_t*>(agnes_smem);
            for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) pc[k] = a.power32[k];
        }
        __syncthreads();
    }
    unsigned char* const base = agnes_smem + a.power_cache + wave * lds_per_wave;
    unsigned char* const slot = base;
    const uint32_t slotl = lds_addr(slot);
    uint32_t* const crow = reinterpret_cast<uint32_t*>(base + F_BYTES);
    const uint32_t cw = (W64 ? 8u : (REC ? 6u : 4u)) * R; /* one carry copy: vw[2R], vn[2R] (u32 words), (REC) vl[2R] */
    const uint32_t CB = carry_bytes(R, W64, REC);
    uint32_t* const itab = reinterpret_cast<uint32_t*>(base + F_BYTES + CB);
    unsigned long long* const vtab = reinterpret_cast<unsigned long long*>(base + F_BYTES + CB + FB * RW * 4u);
    unsigned char* const sb = base + F_BYTES + CB + FB * RW * 4u + FB * 8u;
    uint32_t* const etab = reinterpret_cast<uint32_t*>(base + F_BYTES + CB + FB * RW * 4u +
                                                       (SM ? FB * 8u + 2u * FB * 64u : 0u)); /* (EVC) records */
    /* (EDG) each executor's edge state after the votes so far, [instance][round * 2 + type] bytes */
    unsigned char* const elab = reinterpret_cast<unsigned char*>(etab + FB);
    /* (REC) this chunk's last non-nil vote of each executor of the instance carried into the
     * next chunk: (position + 1) << 32 | value, an LDS max, [2R] */
    unsigned long long* const vmx = reinterpret_cast<unsigned long long*>(etab + FB);
    const agnes_state* const st_in = a.states_in ? a.states_in : a.states;
    uint32_t cpar = 0;
    uint64_t pf_at = ~0ull;
    uint32_t bad = 0;
    /* r < R <=> ((r & 0x7F) + 128 - R) < 128 and r < 128 (R <= 15) */
    const uint32_t RK = (128u - R) * 0x01010101u;

    /* ---- work queue: batches of FB, then SMALLB ones for the tail ---- */
    const uint32_t qn = gridDim.x < AGNES_FLOW_QN ? gridDim.x : AGNES_FLOW_QN;
    const uint32_t qk = blockIdx.x % qn;
    uint32_t* const ctr = a.list_count + 1u + qk;
    /* batch size: FB, or (launcher) fewer for a batch too small to give every wave
     * several batches -- the makespan is a wave's last batch */
    const uint32_t fb = a.batch && a.batch < FB ? a.batch : FB;
    /* the queue's tail: the last a.tail_n instances in batches of a.tail_batch (the
     * launcher sizes them to about AGNES_FLOW_TAIL_VOTES votes, a couple per wave, so
     * the waves of a counter finish within a small batch of each other), or (0) the
     * last 1/AGNES_FLOW_TAIL_DIV in SMALLB batches */
    const uint32_t sb_ = a.tail_batch ? (a.tail_batch < fb ? a.tail_batch : fb) : (SMALLB < fb ? SMALLB : fb);
    const uint64_t NB = a.tail_batch ? (uint64_t)(n - (a.tail_n < n ? a.tail_n : n)) / fb
                                     : (uint64_t)(n / fb) * (AGNES_FLOW_TAIL_DIV - 1u) / AGNES_FLOW_TAIL_DIV;
    auto range_of = [&](uint32_t t, uint32_t& s0, uint32_t& e0) {
        const uint64_t b = (uint64_t)t * qn + qk;
        const uint64_t s = b < NB ? b * fb : NB * fb + (b - NB) * sb_;
        const uint64_t e = s + (b < NB ? fb : sb_);
        s0 = s < n ? (uint32_t)s : n;
        e0 = e < n ? (uint32_t)e : n;
    };
    auto hdr1 = [&](Hdr& h) { /* stage 1: offsets and sets requested */
        const uint32_t m = h.e0 - h.s0;
        uint32_t lo = 0, hi = 0, hs = 0;
        if (m > 0u && lane <= m) {
            const uint64_t o = a.vb.offsets[h.s0 + lane];
            const uint64_t oc = o < NV ? o : NV;
            lo = (uint32_t)oc;
            hi = (uint32_t)(oc >> 32);
        }
        if (lane < m) {
            const uint32_t k = h.s0 + lane;
            hs = a.vb.instance_set ? a.vb.instance_set[k] : (ns ? k % ns : 0u);
        }
        h.olo = lo;
        h.ohi = hi;
        h.hs = hs;
        h.stage = 1;
        h.stream = 0;
        h.rag = 0;
        h.go = 0;
    };
    auto hdr2 = [&](Hdr& h) { /* stage 2: lengths, offset checks; set constants requested */
        const uint32_t m = h.e0 - h.s0;
        const bool il = lane < m;
        const uint64_t ob = u64of(h.olo, h.ohi);
        const uint64_t oe = u64of(shfl(h.olo, lane + 1u), shfl(h.ohi, lane + 1u));
        const uint64_t len = il && oe > ob ? oe - ob : 0ull;
        h.ln = len < (1ull << 31) ? (uint32_t)len : (1u << 31);
        /* rag: some offset off a multiple of 4 -- the U loop's batch (RG; else the walk list's),
         * 2 when an instance also holds 1 .. 7 votes (the walk list's) */
        h.rag = (RG && AGNES_FLOW_FORCE_U) || ballot(lane <= m && (h.olo & 3u) != 0u) != 0ull;
        if (RG) h.rag = h.rag ? 1u + (ballot(il && len > 0ull && len < 8ull) != 0ull) : 0u;
        uint32_t q2 = 0, mp = 0, fa = 2, q2h = 0, mph = 0;
        if (il && h.hs < ns) {
            const agnes_set_info* const si = a.sets + h.hs;
            if (W64) {
                q2 = (uint32_t)si->q2w;
                q2h = (uint32_t)(si->q2w >> 32);
                mp = (uint32_t)si->maxw;
                mph = (uint32_t)(si->maxw >> 32);
                fa = si->w64;
            } else {
                q2 = si->q2;
                mp = si->maxpow;
                fa = si->fast;
            }
        }
        h.q2 = q2;
        h.mp = mp;
        h.q2h = q2h;
        h.mph = mph;
        h.fa = fa;
        /* stream: the offsets and, at stage 3, the sets in the flow domain */
        const bool badl = lane < m && oe < ob;
        const uint64_t O0 = u64of(rdl(h.olo, 0u), rdl(h.ohi, 0u)), Om = u64of(rdl(h.olo, m), rdl(h.ohi, m));
        h.stream = m > 0u && !ballot(badl) && Om - O0 < (1ull << 30);
        h.go = 0;
        h.stage = 2u;
    };
    auto hdr3 = [&](Hdr& h) { /* stage 3: quorum thresholds; a flow stream or the walk list */
        const uint32_t m = h.e0 - h.s0;
        const bool il = lane < m;
        bool fl = true;
        uint32_t q2 = 0;
        if (il) {
            const uint64_t len = h.ln;
            if (W64 && h.fa != 2u) {
                /* u64 sums below 2^61 (defer_si's test): thresholds in two words */
                const uint64_t mw = u64of(h.mp, h.mph);
                fl = h.fa != 0u && len < (1ull << 30) && __umul64hi(len, mw) == 0ull && len * mw < (1ull << 61);
                q2 = h.q2;
            } else if (h.fa != 2u) {
                const uint64_t wmax = len * (uint64_t)h.mp; /* no sum of the instance exceeds it */
                /* u32 sums, per-lane bucket prefixes < 2^15 (8 votes x maxpow), signed thresholds */
                fl = h.fa != 0u && len < (1ull << 30) && wmax < (1ull << 30) && h.mp < 4096u;
                const uint64_t qq = (uint64_t)h.q2 < wmax ? (uint64_t)h.q2 : wmax;
                q2 = (uint32_t)(qq < 0x7FFFFFFFull ? qq : 0x7FFFFFFFull);
            } else {
                fl = len < (1ull << 30); /* no such set: every vote INVALID */
            }
        }
        h.q2 = q2;
        h.stream = h.stream && !ballot(!fl);
        h.stage = 3;
        /* this kernel walks it: the aligned streams, and (RG) the others whose instances all
         * hold 0 or >= 8 votes */
        h.go = RG ? (h.stream && h.rag != 2u) : (h.stream && !h.rag);
    };
    uint32_t spar = 0; /* States staging buffer of the current batch */
    /* the last flush sent a whole chunk's codes as ONE store with every lane active and
     * no DMA has been issued since: the chunk top's wait may leave that store in flight */
    bool dc_one = false;
    auto dma_states = [&](const Hdr& h, uint32_t par) { /* the batch's States into LDS (64 B each) */
        const uint32_t m = h.e0 - h.s0;
        dc_one = false;
        if (!SM || m == 0u) return;
        const unsigned char* const g = reinterpret_cast<const unsigned char*>(st_in + h.s0);
        glds16(g + 16u * (lane < 4u * m ? lane : 0u), sb + par * (FB * 64u));
        if (m > 16u) glds16(g + 16u * (64u + lane < 4u * m ? 64u + lane : 0u), sb + par * (FB * 64u) + 1024u);
    };
    auto dma_chunk = [&](uint64_t c, uint32_t lo, uint32_t lim) { /* the chunk's votes lo..lim into the slot */
        dc_one = false;
        __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): the slot's LDS reads are done */
        if (lo == 0u && lim >= CH) {
            sdma_chunk(a.vb.instance + c, a.vb.value + c, a.vb.validator + c, a.vb.round + c, a.vb.type + c, o16, o4,
                       slotl);
        } else { /* a stream's first or last chunk: only the 4-vote groups holding its votes
                  * load (the rest of the slot is never read as active).  An unaligned stream's
                  * first / last group also reads a neighbour's votes, inside the same 16-B
                  * aligned block of every column, so never past the columns' last page */
            if (4u * lane + 4u > lo && 4u * lane < lim) {
                sdma16(a.vb.instance + c, o16, slotl + F_INST);
                sdma16(a.vb.value + c, o16, slotl + F_VALUE);
                sdma16(a.vb.validator + c, o16, slotl + F_VAL);
                sdma4(a.vb.round + c, o4, slotl + F_ROUND);
                sdma4(a.vb.type + c, o4, slotl + F_TYPE);
            }
            if (256u + 4u * lane + 4u > lo && 256u + 4u * lane < lim) {
                sdma16(a.vb.instance + c + 256u, o16, slotl + F_INST + 1024u);
                sdma16(a.vb.value + c + 256u, o16, slotl + F_VALUE + 1024u);
                sdma16(a.vb.validator + c + 256u, o16, slotl + F_VAL + 1024u);
                sdma4(a.vb.round + c + 256u, o4, slotl + F_ROUND + 256u);
                sdma4(a.vb.type + c + 256u, o4, slotl + F_TYPE + 256u);
            }
        }
    };

    /* deferred code stores: issued behind the next chunk's gather and DMA (vmcnt
     * retires in issue order) */
    uint64_t dc_at = ~0ull;
    uint32_t dc0 = 0, dc1 = 0, dc_act = 0; /* dc_act: bit 0 unit A, bit 1 unit B active */
    uint32_t dcm0 = 0, dcm1 = 0;           /* (U) the active votes' bytes (a lane that is not all active) */
    bool dc_u = false;                     /* the deferred codes are the U loop's */
    auto flush = [&]() {
        dc_one = false;
        if (dc_at != ~0ull) {
            if (AGNES_FLOW_CODE_VMCNT && !ballot(dc_act != 3u)) {
                sstore8(a.codes + dc_at, o8, dc0, dc1);
                dc_one = true;
            } else {
                if (dc_act == 3u) {
                    sstore8(a.codes + dc_at, o8, dc0, dc1);
                } else if (RG && dc_u) { /* a stream's first or last lanes: byte stores, the neighbours' codes are another wave's */
#pragma unroll
                    for (uint32_t q = 0; q < LV; ++q)
                        if ((((q < 4u ? dcm0 : dcm1) >> (8u * (q & 3u))) & 1u) != 0u)
                            a.codes[dc_at + o8 + q] = (uint8_t)((q < 4u ? dc0 : dc1) >> (8u * (q & 3u)));
                } else if (dc_act == 1u) sstore4(a.codes + dc_at, o8, dc0);
                else if (dc_act == 2u) sstore4(a.codes + dc_at, o8 + 4u, dc1);
            }
            dc_at = ~0ull;
        }
    };

    /* a finished batch's staged States patched from its records and written out (the
     * locked / decision values are in them already, the valid one is in vtab) */
    auto finalize = [&](uint32_t mm, uint32_t s0, const unsigned char* sbp) {
        if (lane < mm) {
            const uint32_t* const rk = itab + RW * lane;
            const uint32_t p1 = rk[R_P1], cc = rk[R_C], df = rk[R_DF];
            const unsigned long long vv = vtab[lane];
            uint32_t* const sp = reinterpret_cast<uint32_t*>(const_cast<unsigned char*>(sbp) + 64u * lane);
            const uint32_t step = cc != NONE ? (uint32_t)AGNES_STEP_COMMIT
                                             : (p1 < cc ? (uint32_t)AGNES_STEP_PRECOMMIT : rk[R_STEP]);
            uint32_t fl = (sp[13] & ~0xFFu) | step;
            if (df & F_LOCK) { sp[4] = sp[2]; sp[5] = sp[3]; fl |= 1u << 8; } /* (P1 precedes any C) */
            if (vv) { sp[6] = sp[2]; sp[7] = sp[3]; sp[11] = (uint32_t)vv; fl |= 1u << 16; }
            if (cc != NONE) { sp[8] = rk[R_DR]; sp[9] = 0u; fl |= 1u << 24; }
            sp[13] = fl;
        }
        __builtin_amdgcn_wave_barrier();
        for (uint32_t j = lane; j < 4u * mm; j += 64u) st_out(reinterpret_cast<uint4*>(a.states + s0) + j,
                                                             *reinterpret_cast<const uint4*>(sbp + 16u * j));
    };

    Hdr H, N;
    uint32_t tq = 0; /* lane 0: slot of the batch after N (atomic in flight) */
#if AGNES_FLOW_FAST_START
    /* the first two batches of a wave need no atomic: the waves of counter qk (blocks
     * qk, qk + qn, ...) take static slots rank and S + rank; the counter hands out slots
     * from 2 S on */
    const uint32_t qS = ((gridDim.x - 1u - qk) / qn + 1u) * AGNES_WAVES_PER_BLOCK;
    {
        const uint32_t rank = (blockIdx.x / qn) * AGNES_WAVES_PER_BLOCK + wave;
        range_of(rank, H.s0, H.e0);
        range_of(qS + rank, N.s0, N.e0);
        if (AGNES_FLOW_AHEAD > 1 && lane == 0) tq = atomicAdd(ctr, 1u) + 2u * qS;
    }
#else
    const uint32_t qS = 0u;
    {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(ctr, 2u);
        t = rdl(t, 0u);
        range_of(t, H.s0, H.e0);
        range_of(t + 1u, N.s0, N.e0);
        if (AGNES_FLOW_AHEAD > 1 && lane == 0) tq = atomicAdd(ctr, 1u);
    }
#endif
    FDIAG(unsigned long long* const dg = flow_diag_buf + 64ull * (blockIdx.x * AGNES_WAVES_PER_BLOCK + wave);
          uint32_t dg_b = 0, dg_c = 0;
          if (lane == 0) dg[0] = __builtin_amdgcn_s_memrealtime();)
    if (H.s0 >= H.e0) {
        FDIAG(if (lane == 0) { dg[1] = __builtin_amdgcn_s_memrealtime(); dg[2] = 0; dg[3] = 0; })
        return;
    }
    hdr1(H);
#if AGNES_FLOW_FAST_START
    { /* the first chunk's DMA as soon as the offsets are in, ahead of the set constants
       * (only for offsets that bound a stream inside the columns; hdr2 decides the rest) */
        const uint32_t m = H.e0 - H.s0;
        const uint64_t O0 = u64of(rdl(H.olo, 0u), rdl(H.ohi, 0u)), Om = u64of(rdl(H.olo, m), rdl(H.ohi, m));
        const bool ragb = ballot(lane <= m && (H.olo & 3u) != 0u) != 0ull;
        if (Om > O0 && Om - O0 < (1ull << 30) && (RG || !ragb)) {
            const uint64_t Sa0 = O0 & ~127ull;
            dma_chunk(Sa0, (uint32_t)(O0 - Sa0), (uint32_t)(Om - Sa0));
            pf_at = Sa0;
        }
    }
#endif
    hdr2(H);
    hdr3(H);
    dma_states(H, spar);
    hdr1(N);

    for (;;) { /* batches: H current, N next */
        const uint32_t m = H.e0 - H.s0;
        FDIAG(const uint32_t dg_c0 = dg_c; const unsigned long long dg_t = __builtin_amdgcn_s_memrealtime();)
        unsigned char* const sbh = sb + spar * (FB * 64u);
        bool smf = SM; /* the State views are not yet set up from the staged States */
        if (!H.go) { /* not this kernel's stream */
            if (pf_at != ~0ull) { /* an early first-chunk DMA of this batch: drained, dropped */
                dma_wait();
                pf_at = ~0ull;
            }
            /* the walk list (agnes_sweep.hip) takes the batches that are no stream of this kernel */
            {
                uint32_t w0 = 0;
                if (lane == 0) w0 = atomicAdd(a.list_count + AGNES_WALK_COUNT, m);
                w0 = rdl(w0, 0u);
                if (lane < m) a.walk[w0 + lane] = H.s0 + lane;
                /* the walk kernel works in place on a.states: bring the batch's input States over */
                if (SM && a.states_in && a.states_in != a.states)
                    for (uint32_t j = lane; j < 4u * m; j += 64u)
                        reinterpret_cast<uint4*>(a.states + H.s0)[j] = reinterpret_cast<const uint4*>(a.states_in + H.s0)[j];
            }
        } else {
            /* the instance records' constants (written at the first chunk's top, once the
             * batch before has been finalized from its records) */
            const uint32_t q2k = H.q2, q2hk = H.q2h;
            const uint32_t setk = H.hs;
            /* the stream: instance starts relative to its first vote */
            const uint64_t S0 = u64of(rdl(H.olo, 0u), rdl(H.ohi, 0u));
            const uint32_t s0lo = (uint32_t)S0;
            /* chunks at 128-vote boundaries (whole lines of every column): the first one
             * starts `lead` votes before the stream; positions are relative to Sa */
            const uint64_t Sa = S0 & ~127ull;
            const uint32_t lead = (uint32_t)(S0 - Sa);
            const uint32_t Lend = rdl(H.olo, m) - s0lo + lead;
            const uint32_t rl = H.olo - s0lo + lead;
            const uint32_t rn = shfl(rl, lane + 1u);
            const uint64_t NE = ballot(lane < m && rn > rl);
            const uint32_t relv = lane <= m ? rl : 0x7FFFFFFFu;
            const uint64_t mm64 = (1ull << m) - 1ull;

            /* the chunks: the aligned loop, or (RG, an unaligned stream) the U loop */
            auto chunks = [&](auto u_t) {
            constexpr bool U = decltype(u_t)::value;
            for (uint32_t rc = 0; rc < Lend; rc += CH) {
                FDIAG(++dg_c;)
                const uint64_t c = Sa + rc;
                const uint32_t lo_r = rc == 0u ? lead : 0u; /* the chunk's active votes: lo_r .. hi_r */
                const bool fresh = pf_at != c;
                if (fresh) dma_chunk(c, lo_r, Lend - rc); /* not prefetched: a wave's first chunk */
                /* this chunk's DMA (and a new batch's States) have landed; a whole-chunk code
                 * store issued behind that DMA may stay in flight */
                if (AGNES_FLOW_CODE_VMCNT && dc_one && !fresh) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
                else dma_wait();
                dc_one = false;
                /* raised priority from here until the next chunk's DMA and the deferred code
                 * store are out: a wave's memory traffic goes out ahead of the other waves'
                 * K2-K4 work (same-box A/B: flow -1 % on C2 and C3) */
                __builtin_amdgcn_s_setprio(1);
                if (rc == 0u && lane < m) { /* instance records */
                    uint32_t* const rk = itab + RW * lane;
                    rk[R_Q2] = q2k;
                    if (W64) rk[R_Q2H] = q2hk;
                    rk[R_PBASE] = setk < ns ? setk * nv : 0u;
                    rk[R_NV] = setk < ns ? nv : 0u;
                    rk[R_SMASK] = 0u; /* no State machine: no role */
                    rk[R_P1] = NONE;
                    rk[R_C] = NONE;
                    rk[R_DF] = 0u;
                    rk[R_DR] = 0u;
                    if (SM) vtab[lane] = 0ull;
                    if (EVC) etab[lane] = 0u;
                    if (EDG) {
                        for (uint32_t q = 0; q < 2u * R; ++q) elab[lane * 2u * R + q] = 0u; /* VoteCount::new, no message */
                    }
                }
                if (SM && smf) { /* the State machine's view of each instance (state_machine.rs:184) */
                    if (lane < m) {
                        const uint32_t* const sp = reinterpret_cast<const uint32_t*>(sbh + 64u * lane);
                        const int64_t rnd = (int64_t)u64of(sp[2], sp[3]);
                        const uint32_t step = sp[13] & 0xFFu;
                        uint32_t smask = __builtin_amdgcn_perm(SM_HI, SM_LO, rep4(step < 7u ? step : 7u));
                        if (rnd < 0 || rnd > 255) smask &= X_C * 0x01010101u; /* no vote round equals State.round */
                        uint32_t* const rk = itab + RW * lane;
                        rk[R_SMASK] = smask;
                        rk[R_EQ8] = (rnd >= 0 && rnd <= 255) ? (uint32_t)rnd : 0x100u;
                        rk[R_EQ] = rep4((uint32_t)rnd);
                        rk[R_VALL] = step == AGNES_STEP_PRECOMMIT ? 0xFFFFFFFFu : 0u;
                        rk[R_STEP] = step;
                    }
                    smf = false;
                }
                /* the next batch's header, one stage per chunk; its States behind it */
                if (AGNES_FLOW_AHEAD == 1 && N.stage == 0u) { /* N's slot, claimed at this batch's start */
                    range_of(rdl(tq, 0u), N.s0, N.e0);
                    hdr1(N);
                } else if (N.s0 < N.e0) {
                    if (N.stage == 1u) {
                        hdr2(N);
                    } else if (N.stage == 2u) {
                        hdr3(N);
                        if (N.go) dma_states(N, spar ^ 1u);
                    }
                }

                /* ---- segments: the instances the chunk straddles, at unit granularity ---- */
                const uint32_t tj = relv - rc; /* instance start relative to the chunk */
                const uint32_t k0 = 63u - (uint32_t)__builtin_clzll(ballot((int32_t)tj <= (int32_t)lo_r) & mm64);
                uint64_t bk = ballot(tj - lo_r - 1u < CH - lo_r - 1u) & NE; /* non-empty, starting inside */
                const bool multi = bk != 0ull;
                const bool cont0 = ((ballot((int32_t)tj < 0) >> k0) & 1ull) != 0ull;
                const uint32_t left = Lend - rc;
                const bool lastc = left > CH && !ballot(tj == CH);
                const uint32_t hi_r = left < CH ? left : CH;
                /* the lane's votes inside the stream: whole units (aligned), or (U) bytes */
                uint32_t act0, act1;
                if (U) {
                    const int32_t nlo = (int32_t)lo_r - (int32_t)o8, nhi = (int32_t)hi_r - (int32_t)o8;
                    act0 = below_bytes(nhi) & ~below_bytes(nlo);
                    act1 = below_bytes(nhi - 4) & ~below_bytes(nlo - 4);
                } else {
                    act0 = o8 >= lo_r && o8 < hi_r ? 0xFFFFFFFFu : 0u;
                    act1 = o8 + 4u >= lo_r && o8 + 4u < hi_r ? 0xFFFFFFFFu : 0u;
                }
                const bool actA = act0 != 0u, actB = act1 != 0u;
                uint32_t kA = k0, kB = k0, sA = 0, klast = k0, slast = 0;
                bool split = false;
                /* lanes whose unit A / B starts an instance; (U) unit A = the lane's votes before
                 * spI, the position of the instance start inside the lane (8: none), unit B the rest */
                uint64_t SA = 0, SBm = 0;
                uint32_t spI = 8u;
                if (multi) {
                    uint32_t segw = k0, D = 0;
                    while (bk) {
                        const uint32_t k = (uint32_t)__builtin_ctzll(bk);
                        bk &= bk - 1ull;
                        ++D;
                        uint32_t L;
                        if (U) { /* its lane and position in the lane */
                            const uint32_t t = rdl(tj, k);
                            L = t >> 3;
                            if (t & 7u) SBm |= 1ull << L;
                            else SA |= 1ull << L;
                            segw = lane == D ? (k | (L << 8) | ((t & 7u) << 16)) : segw;
                        } else {
                            const uint32_t u = rdl(tj, k) >> 2; /* its first unit */
                            L = u >> 1;
                            if (u & 1u) SBm |= 1ull << L;
                            else SA |= 1ull << L;
                            segw = lane == D ? (k | (L << 8)) : segw;
                        }
                        klast = k;
                        slast = L;
                    }
                    /* segments started at or before my unit A, and whether unit B starts one */
                    const uint32_t dA = mbcnt64(SA) + (uint32_t)((SA >> lane) & 1ull) + mbcnt64(SBm);
                    split = ((SBm >> lane) & 1ull) != 0ull;
                    const uint32_t wA = shfl(segw, dA), wB = shfl(segw, dA + (split ? 1u : 0u));
                    kA = wA & 0xFFu;
                    sA = (wA >> 8) & 0xFFu;
                    kB = wB & 0xFFu;
                    if (U && split) spI = wB >> 16;
                }
                /* vote s of the lane in unit B: the aligned kernel's unit is fixed (s >= 4), the U
                 * kernel's starts at spI (no start: 8, and kB == kA) */
                auto inB = [&](uint32_t s) -> bool { return U ? s >= spI : s >= 4u; };
                const uint4 recA = *reinterpret_cast<const uint4*>(itab + RW * kA); /* q2, pbase, nv, State.round (0x100: none) */
                const uint4 recB = multi ? *reinterpret_cast<const uint4*>(itab + RW * kB) : recA;

                /* the next chunk by LDS-DMA (this stream's, or the next batch's first) */
                auto next_dma = [&]() {
                    uint64_t nc = ~0ull;
                    uint32_t nl = 0, nlo = 0;
                    if (rc + CH < Lend) {
                        nc = c + CH;
                        nl = Lend - rc - CH;
                    } else if (N.s0 < N.e0 && N.stage == 3u && N.go) {
                        const uint32_t mN = N.e0 - N.s0;
                        const uint64_t n0 = u64of(rdl(N.olo, 0u), rdl(N.ohi, 0u));
                        nc = n0 & ~127ull;
                        nlo = (uint32_t)(n0 - nc);
                        nl = rdl(N.olo, mN) - (uint32_t)n0 + nlo;
                    }
                    if (nc != ~0ull && nl != nlo) {
                        dma_chunk(nc, nlo, nl);
                        pf_at = nc;
                    } else {
                        pf_at = ~0ull;
                    }
                };
                /* ---- K1: votes of the chunk + validation + weight gather ---- */
                uint32_t value[LV], val[LV], r8[2], t8[2];
                uint32_t w[LV];
                uint64_t wq[W64 ? LV : 1u]; /* (W64) the weights from the i64 table */
                uint32_t nb0 = 0, nb1 = 0; /* 0x10 in the bytes of nil votes */
                bool all_ok;
                uint32_t okb0, okb1; /* byte masks of the votes that checked in (exact path) */
                {
                    uint32_t inst[LV];
                    {
                        const uint4 i0 = *reinterpret_cast<const uint4*>(slot + F_INST + o32);
                        const uint4 i1 = *reinterpret_cast<const uint4*>(slot + F_INST + o32 + 16u);
                        const uint4 v0 = *reinterpret_cast<const uint4*>(slot + F_VALUE + o32);
                        const uint4 v1 = *reinterpret_cast<const uint4*>(slot + F_VALUE + o32 + 16u);
                        const uint4 d0 = *reinterpret_cast<const uint4*>(slot + F_VAL + o32);
                        const uint4 d1 = *reinterpret_cast<const uint4*>(slot + F_VAL + o32 + 16u);
                        const uint2 rr = *reinterpret_cast<const uint2*>(slot + F_ROUND + o8);
                        const uint2 tt = *reinterpret_cast<const uint2*>(slot + F_TYPE + o8);
                        inst[0] = i0.x; inst[1] = i0.y; inst[2] = i0.z; inst[3] = i0.w;
                        inst[4] = i1.x; inst[5] = i1.y; inst[6] = i1.z; inst[7] = i1.w;
                        value[0] = v0.x; value[1] = v0.y; value[2] = v0.z; value[3] = v0.w;
                        value[4] = v1.x; value[5] = v1.y; value[6] = v1.z; value[7] = v1.w;
                        val[0] = d0.x; val[1] = d0.y; val[2] = d0.z; val[3] = d0.w;
                        val[4] = d1.x; val[5] = d1.y; val[6] = d1.z; val[7] = d1.w;
                        r8[0] = rr.x; r8[1] = rr.y;
                        t8[0] = tt.x; t8[1] = tt.y;
                    }
                    /* K1: w = power[set][validator] (consensus_executor.rs:62-63 ->
                     * validators.rs:7), gathered before the checks so their VALU work
                     * covers the latency: an index outside the set's row reads entry 0
                     * (a vote that checks out weighs 0, below) */
                    {
                        const uint32_t pbA = recA.y, pbB = recB.y;
#pragma unroll
                        for (uint32_t s = 0; s < LV; ++s) {
                            const uint32_t v = val[s], pb = inB(s) ? pbB : pbA, nvs = inB(s) ? recB.z : recA.z;
                            const uint32_t idx = v < nvs ? pb + v : 0u;
                            if constexpr (W64)
                                wq[s] = PC ? reinterpret_cast<const uint64_t*>(agnes_smem)[idx] : (uint64_t)a.power[idx];
                            else
                                w[s] = PC ? reinterpret_cast<const uint32_t*>(agnes_smem)[idx] : a.power32[idx];
                        }
                    }
#pragma unroll
                    for (uint32_t s = 0; s < 4u; ++s) {
                        nb0 |= value[s] == AGNES_NIL ? 0x10u << (8u * s) : 0u;
                        nb1 |= value[4u + s] == AGNES_NIL ? 0x10u << (8u * s) : 0u;
                    }
                    /* the boundary's checks: round < R, type in {0, 1}, the vote names its
                     * instance, validator in the set */
                    const uint32_t idA = H.s0 + kA, idB = H.s0 + kB;
                    const uint32_t bad0 = R == 1u ? (t8[0] & 0xFEFEFEFEu) | r8[0]
                                                  : (t8[0] & 0xFEFEFEFEu) | ((r8[0] | ((r8[0] & 0x7F7F7F7Fu) + RK)) & 0x80808080u);
                    const uint32_t bad1 = R == 1u ? (t8[1] & 0xFEFEFEFEu) | r8[1]
                                                  : (t8[1] & 0xFEFEFEFEu) | ((r8[1] | ((r8[1] & 0x7F7F7F7Fu) + RK)) & 0x80808080u);
                    if (U) {
                        /* the unit's instance and set per vote: the lane is checked as a whole (a
                         * lane with votes outside the stream fails and takes the exact path) */
                        uint32_t d = bad0 | bad1;
                        bool vin = true;
#pragma unroll
                        for (uint32_t s = 0; s < LV; ++s) {
                            d |= inst[s] ^ (inB(s) ? idB : idA);
                            vin = vin && val[s] < (inB(s) ? recB.z : recA.z);
                        }
                        all_ok = !ballot((actA || actB) && !(d == 0u && vin));
                    } else {
                        const uint32_t mA = max(max(val[0], val[1]), max(val[2], val[3]));
                        const uint32_t mB = max(max(val[4], val[5]), max(val[6], val[7]));
                        /* a unit names its instance: the OR of the four ids XOR the id is zero (three
                         * bitwise ops, not four compares whose lane masks are rebuilt as bits) */
                        const uint32_t dA = (inst[0] ^ idA) | (inst[1] ^ idA) | (inst[2] ^ idA) | (inst[3] ^ idA);
                        const uint32_t dB = (inst[4] ^ idB) | (inst[5] ^ idB) | (inst[6] ^ idB) | (inst[7] ^ idB);
                        const bool okA = (bad0 | dA) == 0u && mA < recA.z;
                        const bool okB = (bad1 | dB) == 0u && mB < recB.z;
                        all_ok = !ballot((actA && !okA) || (actB && !okB));
                    }
                    okb0 = act0;
                    okb1 = act1;
                    if (!all_ok) { /* the exact per-vote checks */
                        uint32_t o0 = 0, o1 = 0;
#pragma unroll
                        for (uint32_t s = 0; s < 4u; ++s) {
                            const uint32_t iA = inB(s) ? idB : idA, iB = inB(4u + s) ? idB : idA;
                            const uint32_t nA = inB(s) ? recB.z : recA.z, nB = inB(4u + s) ? recB.z : recA.z;
                            const bool g0 = ((bad0 >> (8u * s)) & 0xFFu) == 0u && inst[s] == iA && val[s] < nA;
                            const bool g1 = ((bad1 >> (8u * s)) & 0xFFu) == 0u && inst[4u + s] == iB && val[4u + s] < nB;
                            o0 |= g0 ? 0xFFu << (8u * s) : 0u;
                            o1 |= g1 ? 0xFFu << (8u * s) : 0u;
                        }
                        const uint32_t p0m = okb0, p1m = okb1;
                        okb0 &= o0;
                        okb1 &= o1;
                        bad += (uint32_t)(__builtin_popcount(p0m & ~okb0) + __builtin_popcount(p1m & ~okb1)) >> 3;
                    }
                }
                if (!(all_ok && lo_r == 0u && hi_r == CH)) { /* votes that checked out weigh 0 */
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        const bool o = (((s < 4u ? okb0 : okb1) >> (8u * (s & 3u))) & 1u) != 0u;
                        if constexpr (W64) wq[s] = o ? wq[s] : 0ull;
                        else w[s] = o ? w[s] : 0u;
                    }
                }
                /* a gather from HBM retires before the DMA below is issued: a wait on it
                 * behind the DMA would wait for the DMA too (in-order vmcnt) */
                if (W64 && !PC) asm volatile("" ::"v"(wq[0]), "v"(wq[1]), "v"(wq[2]), "v"(wq[3]), "v"(wq[4]), "v"(wq[5]),
                                      "v"(wq[6]), "v"(wq[7]));
                else if (!PC) asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]),
                                      "v"(w[6]), "v"(w[7]));
                next_dma();
                flush(); /* the previous chunk's codes */
                __builtin_amdgcn_s_setprio(0);

                /* ---- K2 + K3 ---- */
                uint32_t* const A = crow + cpar * cw;
                uint32_t* const B = crow + (cpar ^ 1u) * cw;
                /* per-vote bucket shifts as bytes, no per-vote masks: type * 32 (the
                 * precommit half of the accumulator) | nil * 16 */
                const uint32_t ts0c = (t8[0] & 0x01010101u) << 5, ts1c = (t8[1] & 0x01010101u) << 5;
                const uint32_t sh0c = ts0c | nb0, sh1c = ts1c | nb1;
                /* Several rounds (!R1): when every unit holds one round and, inside the chunk,
                 * an instance's rounds only increase, the segments are the (instance, round)
                 * RUNS, each one executor (RoundVotes of that round, round_votes.rs:74-97) with
                 * its carry-in from the previous chunk's row (no run of the chunk revisits a
                 * round), and one pass tallies every round (`runs`).  Otherwise one pass per
                 * round present, the other rounds' votes masked.  (Generated streams hold an
                 * instance's rounds in order: C3's chunks take one pass.) */
                bool runs = false;
                uint32_t uA = 0, uB = 0, sAr = sA;
                bool splitr = split, multir = multi;
                uint64_t SAr = 0, SBr = 0;
                uint32_t spR = spI; /* (U) the position of the run start inside the lane (8: none) */
                if (U && !R1 && all_ok) {
                    /* (U) runs at any position: a lane may hold one run start after its first
                     * vote (an instance start or a round change), and the rounds of an instance
                     * only increase inside the chunk */
                    uint32_t q0 = r8[0], q1 = r8[1];
                    if (lo_r != 0u || hi_r != CH) { /* the votes outside the stream take the nearest round inside */
                        const uint32_t hz = hi_r - 1u;
                        const uint32_t rf = (rdl(((lo_r >> 2) & 1u) ? r8[1] : r8[0], lo_r >> 3) >> (8u * (lo_r & 3u))) & 0xFFu;
                        const uint32_t rz = (rdl(((hz >> 2) & 1u) ? r8[1] : r8[0], hz >> 3) >> (8u * (hz & 3u))) & 0xFFu;
                        const int32_t nlo = (int32_t)lo_r - (int32_t)o8;
                        const uint32_t bl0 = below_bytes(nlo), bl1 = below_bytes(nlo - 4);
                        q0 = (q0 & act0) | (~act0 & ((bl0 & (rf * 0x01010101u)) | (~bl0 & (rz * 0x01010101u))));
                        q1 = (q1 & act1) | (~act1 & ((bl1 & (rf * 0x01010101u)) | (~bl1 & (rz * 0x01010101u))));
                    }
                    const uint32_t pl = shfl(q1, lane - 1u) >> 24; /* the previous lane's last round */
                    const uint32_t pw0 = (q0 << 8) | (lane ? pl : (q0 & 0xFFu)), pw1 = (q1 << 8) | (q0 >> 24);
                    const uint32_t ch0 = nz_marks(q0 ^ pw0), ch1 = nz_marks(q1 ^ pw1); /* round changes */
                    const uint32_t ge0 = ((q0 | 0x80808080u) - pw0) & 0x80808080u; /* round >= the one before */
                    const uint32_t ge1 = ((q1 | 0x80808080u) - pw1) & 0x80808080u;
                    const bool iA = ((SA >> lane) & 1ull) != 0ull;
                    const uint32_t is0 = (iA ? 0x80u : 0u) | (spI < 4u ? 0x80u << (8u * spI) : 0u);
                    const uint32_t is1 = (spI >= 4u && spI < 8u) ? 0x80u << (8u * (spI - 4u)) : 0u;
                    const uint32_t in0 = (ch0 | is0) & ~0x80u, in1 = ch1 | is1; /* run starts after vote 0 */
                    const bool badr = ((ch0 & ~ge0 & ~is0) | (ch1 & ~ge1 & ~is1)) != 0u ||
                                      __builtin_popcount(in0) + __builtin_popcount(in1) > 1;
                    if (!ballot(badr)) {
                        runs = true;
                        const bool rsA = (ch0 & 0x80u) != 0u && !iA;
                        spR = in0 ? (uint32_t)__builtin_ctz(in0) >> 3 : (in1 ? 4u + ((uint32_t)__builtin_ctz(in1) >> 3) : 8u);
                        splitr = spR < 8u;
                        SAr = SA | ballot(rsA);
                        SBr = ballot(splitr);
                        multir = (SAr | SBr) != 0ull;
                        uA = q0 & 0xFFu;
                        uB = splitr ? ((spR < 4u ? q0 : q1) >> (8u * (spR & 3u))) & 0xFFu : uA;
                        const uint64_t mA = SAr & ((2ull << lane) - 1ull), mB = SBr & ((1ull << lane) - 1ull);
                        const uint32_t la = mA ? 63u - (uint32_t)__builtin_clzll(mA) : 0u;
                        const uint32_t lb = mB ? 63u - (uint32_t)__builtin_clzll(mB) : 0u;
                        sAr = la > lb ? la : lb;
                    }
                } else if (!R1 && all_ok) {
                    uA = r8[0] & 0xFFu;
                    uB = r8[1] & 0xFFu;
                    if (lo_r != 0u || hi_r != CH) {
                        /* a stream's first or last chunk (round 5): the units outside it (no votes,
                         * weight 0) take the round of the nearest unit inside, so they extend its
                         * run and never start one */
                        const uint32_t rf = rdl(((lo_r >> 2) & 1u) ? uB : uA, lo_r >> 3);
                        const uint32_t rz = rdl((((hi_r - 1u) >> 2) & 1u) ? uB : uA, (hi_r - 1u) >> 3);
                        if (!actA) uA = o8 < lo_r ? rf : rz;
                        if (!actB) uB = o8 + 4u < lo_r ? rf : rz;
                    }
                    const uint32_t pA = shfl(uB, lane - 1u); /* the unit before unit A (lane 0: none) */
                    const bool iA = ((SA >> lane) & 1ull) != 0ull, iB = ((SBm >> lane) & 1ull) != 0ull;
                    const bool rsA = lane != 0u && !iA && uA != pA, rsB = !iB && uB != uA;
                    const bool badr = (actA && r8[0] != uA * 0x01010101u) || (actB && r8[1] != uB * 0x01010101u) ||
                                      (rsA && uA < pA) || (rsB && uB < uA);
                    if (!ballot(badr)) {
                        runs = true;
                        SAr = SA | ballot(rsA);
                        SBr = SBm | ballot(rsB);
                        multir = (SAr | SBr) != 0ull;
                        splitr = ((SBr >> lane) & 1ull) != 0ull;
                        /* unit A's run starts at the last run start at or before it: a unit A of a
                         * lane <= mine or a unit B of a lane < mine (that lane's last-segment
                         * prefix is its unit B alone) */
                        const uint64_t mA = SAr & ((2ull << lane) - 1ull), mB = SBr & ((1ull << lane) - 1ull);
                        const uint32_t la = mA ? 63u - (uint32_t)__builtin_clzll(mA) : 0u;
                        const uint32_t lb = mB ? 63u - (uint32_t)__builtin_clzll(mB) : 0u;
                        sAr = la > lb ? la : lb;
                    }
                }
                if (lastc) { /* row B: the executors the last instance carries into the next chunk */
                    const bool keep = cont0 && klast == k0 && (runs || !multi);
                    for (uint32_t k = lane; k < cw; k += 64u) B[k] = keep ? A[k] : 0u;
                    __builtin_amdgcn_wave_barrier();
                }
                const bool cA = cont0 && kA == k0;   /* unit A continues the previous chunk's instance */
                const bool cL = cont0 && klast == k0; /* so does the last segment */
                uint32_t lv0 = 0, lv1 = 0; /* levels 0..3, byte s & 3 of unit s >> 2 */
                uint32_t lvb0 = 0, lvb1 = 0; /* (EDG) the levels BEFORE each vote (its executor's sums without it) */
                /* (State machine) quorums crossed before each unit: bit 0 / 2 the prevote nil or
                 * value one at State.round (P1 is then behind the unit A / B), bit 1 / 3 a precommit
                 * value one (C behind it) -- the sums only grow, so a unit's first candidate is
                 * the instance's first exactly when its bit is clear */
                uint32_t cf = 0;
                /* one tally pass: the round r's votes (ONE: every round, each unit in its run) */
                auto pass = [&](auto one_t, uint32_t r) {
                    constexpr bool ONE = decltype(one_t)::value;
                    const uint32_t sAx = ONE ? sAr : sA;
                    const bool splitx = ONE ? splitr : split, multix = ONE ? multir : multi;
                    /* (U) the lane's segment split: a run start in runs mode, else an instance start */
                    const uint32_t spx = ONE ? spR : spI;
                    auto inBx = [&](uint32_t s) -> bool { return U ? s >= spx : s >= 4u; };
                    uint32_t sh0 = sh0c, sh1 = sh1c, ts0 = ts0c, ts1 = ts1c;
                    if (!R1) asm volatile("" : "+v"(sh0), "+v"(sh1), "+v"(ts0), "+v"(ts1)); /* extracts stay per pass */
                    /* 0xFF in the bytes of this round's votes */
                    const uint32_t rm0 = (R > 1u && !ONE) ? mark_bytes(zero_marks(r8[0] ^ (r * 0x01010101u))) : 0xFFFFFFFFu;
                    const uint32_t rm1 = (R > 1u && !ONE) ? mark_bytes(zero_marks(r8[1] ^ (r * 0x01010101u))) : 0xFFFFFFFFu;
                    /* lane-serial prefix of the round's four buckets, 16-bit fields:
                     * prevote value | prevote nil << 16 | precommit value << 32 | precommit nil << 48;
                     * Dw: the vote's own type's half after it */
                    uint64_t P = 0, P3 = 0;
                    uint32_t Dw[LV];
                    uint32_t Dwb[EDG ? LV : 1u]; /* (EDG) the same before the vote */
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        const uint32_t bs = 8u * (s & 3u);
                        uint32_t ws = w[s];
                        if (R > 1u && !ONE) ws &= (uint32_t)__builtin_amdgcn_sbfe((int32_t)(s < 4u ? rm0 : rm1), bs, 8u);
                        if constexpr (EDG) Dwb[s] = (uint32_t)(P >> __builtin_amdgcn_ubfe(s < 4u ? ts0 : ts1, bs, 8u));
                        P += (uint64_t)ws << __builtin_amdgcn_ubfe(s < 4u ? sh0 : sh1, bs, 8u);
                        if (U) { /* P3: the prefix of unit A (through vote spx - 1) */
                            if (s < 7u) P3 = s < spx ? P : P3;
                        } else if (s == 3u) {
                            P3 = P;
                        }
                        Dw[s] = (uint32_t)(P >> __builtin_amdgcn_ubfe(s < 4u ? ts0 : ts1, bs, 8u));
                    }
                    /* the lane's last segment (unit B alone when it starts a segment) */
                    const uint64_t T = splitx ? P - P3 : P;
                    const uint32_t Tvp = (uint32_t)T & 0xFFFFu, Tnp = (uint32_t)T >> 16;
                    const uint32_t Tvc = (uint32_t)(T >> 32) & 0xFFFFu, Tnc = (uint32_t)(T >> 48);
                    const uint32_t Ivp = scan(Tvp), Inp = scan(Tnp), Ivc = scan(Tvc), Inc = scan(Tnc);
                    const uint32_t Evp = Ivp - Tvp, Enp = Inp - Tnp, Evc = Ivc - Tvc, Enc = Inc - Tnc;
                    /* carried executors of the instance continuing from the previous chunk
                     * (keys 2r prevote, 2r + 1 precommit): uniform LDS reads per pass, or (ONE)
                     * each unit's own round's */
                    const uint32_t K = 2u * r;
                    uint32_t cvp = 0, cnp = 0, cvc = 0, cnc = 0;
                    if (ONE) {
                        if (cA) {
                            const uint2 cv = *reinterpret_cast<const uint2*>(A + 2u * uA);
                            const uint2 cn = *reinterpret_cast<const uint2*>(A + 2u * R + 2u * uA);
                            cvp = cv.x; cvc = cv.y; cnp = cn.x; cnc = cn.y;
                        }
                    } else if (cont0) {
                        cvp = A[K];
                        cvc = A[K + 1u];
                        cnp = A[2u * R + K];
                        cnc = A[2u * R + K + 1u];
                    }
                    /* unit A's running sums before the lane: scan - (scan at its segment's
                     * first lane) + carry */
                    uint32_t bvp = Evp, bnp = Enp, bvc = Evc, bnc = Enc;
                    if (multix) { /* every lane runs the shuffles */
                        const uint32_t xvp = shfl(Evp, sAx), xnp = shfl(Enp, sAx), xvc = shfl(Evc, sAx), xnc = shfl(Enc, sAx);
                        bvp -= xvp;
                        bnp -= xnp;
                        bvc -= xvc;
                        bnc -= xnc;
                    }
                    if (ONE || cA) {
                        bvp += cvp;
                        bnp += cnp;
                        bvc += cvc;
                        bnc += cnc;
                    }
                    /* thresholds on the lane prefix (sum > q2 <=> prefix > q2 - base), the
                     * prevote one in the low half and the precommit one in the high half of a
                     * u64, so the vote's own is one shift by its type byte */
                    const uint32_t qA = recA.x;
                    uint64_t TVa = u64of(qA - bvp, qA - bvc), TNa = u64of(qA - bnp, qA - bnc);
                    uint64_t TAa = u64of(qA - bvp - bnp, qA - bvc - bnc);
                    /* unit B: unit A's thresholds, or (split) its own segment from its carry-in
                     * (a new instance: none): the lane prefix there includes unit A's part, P3 */
                    uint64_t TVb = TVa, TNb = TNa, TAb = TAa;
                    const uint32_t p3vp = (uint32_t)P3 & 0xFFFFu, p3np = (uint32_t)P3 >> 16;
                    const uint32_t p3vc = (uint32_t)(P3 >> 32) & 0xFFFFu, p3nc = (uint32_t)(P3 >> 48);
                    uint32_t dvp = 0, dnp = 0, dvc = 0, dnc = 0; /* (ONE) unit B's carry-in */
                    if (multix && splitx) {
                        if (ONE && cont0 && kB == k0) {
                            const uint2 cv = *reinterpret_cast<const uint2*>(A + 2u * uB);
                            const uint2 cn = *reinterpret_cast<const uint2*>(A + 2u * R + 2u * uB);
                            dvp = cv.x; dvc = cv.y; dnp = cn.x; dnc = cn.y;
                        }
                        const uint32_t qB = recB.x;
                        TVb = u64of(qB + p3vp - dvp, qB + p3vc - dvc);
                        TNb = u64of(qB + p3np - dnp, qB + p3nc - dnc);
                        TAb = u64of(qB + p3vp + p3np - dvp - dnp, qB + p3vc + p3nc - dvc - dnc);
                    }
                    /* per vote: is_quorum on its own type's sums, precedence as a level */
                    uint32_t l0 = 0, l1 = 0, lb0x = 0, lb1x = 0;
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        const uint32_t bs = 8u * (s & 3u);
                        const uint32_t tsh = __builtin_amdgcn_ubfe(s < 4u ? ts0 : ts1, bs, 8u);
                        const int32_t tv = (int32_t)(uint32_t)((inBx(s) ? TVb : TVa) >> tsh);
                        const int32_t tn = (int32_t)(uint32_t)((inBx(s) ? TNb : TNa) >> tsh);
                        const int32_t ta = (int32_t)(uint32_t)((inBx(s) ? TAb : TAa) >> tsh);
                        const int32_t sv = (int32_t)(Dw[s] & 0xFFFFu), sn = (int32_t)(Dw[s] >> 16);
                        uint32_t l = sv + sn > ta ? 1u : 0u;
                        l = sn > tn ? 2u : l;
                        l = sv > tv ? 3u : l;
                        if (s < 4u) l0 |= l << bs;
                        else l1 |= l << bs;
                        if constexpr (EDG) {
                            const int32_t bv = (int32_t)(Dwb[s] & 0xFFFFu), bn = (int32_t)(Dwb[s] >> 16);
                            uint32_t lb = bv + bn > ta ? 1u : 0u;
                            lb = bn > tn ? 2u : lb;
                            lb = bv > tv ? 3u : lb;
                            if (s < 4u) lb0x |= lb << bs;
                            else lb1x |= lb << bs;
                        }
                    }
                    if (SM) {
                        /* unit A: its running sums before the lane exceed q2 <=> the threshold on the
                         * lane prefix is negative; unit B (same segment): the prefix through vote 3
                         * exceeds it; a split lane's unit B starts its segment (a round run's carry-in
                         * past q2 was crossed in an earlier chunk: in the record).  (ONE: C crossed
                         * in another run of the instance is found by K4's ballots.) */
                        const bool eA_ = R1 || (ONE ? uA : r) == recA.w, eB_ = R1 || (ONE ? uB : r) == recB.w;
                        const int32_t tvp = (int32_t)(uint32_t)TVa, tnp = (int32_t)(uint32_t)TNa;
                        const int32_t tvc = (int32_t)(uint32_t)(TVa >> 32);
                        cf |= (eA_ && (tvp < 0 || tnp < 0)) ? 1u : 0u;
                        cf |= tvc < 0 ? 2u : 0u;
                        if (!U && !splitx) { /* (U: K4 takes the lane's unit A whole) */
                            cf |= (eB_ && ((int32_t)p3vp > tvp || (int32_t)p3np > tnp)) ? 4u : 0u;
                            cf |= (int32_t)p3vc > tvc ? 8u : 0u;
                        }
                    }
                    lv0 |= l0 & rm0;
                    lv1 |= l1 & rm1;
                    if constexpr (EDG) {
                        lvb0 |= lb0x & rm0;
                        lvb1 |= lb1x & rm1;
                    }
                    if (lastc) {
                        if (ONE) { /* every run of the last instance: its executors at the run's end
                                    * (the lane holding its last unit writes) */
                            const bool endA = splitx, endB = lane == 63u || ((SAr >> (lane + 1u)) & 1ull) != 0ull;
                            if (endA && kA == klast) {
                                *reinterpret_cast<uint2*>(B + 2u * uA) = make_uint2(bvp + p3vp, bvc + p3vc);
                                *reinterpret_cast<uint2*>(B + 2u * R + 2u * uA) = make_uint2(bnp + p3np, bnc + p3nc);
                            }
                            if (endB && kB == klast) {
                                const uint32_t evp = splitx ? dvp + Tvp : bvp + ((uint32_t)P & 0xFFFFu);
                                const uint32_t enp = splitx ? dnp + Tnp : bnp + ((uint32_t)P >> 16);
                                const uint32_t evc = splitx ? dvc + Tvc : bvc + ((uint32_t)(P >> 32) & 0xFFFFu);
                                const uint32_t enc = splitx ? dnc + Tnc : bnc + (uint32_t)(P >> 48);
                                *reinterpret_cast<uint2*>(B + 2u * uB) = make_uint2(evp, evc);
                                *reinterpret_cast<uint2*>(B + 2u * R + 2u * uB) = make_uint2(enp, enc);
                            }
                        } else { /* the last segment's executors after the chunk (lane 0 writes) */
                            const uint32_t nvp = rdl(Ivp, 63u) - rdl(Evp, slast) + (cL ? cvp : 0u);
                            const uint32_t nnp = rdl(Inp, 63u) - rdl(Enp, slast) + (cL ? cnp : 0u);
                            const uint32_t nvc = rdl(Ivc, 63u) - rdl(Evc, slast) + (cL ? cvc : 0u);
                            const uint32_t nnc = rdl(Inc, 63u) - rdl(Enc, slast) + (cL ? cnc : 0u);
                            if (lane == 0u) {
                                B[K] = nvp;
                                B[K + 1u] = nvc;
                                B[2u * R + K] = nnp;
                                B[2u * R + K + 1u] = nnc;
                            }
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                };
                /* W64: the same pass with u64 sums (the u64 domain, agnes_fast.h defer_si):
                 * the four buckets as separate lane-serial u64 prefixes (prevote / precommit x
                 * value / nil), four u64 DPP scans, and the compares on each vote's own running
                 * sums (the base before the lane plus the lane prefix) against q2 -- no per-vote
                 * thresholds held.  Pass 1 sums the lane's bucket totals (and through vote 3);
                 * pass 2 recomputes the running sums rather than holding them (VGPRs).  ONE:
                 * every round of the chunk in one pass (runs mode, each unit its run's carry). */
                auto pass64 = [&](auto one_t, uint32_t r) {
                    constexpr bool ONE = decltype(one_t)::value;
                    const uint32_t sAx = ONE ? sAr : sA;
                    const bool splitx = ONE ? splitr : split, multix = ONE ? multir : multi;
                    /* 0xFF in the bytes of this round's votes */
                    const uint32_t rm0 = (R > 1u && !ONE) ? mark_bytes(zero_marks(r8[0] ^ (r * 0x01010101u))) : 0xFFFFFFFFu;
                    const uint32_t rm1 = (R > 1u && !ONE) ? mark_bytes(zero_marks(r8[1] ^ (r * 0x01010101u))) : 0xFFFFFFFFu;
                    auto wt = [&](uint32_t s) -> uint64_t { /* the vote's weight in this pass */
                        uint64_t x = wq[s];
                        if (R > 1u && !ONE) {
                            const int32_t m = __builtin_amdgcn_sbfe((int32_t)(s < 4u ? rm0 : rm1), 8u * (s & 3u), 8u);
                            x &= (uint64_t)(int64_t)m;
                        }
                        return x;
                    };
                    uint64_t Svp = 0, Snp = 0, Svc = 0, Snc = 0, P3vp = 0, P3np = 0, P3vc = 0, P3nc = 0;
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        const uint32_t bs = 8u * (s & 3u);
                        const bool pc = (((s < 4u ? t8[0] : t8[1]) >> bs) & 1u) != 0u;
                        const bool nil = (((s < 4u ? nb0 : nb1) >> bs) & 0x10u) != 0u;
                        const uint64_t x = wt(s);
                        Svp += (!pc && !nil) ? x : 0ull;
                        Snp += (!pc && nil) ? x : 0ull;
                        Svc += (pc && !nil) ? x : 0ull;
                        Snc += (pc && nil) ? x : 0ull;
                        if (s == 3u) { P3vp = Svp; P3np = Snp; P3vc = Svc; P3nc = Snc; }
                    }
                    const uint64_t Tvp = splitx ? Svp - P3vp : Svp, Tnp = splitx ? Snp - P3np : Snp;
                    const uint64_t Tvc = splitx ? Svc - P3vc : Svc, Tnc = splitx ? Snc - P3nc : Snc;
                    const uint64_t Ivp = scan(Tvp), Inp = scan(Tnp), Ivc = scan(Tvc), Inc = scan(Tnc);
                    const uint64_t Evp = Ivp - Tvp, Enp = Inp - Tnp, Evc = Ivc - Tvc, Enc = Inc - Tnc;
                    /* carried executors (u64 rows: vw[2R] then vn[2R], keys 2r prevote, 2r + 1
                     * precommit): uniform reads per pass, or (ONE) each unit's own round's */
                    const uint64_t* const A64 = reinterpret_cast<const uint64_t*>(A);
                    const uint32_t K = 2u * r;
                    uint64_t cvp = 0, cnp = 0, cvc = 0, cnc = 0;
                    if (ONE) {
                        if (cA) {
                            cvp = A64[2u * uA];
                            cvc = A64[2u * uA + 1u];
                            cnp = A64[2u * R + 2u * uA];
                            cnc = A64[2u * R + 2u * uA + 1u];
                        }
                    } else if (cont0) {
                        cvp = A64[K];
                        cvc = A64[K + 1u];
                        cnp = A64[2u * R + K];
                        cnc = A64[2u * R + K + 1u];
                    }
                    uint64_t bvp = Evp, bnp = Enp, bvc = Evc, bnc = Enc;
                    if (multix) {
                        bvp -= shfl(Evp, sAx);
                        bnp -= shfl(Enp, sAx);
                        bvc -= shfl(Evc, sAx);
                        bnc -= shfl(Enc, sAx);
                    }
                    if (ONE || cA) {
                        bvp += cvp;
                        bnp += cnp;
                        bvc += cvc;
                        bnc += cnc;
                    }
                    /* unit B of a split lane starts its segment from its own carry-in (a new
                     * instance, or a new run: the run's carried row) */
                    uint64_t dvp = 0, dnp = 0, dvc = 0, dnc = 0;
                    if (ONE && multix && splitx && cont0 && kB == k0) {
                        dvp = A64[2u * uB];
                        dvc = A64[2u * uB + 1u];
                        dnp = A64[2u * R + 2u * uB];
                        dnc = A64[2u * R + 2u * uB + 1u];
                    }
                    const uint64_t qA = u64of(recA.x, itab[RW * kA + R_Q2H]);
                    const uint64_t qB = (multix && splitx) ? u64of(recB.x, itab[RW * kB + R_Q2H]) : qA;
                    uint32_t l0 = 0, l1 = 0;
                    uint64_t Avp = bvp, Anp = bnp, Avc = bvc, Anc = bnc, q = qA;
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        if (s == 4u && multix && splitx) {
                            Avp = dvp;
                            Anp = dnp;
                            Avc = dvc;
                            Anc = dnc;
                            q = qB;
                        }
                        const uint32_t bs = 8u * (s & 3u);
                        const bool pc = (((s < 4u ? t8[0] : t8[1]) >> bs) & 1u) != 0u;
                        const bool nil = (((s < 4u ? nb0 : nb1) >> bs) & 0x10u) != 0u;
                        const uint64_t x = wt(s);
                        Avp += (!pc && !nil) ? x : 0ull;
                        Anp += (!pc && nil) ? x : 0ull;
                        Avc += (pc && !nil) ? x : 0ull;
                        Anc += (pc && nil) ? x : 0ull;
                        const uint64_t sv = pc ? Avc : Avp, sn = pc ? Anc : Anp;
                        uint32_t l = sv + sn > q ? 1u : 0u;
                        l = sn > q ? 2u : l;
                        l = sv > q ? 3u : l;
                        if (s < 4u) l0 |= l << bs;
                        else l1 |= l << bs;
                    }
                    if (SM) { /* crossed before the unit: the sums before it already past q2 */
                        const bool eA_ = R1 || (ONE ? uA : r) == recA.w, eB_ = R1 || (ONE ? uB : r) == recB.w;
                        cf |= (eA_ && (bvp > qA || bnp > qA)) ? 1u : 0u;
                        cf |= bvc > qA ? 2u : 0u;
                        if (!splitx) {
                            cf |= (eB_ && (bvp + P3vp > qA || bnp + P3np > qA)) ? 4u : 0u;
                            cf |= bvc + P3vc > qA ? 8u : 0u;
                        }
                    }
                    lv0 |= l0 & rm0;
                    lv1 |= l1 & rm1;
                    if (lastc) {
                        uint64_t* const B64 = reinterpret_cast<uint64_t*>(B);
                        if (ONE) { /* every run of the last instance: its executors at the run's end */
                            const bool endA = splitx, endB = lane == 63u || ((SAr >> (lane + 1u)) & 1ull) != 0ull;
                            if (endA && kA == klast) {
                                B64[2u * uA] = bvp + P3vp;
                                B64[2u * uA + 1u] = bvc + P3vc;
                                B64[2u * R + 2u * uA] = bnp + P3np;
                                B64[2u * R + 2u * uA + 1u] = bnc + P3nc;
                            }
                            if (endB && kB == klast) {
                                B64[2u * uB] = splitx ? dvp + Tvp : bvp + Svp;
                                B64[2u * uB + 1u] = splitx ? dvc + Tvc : bvc + Svc;
                                B64[2u * R + 2u * uB] = splitx ? dnp + Tnp : bnp + Snp;
                                B64[2u * R + 2u * uB + 1u] = splitx ? dnc + Tnc : bnc + Snc;
                            }
                        } else { /* the last segment's executors after the chunk (lane 0 writes) */
                            const uint64_t nvp = rdl(Ivp, 63u) - rdl(Evp, slast) + (cL ? cvp : 0ull);
                            const uint64_t nnp = rdl(Inp, 63u) - rdl(Enp, slast) + (cL ? cnp : 0ull);
                            const uint64_t nvc = rdl(Ivc, 63u) - rdl(Evc, slast) + (cL ? cvc : 0ull);
                            const uint64_t nnc = rdl(Inc, 63u) - rdl(Enc, slast) + (cL ? cnc : 0ull);
                            if (lane == 0u) {
                                B64[K] = nvp;
                                B64[K + 1u] = nvc;
                                B64[2u * R + K] = nnp;
                                B64[2u * R + K + 1u] = nnc;
                            }
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                };
                auto passes = [&](auto pf) {
                    if (R1) {
                        pf(std::false_type{}, 0u);
                    } else if (runs) {
                        pf(std::true_type{}, 0u);
                    } else {
                        /* the rounds present among the votes that checked in, one pass each */
                        uint32_t rb = 0;
#pragma unroll
                        for (uint32_t s = 0; s < LV; ++s) {
                            const uint32_t ok = ((s < 4u ? okb0 : okb1) >> (8u * (s & 3u))) & 1u;
                            rb |= ok << ((r8[s >> 2] >> (8u * (s & 3u))) & 15u);
                        }
                        uint32_t rset = wave_or(rb);
                        while (rset) {
                            const uint32_t r = (uint32_t)__builtin_ctz(rset);
                            rset &= rset - 1u;
                            pf(std::false_type{}, r);
                        }
                    }
                };
                if constexpr (W64) {
                    passes(pass64);
                } else if (R1) { /* (the u32 chain spelled out: the same code as before W64 took R > 1) */
                    pass(std::false_type{}, 0u);
                } else if (runs) {
                    pass(std::true_type{}, 0u);
                } else {
                    /* the rounds present among the votes that checked in, one pass each */
                    uint32_t rb = 0;
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        const uint32_t ok = ((s < 4u ? okb0 : okb1) >> (8u * (s & 3u))) & 1u;
                        rb |= ok << ((r8[s >> 2] >> (8u * (s & 3u))) & 15u);
                    }
                    uint32_t rset = wave_or(rb);
                    while (rset) {
                        const uint32_t r = (uint32_t)__builtin_ctz(rset);
                        rset &= rset - 1u;
                        pass(std::false_type{}, r);
                    }
                }
                if (lastc) cpar ^= 1u;
                /* to_event by (type, level); INVALID for a vote that checked out */
                uint32_t c0 = __builtin_amdgcn_perm(EV_HI, EV_LO, lv0 | (ts0c >> 3));
                uint32_t c1 = __builtin_amdgcn_perm(EV_HI, EV_LO, lv1 | (ts1c >> 3));
                if (!all_ok) {
                    c0 = (c0 & okb0) | ((act0 & ~okb0) & (AGNES_CODE_INVALID * 0x01010101u));
                    c1 = (c1 & okb1) | ((act1 & ~okb1) & (AGNES_CODE_INVALID * 0x01010101u));
                }

                /* ---- K4: State::apply(v.round, event) in stream order ---- */
                if (SM) {
                    uint32_t* const rA = itab + RW * kA;
                    uint32_t* const rB = itab + RW * kB;
                    /* State.round bytes, valid-from-start, P1, C */
                    const uint4 eA = *reinterpret_cast<const uint4*>(rA + R_SMASK); /* smask, eq, vall, step */
                    const uint4 eB = *reinterpret_cast<const uint4*>(rB + R_SMASK);
                    /* the roles of a unit's votes its step keeps; all but the commit one only at
                     * State.round (state_machine.rs:184-211) */
                    auto roles = [&](uint32_t smask, uint32_t eq, uint32_t r4, uint32_t c4, bool act) -> uint32_t {
                        /* one round (R1): every vote is of round 0 */
                        const uint32_t eqb = R1 ? (eq == 0u ? 0xFFFFFFFFu : 0u) : mark_bytes(zero_marks(r4 ^ eq));
                        const uint32_t x = __builtin_amdgcn_perm(XT_HI, XT_LO, c4 & 0x07070707u) & smask &
                                           (eqb | (X_C * 0x01010101u));
                        return act ? x : 0u;
                    };
                    if constexpr (U) {
                        /* (U) the lane's two PARTS as 8-byte masks: unit A = votes before spk (the
                         * split of the tally pass: a run start in runs mode, else an instance
                         * start), unit B the rest; the same derivation as the aligned units below */
                        const uint32_t spk = (!R1 && runs) ? spR : spI;
                        const uint64_t pmA = u64of(below_bytes((int32_t)spk), below_bytes((int32_t)spk - 4));
                        const uint64_t xA = u64of(roles(eA.x, eA.y, r8[0], c0, true) & act0, roles(eA.x, eA.y, r8[1], c1, true) & act1);
                        const uint64_t xB = kB == kA ? xA
                                                     : u64of(roles(eB.x, eB.y, r8[0], c0, true) & act0,
                                                             roles(eB.x, eB.y, r8[1], c1, true) & act1);
                        const uint64_t XPA = xA & pmA, XPB = xB & ~pmA;
                        if (ballot((XPA | XPB) != 0ull)) {
                            constexpr uint64_t B8 = 0x0101010101010101ull;
                            const uint32_t pos0 = rc + o8; /* stream-relative position of the lane's vote 0 */
                            const uint2 qA = *reinterpret_cast<const uint2*>(rA + R_P1);
                            const uint2 qB = *reinterpret_cast<const uint2*>(rB + R_P1);
                            const uint64_t nn = ~u64of(mark_bytes(nb0 << 3), mark_bytes(nb1 << 3)); /* non-nil votes */
                            const uint64_t r64 = u64of(r8[0], r8[1]);
                            auto vsel8 = [&](uint32_t b) -> uint32_t {
                                const uint32_t l0 = (b & 1u) ? value[1] : value[0], l1 = (b & 1u) ? value[3] : value[2];
                                const uint32_t h0 = (b & 1u) ? value[5] : value[4], h1 = (b & 1u) ? value[7] : value[6];
                                const uint32_t lo = (b & 2u) ? l1 : l0, hi = (b & 2u) ? h1 : h0;
                                return (b & 4u) ? hi : lo;
                            };
                            auto part = [&](uint64_t x, bool crossedP, bool crossedC, uint32_t* rk, uint32_t* sx, uint32_t vall,
                                            uint64_t& vc) -> uint64_t {
                                const uint64_t pm = x & (X_P1 * B8), cm = x & (X_C * B8);
                                const uint64_t lp = pm & (0ull - pm), lc = (cm & (0ull - cm)) >> 1;
                                const uint64_t preR = lp - 1ull, aliveR = lc - 1ull;
                                const bool p1ok = !crossedP && !crossedC && preR < aliveR;
                                const uint64_t alive = crossedC ? 0ull : aliveR;
                                const uint64_t pre = (crossedP || crossedC) ? 0ull : (preR < aliveR ? preR : aliveR);
                                const uint64_t atC = crossedC ? 0ull : (lc << 8) - lc; /* (byte 7: wraps to 0xFF << 56) */
                                const uint64_t atP = p1ok ? (lp << 8) - lp : 0ull;
                                if (!crossedC && lc) {
                                    const uint32_t b = (uint32_t)__builtin_ctzll(lc) >> 3;
                                    rk[R_C] = pos0 + b;
                                    sx[12] = vsel8(b);
                                    if (!R1) rk[R_DR] = (uint32_t)(r64 >> (8u * b)) & 0xFFu;
                                }
                                if (p1ok) {
                                    const uint32_t b = (uint32_t)__builtin_ctzll(lp) >> 3;
                                    rk[R_P1] = pos0 + b;
                                    if ((x >> (8u * b)) & X_PV) {
                                        rk[R_DF] = F_LOCK;
                                        sx[10] = vsel8(b);
                                    }
                                }
                                vc = x & alive & (~pre | u64of(vall, vall)) & nn & (X_PV * B8);
                                uint64_t msg = (x & ((pre & (X_TP * B8)) | (alive & (X_TC * B8)))) << 2;
                                msg |= atP & ((AGNES_VMSG_PRECOMMIT_NIL << AGNES_CODE_MSG_SHIFT) * B8 + (x & (X_PV * B8)));
                                msg |= atC & ((AGNES_VMSG_DECISION << AGNES_CODE_MSG_SHIFT) * B8);
                                return msg;
                            };
                            uint32_t* const sA = reinterpret_cast<uint32_t*>(sbh + 64u * kA);
                            uint32_t* const sB = reinterpret_cast<uint32_t*>(sbh + 64u * kB);
                            bool xcA = false, xcB = false;
                            if (!R1 && runs) { /* C crossed in an earlier part of the instance, another run */
                                const uint64_t XA = ballot((XPA & (X_C * B8)) != 0ull);
                                const uint64_t XB = ballot((XPB & (X_C * B8)) != 0ull);
                                const uint64_t iAm = SA & ((2ull << lane) - 1ull), iBm = SBm & ((1ull << lane) - 1ull);
                                const uint32_t fa = iAm ? 2u * (63u - (uint32_t)__builtin_clzll(iAm)) : 0u;
                                const uint32_t fb = iBm ? 2u * (63u - (uint32_t)__builtin_clzll(iBm)) + 1u : 0u;
                                const uint32_t ui = fa > fb ? fa : fb;
                                const uint64_t below = (1ull << lane) - 1ull;
                                const uint64_t fromA = ~((1ull << ((ui + 1u) >> 1)) - 1ull), fromB = ~((1ull << (ui >> 1)) - 1ull);
                                xcA = ((XA & fromA & below) | (XB & fromB & below)) != 0ull;
                                xcB = ((SBm >> lane) & 1ull) == 0ull && (xcA || ((XA >> lane) & 1ull) != 0ull);
                            }
                            uint64_t vA = 0, vB = 0;
                            uint64_t msg = part(XPA, (cf & 1u) || qA.x != NONE, (cf & 2u) || xcA || qA.y != NONE, rA, sA, eA.z, vA);
                            if (XPB) msg |= part(XPB, qB.x != NONE, xcB || qB.y != NONE, rB, sB, eB.z, vB);
                            c0 |= (uint32_t)msg;
                            c1 |= (uint32_t)(msg >> 32);
                            if (ballot((vA | vB) != 0ull)) { /* valid (:198, :202): the last candidate */
                                if (vA) {
                                    const uint32_t b = (63u - (uint32_t)__builtin_clzll(vA)) >> 3;
                                    atomicMax(vtab + kA, ((unsigned long long)(pos0 + b + 1u) << 32) | vsel8(b));
                                }
                                if (vB) {
                                    const uint32_t b = (63u - (uint32_t)__builtin_clzll(vB)) >> 3;
                                    atomicMax(vtab + kB, ((unsigned long long)(pos0 + b + 1u) << 32) | vsel8(b));
                                }
                            }
                        }
                    } else {
                    const uint32_t x0 = roles(eA.x, eA.y, r8[0], c0, actA), x1 = roles(eB.x, eB.y, r8[1], c1, actB);
                    if (ballot((x0 | x1) != 0u)) {
                        const uint32_t pos0 = rc + o8, pos1 = pos0 + 4u; /* stream-relative */
                        /* (an earlier chunk's P1 / C: in the record -- a round absent from this
                         * chunk has no crossing bit) */
                        const uint2 qA = *reinterpret_cast<const uint2*>(rA + R_P1);
                        const uint2 qB = *reinterpret_cast<const uint2*>(rB + R_P1);
                        const uint32_t nn0 = ~mark_bytes(nb0 << 3), nn1 = ~mark_bytes(nb1 << 3); /* non-nil votes */
                        /* One unit, every mask straight from its role bits.  P1 and C are behind the
                         * unit when their quorum was crossed before it (crossedP / crossedC), else at
                         * its first candidate byte (none: past it).  The Prevote step ends at P1 or
                         * at C, whichever comes first (a P1 after the commit never happens).
                         *   alive  bytes before C         pre  bytes before the Prevote step ends
                         *   atC    C's byte               atP  P1's byte (when P1 precedes C)
                         * TimeoutPrevote before P1 (:196), TimeoutPrecommit before C (:208), the
                         * precommit at P1 (:197-198), the Decision at C (:211); valid candidates:
                         * non-nil PolkaValues at State.round from P1 on (or from the start, entering
                         * in Precommit), before C (:198, :202).  The unit holding the instance's P1 /
                         * C records its position. */
                        /* the value of byte b of unit u's votes (registers) */
                        auto vsel = [&](uint32_t u, uint32_t b) -> uint32_t {
                            const uint32_t* const vv = value + 4u * u;
                            const uint32_t lo = (b & 1u) ? vv[1] : vv[0], hi = (b & 1u) ? vv[3] : vv[2];
                            return (b & 2u) ? hi : lo;
                        };
                        auto unit = [&](uint32_t u, uint32_t x, bool crossedP, bool crossedC, uint32_t pos, uint32_t* rk,
                                        uint32_t* sx, uint32_t r4, uint32_t vall, uint32_t nnb, uint32_t& vc) -> uint32_t {
                            const uint32_t pm = x & (X_P1 * 0x01010101u), cm = x & (X_C * 0x01010101u);
                            const uint32_t lp = pm & (0u - pm);        /* bit 0 of the first P1 candidate byte */
                            const uint32_t lc = (cm & (0u - cm)) >> 1; /* ... of the first commit candidate byte */
                            const uint32_t preR = lp - 1u, aliveR = lc - 1u; /* 0xFF below them (none: all) */
                            const bool p1ok = !crossedP && !crossedC && preR < aliveR;
                            const uint32_t alive = crossedC ? 0u : aliveR;
                            const uint32_t pre = (crossedP || crossedC) ? 0u : min(preR, aliveR);
                            const uint32_t atC = crossedC ? 0u : (lc << 8) - lc;
                            const uint32_t atP = p1ok ? (lp << 8) - lp : 0u;
                            /* the unit holding C: its position, the decision's value and round (:211) */
                            if (!crossedC && lc) {
                                const uint32_t b = (uint32_t)__builtin_ctz(lc) >> 3;
                                rk[R_C] = pos + b;
                                sx[12] = vsel(u, b);
                                if (!R1) rk[R_DR] = (r4 >> (8u * b)) & 0xFFu;
                            }
                            /* the unit holding P1: its position; a PolkaValue locks (:198) */
                            if (p1ok) {
                                const uint32_t b = (uint32_t)__builtin_ctz(lp) >> 3;
                                rk[R_P1] = pos + b;
                                if ((x >> (8u * b)) & X_PV) {
                                    rk[R_DF] = F_LOCK;
                                    sx[10] = vsel(u, b);
                                }
                            }
                            vc = x & alive & (~pre | vall) & nnb & (X_PV * 0x01010101u);
                            uint32_t msg = (x & ((pre & (X_TP * 0x01010101u)) | (alive & (X_TC * 0x01010101u)))) << 2;
                            msg |= atP & ((AGNES_VMSG_PRECOMMIT_NIL << AGNES_CODE_MSG_SHIFT) * 0x01010101u +
                                          (x & (X_PV * 0x01010101u)));
                            msg |= atC & ((AGNES_VMSG_DECISION << AGNES_CODE_MSG_SHIFT) * 0x01010101u);
                            return msg;
                        };
                        uint32_t* const sA = reinterpret_cast<uint32_t*>(sbh + 64u * kA);
                        uint32_t* const sB = reinterpret_cast<uint32_t*>(sbh + 64u * kB);
                        uint32_t cfx = cf;
                        if (!R1 && runs) {
                            /* C is the first PrecommitValue of ANY round (:211): crossed before a unit
                             * when an earlier unit of its instance in this chunk holds a commit
                             * candidate (another run's sums are not in the unit's own pass) */
                            const uint64_t XA = ballot((x0 & (X_C * 0x01010101u)) != 0u);
                            const uint64_t XB = ballot((x1 & (X_C * 0x01010101u)) != 0u);
                            /* the instance's first unit in the chunk: its last start at or before unit A */
                            const uint64_t iAm = SA & ((2ull << lane) - 1ull), iBm = SBm & ((1ull << lane) - 1ull);
                            const uint32_t fa = iAm ? 2u * (63u - (uint32_t)__builtin_clzll(iAm)) : 0u;
                            const uint32_t fb = iBm ? 2u * (63u - (uint32_t)__builtin_clzll(iBm)) + 1u : 0u;
                            const uint32_t ui = fa > fb ? fa : fb;
                            const uint64_t below = (1ull << lane) - 1ull;
                            const uint64_t fromA = ~((1ull << ((ui + 1u) >> 1)) - 1ull), fromB = ~((1ull << (ui >> 1)) - 1ull);
                            const bool xcA = ((XA & fromA & below) | (XB & fromB & below)) != 0ull;
                            const bool xcB = ((SBm >> lane) & 1ull) == 0ull && (xcA || ((XA >> lane) & 1ull) != 0ull);
                            cfx |= (xcA ? 2u : 0u) | (xcB ? 8u : 0u);
                        }
                        uint32_t v0, v1;
                        c0 |= unit(0u, x0, (cfx & 1u) || qA.x != NONE, (cfx & 2u) || qA.y != NONE, pos0, rA, sA, r8[0],
                                   eA.z, nn0, v0);
                        c1 |= unit(1u, x1, (cfx & 4u) || qB.x != NONE, (cfx & 8u) || qB.y != NONE, pos1, rB, sB, r8[1],
                                   eB.z, nn1, v1);
                        if (ballot((v0 | v1) != 0u)) { /* valid (:198, :202): the last candidate */
                            if (v0) {
                                const uint32_t b = (31u - (uint32_t)__builtin_clz(v0)) >> 3;
                                atomicMax(vtab + kA, ((unsigned long long)(pos0 + b + 1u) << 32) | vsel(0u, b));
                            }
                            if (v1) {
                                const uint32_t b = (31u - (uint32_t)__builtin_clz(v1)) >> 3;
                                atomicMax(vtab + kB, ((unsigned long long)(pos1 + b + 1u) << 32) | vsel(1u, b));
                            }
                        }
                    }
                    } /* (aligned units) */
                }

                if constexpr (REC) {
                    /* ---- the records themselves (agnes_tally_records): every vote whose event is
                     * Some (codes 1..5) as a 16-B agnes_seg_event in its instance's segment,
                     * out[offsets[i] + k] with k the instance's records before it, written while
                     * the votes are in registers (vote_executor.rs:20-36).  A record's slot is at
                     * most its own vote's position (k counts records of earlier votes of the
                     * instance), so the writes stay inside the n_votes records out holds ---- */
                    auto recm = [](uint32_t cw4) -> uint32_t { /* 0x80 in the bytes of votes with a record */
                        const uint32_t e = cw4 & 0x07070707u;
                        return (e + 0x7F7F7F7Fu) & ~(e + 0x7A7A7A7Au) & 0x80808080u;
                    };
                    const uint32_t h0 = recm(c0) & act0, h1 = recm(c1) & act1;
                    /* the instance's units: bytes before spI (U), or the lane's two words */
                    const uint32_t mI0 = U ? below_bytes((int32_t)spI) : 0xFFFFFFFFu;
                    const uint32_t mI1 = U ? below_bytes((int32_t)spI - 4) : 0u;
                    const uint32_t nA = (uint32_t)__builtin_popcount(h0 & mI0) + (uint32_t)__builtin_popcount(h1 & mI1);
                    const uint32_t nB = (uint32_t)__builtin_popcount(h0 & ~mI0) + (uint32_t)__builtin_popcount(h1 & ~mI1);
                    const bool fast = R1 || runs; /* a lane part of one segment is one executor per type */
                    const bool spl = R1 ? split : splitr;
                    /* the executors' split inside the lane: unit B from vote spE (U), or from vote 4 */
                    const uint32_t spE = U ? (R1 ? spI : (runs ? spR : 8u)) : 4u;
                    auto inBe = [&](uint32_t q) -> bool { return U ? q >= spE : q >= 4u; };
                    const uint32_t vok0 = okb0 & ~mark_bytes(nb0 << 3), vok1 = okb1 & ~mark_bytes(nb1 << 3); /* valid non-nil */
                    const uint32_t K2 = 2u * R;
                    auto key_of = [&](uint32_t q) -> uint32_t { /* batch instance, round, type */
                        const uint32_t bs = 8u * (q & 3u);
                        return (inB(q) ? kB : kA) * K2 + 2u * (((q < 4u ? r8[0] : r8[1]) >> bs) & 0xFFu) +
                               (((q < 4u ? t8[0] : t8[1]) >> bs) & 1u);
                    };
                    /* (lastc) the chunk's last non-nil vote of each executor of the carried
                     * instance, for the value slots of the next chunk */
                    if (lastc) {
                        if (lane < K2) vmx[lane] = 0ull;
                        __builtin_amdgcn_wave_barrier();
#pragma unroll
                        for (uint32_t q = 0; q < LV; ++q) {
                            const uint32_t bs = 8u * (q & 3u);
                            if ((((q < 4u ? vok0 : vok1) >> bs) & 1u) && (inB(q) ? kB : kA) == klast)
                                atomicMax(vmx + (key_of(q) - klast * K2),
                                          ((unsigned long long)(o8 + q + 1u) << 32) | value[q]);
                        }
                    }
                    if (ballot((h0 | h1) != 0u)) {
                        /* ranks inside the chunk: an exclusive scan of the lanes' last-instance counts,
                         * less the scan at the instance's first lane; plus the instance's records of
                         * earlier chunks (etab, before this chunk's counts are added below) */
                        const uint32_t Tn = split ? nB : nA + nB;
                        const uint32_t En = scan(Tn) - Tn;
                        const uint32_t rA = etab[kA] + En - (multi ? shfl(En, sA) : 0u);
                        const uint32_t rB = split ? etab[kB] : rA + nA;
                        const uint64_t gA = Sa + shfl(rl, kA), gB = Sa + shfl(rl, kB); /* instance starts */
                        /* the Value a PolkaValue / PrecommitValue carries (round_votes.rs:50-54): the
                         * vote's own when non-nil; for a nil vote the last non-nil value its executor
                         * took before it -- in the lane, else (one round, or runs: the segment is the
                         * executor's run up to its type) the last earlier lane of the segment holding
                         * one, else its value slot from before the chunk (carried in LDS: the instance
                         * continuing from the previous chunk) or Value{} */
                        uint32_t vv[LV];
                        uint32_t pend = 0u; /* bit s: a nil Value vote with a record, not resolved in the lane */
                        const uint64_t h64 = u64of(h0, h1);
                        bool hv0 = false, hv1 = false;
                        uint32_t lv0x = 0u, lv1x = 0u;
#pragma unroll
                        for (uint32_t q = 0; q < LV; ++q) {
                            if (U ? q == spE : (q == 4u && spl)) { hv0 = false; hv1 = false; }
                            const uint32_t bs = 8u * (q & 3u);
                            const uint32_t cq = ((q < 4u ? c0 : c1) >> bs) & 7u;
                            const bool tq = (((q < 4u ? t8[0] : t8[1]) >> bs) & 1u) != 0u;
                            const bool nn = (((q < 4u ? vok0 : vok1) >> bs) & 1u) != 0u;
                            const bool isv = cq == AGNES_CODE_POLKA_VALUE || cq == AGNES_CODE_PRECOMMIT_VALUE;
                            const bool hasT = fast && (tq ? hv1 : hv0);
                            const uint32_t lT = tq ? lv1x : lv0x;
                            vv[q] = nn ? value[q] : (isv && hasT ? lT : AGNES_NIL);
                            pend |= (isv && !nn && !hasT && ((h64 >> (8u * q + 7u)) & 1ull)) ? 1u << q : 0u;
                            if (nn) {
                                if (tq) { hv1 = true; lv1x = value[q]; } else { hv0 = true; lv0x = value[q]; }
                            }
                        }
                        /* the carried slot of a vote's executor: its instance continues from the
                         * previous chunk (the first segment) -- else the executor is new: Value{} */
                        auto carried = [&](uint32_t q) -> uint32_t {
                            const uint32_t k = inB(q) ? kB : kA;
                            return (cont0 && k == k0) ? A[4u * R + (key_of(q) - k * K2)] : 0u;
                        };
                        if (ballot(pend != 0u)) {
                            if (fast) {
                                const uint32_t sx = R1 ? (multi ? sA : 0u) : (multir ? sAr : 0u);
                                const uint64_t seg = (((1ull << lane) - 1ull) >> sx) << sx; /* lanes [sx, lane) */
                                const uint64_t B0 = ballot(hv0), B1 = ballot(hv1);
                                const uint64_t m0 = B0 & seg, m1 = B1 & seg;
                                const uint32_t j0 = m0 ? 63u - (uint32_t)__builtin_clzll(m0) : 0u;
                                const uint32_t j1 = m1 ? 63u - (uint32_t)__builtin_clzll(m1) : 0u;
                                const uint32_t f0 = shfl(lv0x, j0), f1 = shfl(lv1x, j1);
                                for (uint32_t q = 0; q < LV; ++q) {
                                    if (!((pend >> q) & 1u)) continue;
                                    const uint32_t bs = 8u * (q & 3u);
                                    const bool tq = (((q < 4u ? t8[0] : t8[1]) >> bs) & 1u) != 0u;
                                    vv[q] = ((!inBe(q) || !spl) && (tq ? m1 : m0)) ? (tq ? f1 : f0) : carried(q);
                                }
                            } else {
                                /* rounds revisited in the chunk: one executor (instance, round, type) at a
                                 * time -- its last non-nil vote before each of its pending votes, in the
                                 * lane, else in the last earlier lane holding one, else its slot */
                                uint32_t todo = pend;
                                for (;;) {
                                    const uint64_t lm = ballot(todo != 0u);
                                    if (!lm) break;
                                    const uint32_t kl = (uint32_t)__builtin_ctzll(lm);
                                    const uint32_t qs = (uint32_t)__builtin_ctz(rdl(todo, kl));
                                    uint32_t mykey = key_of(0u);
#pragma unroll
                                    for (uint32_t q = 1; q < LV; ++q) mykey = qs == q ? key_of(q) : mykey;
                                    const uint32_t KY = rdl(mykey, kl);
                                    bool has = false;
                                    uint32_t last = 0u, unres = 0u, inb = 0u;
#pragma unroll
                                    for (uint32_t q = 0; q < LV; ++q) {
                                        const uint32_t bs = 8u * (q & 3u);
                                        const bool mk = ((((q < 4u ? okb0 : okb1) >> bs) & 1u) != 0u) && key_of(q) == KY;
                                        /* (the lane's first pending vote is always of key KY: each
                                         * pass clears at least one bit of todo) */
                                        if (key_of(q) == KY && ((todo >> q) & 1u)) {
                                            inb |= 1u << q;
                                            if (has) vv[q] = last;
                                            else unres |= 1u << q;
                                        }
                                        if (mk && (((q < 4u ? vok0 : vok1) >> bs) & 1u)) {
                                            has = true;
                                            last = value[q];
                                        }
                                    }
                                    todo &= ~inb;
                                    const uint64_t M = ballot(has) & ((1ull << lane) - 1ull);
                                    const uint32_t fm = shfl(last, M ? 63u - (uint32_t)__builtin_clzll(M) : 0u);
                                    for (uint32_t q = 0; q < LV; ++q)
                                        if ((unres >> q) & 1u) vv[q] = M ? fm : carried(q);
                                }
                            }
                        }
                        /* the stores: one 16-B record per vote with an event.  Per word, bytewise:
                         * kind = event + 3 (AGNES_EV_POLKA_ANY ..), the message nibble, and the
                         * Value events (3, 5); a record's last word is assembled by two v_perm */
                        uint4* const pA = reinterpret_cast<uint4*>(a.rec_out) + gA + rA;
                        uint4* const pB = reinterpret_cast<uint4*>(a.rec_out) + gB + rB;
                        const uint64_t j0 = c + o8; /* a multiple of 8: + q never carries */
                        const uint32_t jlo = (uint32_t)j0, jhi = (uint32_t)(j0 >> 32);
                        const uint32_t e0 = c0 & 0x07070707u, e1 = c1 & 0x07070707u;
                        const uint32_t kd0 = e0 + 0x03030303u, kd1 = e1 + 0x03030303u;
                        const uint32_t ms0 = (c0 >> 4) & 0x0F0F0F0Fu, ms1 = (c1 >> 4) & 0x0F0F0F0Fu;
                        const uint32_t vm0 = zero_marks(e0 ^ 0x03030303u) | zero_marks(e0 ^ 0x05050505u);
                        const uint32_t vm1 = zero_marks(e1 ^ 0x03030303u) | zero_marks(e1 ^ 0x05050505u);
#pragma unroll
                        for (uint32_t q = 0; q < LV; ++q) {
                            const uint32_t b = q & 3u, bs = 8u * b;
                            if ((h64 >> (8u * q + 7u)) & 1ull) {
                                /* the vote's rank among its unit's records */
                                const uint32_t k = (uint32_t)__builtin_popcountll(h64 & ((1ull << (8u * q)) - 1ull)) -
                                                   (inB(q) ? nA : 0u);
                                /* [round, kind, message, 0] */
                                const uint32_t rk = __builtin_amdgcn_perm(q < 4u ? kd0 : kd1, q < 4u ? r8[0] : r8[1],
                                                                          b | ((4u + b) << 8) | 0x0C0C0000u);
                                const uint32_t w3 = __builtin_amdgcn_perm(q < 4u ? ms0 : ms1, rk, 0x0C000100u | ((4u + b) << 16));
                                const bool isv = (((q < 4u ? vm0 : vm1) >> (bs + 7u)) & 1u) != 0u;
                                (inB(q) ? pB : pA)[k] = make_uint4(jlo | q, jhi, isv ? vv[q] : AGNES_NIL, w3);
                            }
                        }
                    }
                    if (lastc) { /* the carried instance's value slots after the chunk (row B) */
                        __builtin_amdgcn_wave_barrier();
                        if (lane < K2) {
                            const unsigned long long x = vmx[lane];
                            if (x) B[4u * R + lane] = (uint32_t)x;
                        }
                        __builtin_amdgcn_wave_barrier();
                    }
                }

                if constexpr (EDG) {
                    /* ---- the edge summary (agnes_tally_edges, orc_edges): a valid vote is an edge
                     * when its executor's state -- code bits 0..3 | the last non-zero message << 4
                     * -- changes.  On this route (no RoundSkip) a message belongs to one event
                     * code (TimeoutPrevote to PolkaAny, TimeoutPrecommit to PrecommitAny, the
                     * precommit to PolkaNil / PolkaValue at P1, the Decision to PrecommitValue at
                     * C) and an executor's messages only switch off (P1, C), never on, so the
                     * first vote of a code carries its message or none of the code's votes does:
                     * the state changes exactly where the event code changes.  The code before a
                     * vote is to_event(type, level of its executor's sums without it) -- computed
                     * in K3 (lvb) -- so an edge needs no lookup; only its record's previous state
                     * needs the executor's last message: the last earlier edge of the executor
                     * with one (in the lane, else the last earlier lane of the segment, else the
                     * state carried in LDS, elab, which changes only at edges). ---- */
                    const uint32_t cbf0 = __builtin_amdgcn_perm(EV_HI, EV_LO, lvb0 | (ts0c >> 3));
                    const uint32_t cbf1 = __builtin_amdgcn_perm(EV_HI, EV_LO, lvb1 | (ts1c >> 3));
                    auto nzb = [](uint32_t x) -> uint32_t { /* 0x80 in the non-zero bytes of x */
                        return ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu | x) & 0x80808080u;
                    };
                    const uint32_t em0 = nzb((c0 ^ cbf0) & 0x07070707u) & okb0; /* (okb: inside the stream) */
                    const uint32_t em1 = nzb((c1 ^ cbf1) & 0x07070707u) & okb1;
                    /* the instance's units: bytes before spI (U), or the lane's two words */
                    const uint32_t mI0 = U ? below_bytes((int32_t)spI) : 0xFFFFFFFFu;
                    const uint32_t mI1 = U ? below_bytes((int32_t)spI - 4) : 0u;
                    const uint32_t nA = (uint32_t)__builtin_popcount(em0 & mI0) + (uint32_t)__builtin_popcount(em1 & mI1);
                    const uint32_t nB = (uint32_t)__builtin_popcount(em0 & ~mI0) + (uint32_t)__builtin_popcount(em1 & ~mI1);
                    if (ballot((em0 | em1) != 0u)) {
                        const bool fast = R1 || runs;
                        const bool spl = R1 ? split : splitr;
                        /* the executors' split inside the lane: unit B from vote spE (U), or from vote 4 */
                        const uint32_t spE = U ? (R1 ? spI : (runs ? spR : 8u)) : 4u;
                        auto inBe = [&](uint32_t q) -> bool { return U ? q >= spE : q >= 4u; };
                        const uint32_t K2 = 2u * R;
                        auto key_of = [&](uint32_t q) -> uint32_t { /* instance k, round, type */
                            const uint32_t bs = 8u * (q & 3u);
                            const uint32_t r = ((q < 4u ? r8[0] : r8[1]) >> bs) & 0xFFu, t = ((q < 4u ? t8[0] : t8[1]) >> bs) & 1u;
                            return (inB(q) ? kB : kA) * K2 + 2u * r + t;
                        };
                        /* the lane's edges one at a time (a chunk holds few: 2 % of C2's votes) */
                        auto byteq = [](uint32_t x0, uint32_t x1, uint32_t q) -> uint32_t {
                            return ((q < 4u ? x0 : x1) >> (8u * (q & 3u))) & 0xFFu;
                        };
                        auto nib = [](uint32_t x) -> uint32_t { return ((x * 0x01020408u) >> 24) & 0xFu; };
                        const uint32_t emsk = nib(em0 >> 7) | (nib(em1 >> 7) << 4); /* bit q: vote q is an edge */
                        const uint32_t segA = R1 ? kA : (kA * 16u + uA), segB = R1 ? kB : (kB * 16u + uB);
                        uint32_t phw = 0u, php = 0u; /* the last message before each edge (nibble q); bit q: not yet known */
                        bool hm0 = false, hm1 = false, rs = false;
                        uint32_t lm0 = 0u, lm1 = 0u;
                        uint32_t g0 = 0xFFFFFFFFu, g1 = 0xFFFFFFFFu; /* the segment of the lane's first edge per type */
                        for (uint32_t m = emsk; m; m &= m - 1u) {
                            const uint32_t q = (uint32_t)__builtin_ctz(m);
                            if (spl && inBe(q) && !rs) { hm0 = false; hm1 = false; rs = true; }
                            const bool tq = (byteq(t8[0], t8[1], q) & 1u) != 0u;
                            const uint32_t msg = byteq(c0, c1, q) >> 4;
                            const uint32_t sg = inBe(q) ? segB : segA;
                            if (fast && (tq ? hm1 : hm0)) phw |= (tq ? lm1 : lm0) << (4u * q);
                            else php |= 1u << q;
                            if (msg) {
                                if (tq) { hm1 = true; lm1 = msg; } else { hm0 = true; lm0 = msg; }
                            }
                            if (tq) g1 = g1 == 0xFFFFFFFFu ? sg : g1;
                            else g0 = g0 == 0xFFFFFFFFu ? sg : g0;
                        }
                        if (spl && !rs) { hm0 = false; hm1 = false; } /* the lane's last part: unit B */
                        if (fast) {
                            const uint32_t sx = R1 ? (multi ? sA : 0u) : (multir ? sAr : 0u);
                            const uint64_t segm = (((1ull << lane) - 1ull) >> sx) << sx;
                            const uint64_t M0 = ballot(hm0) & segm, M1 = ballot(hm1) & segm;
                            const uint32_t f0 = shfl(lm0, M0 ? 63u - (uint32_t)__builtin_clzll(M0) : 0u);
                            const uint32_t f1 = shfl(lm1, M1 ? 63u - (uint32_t)__builtin_clzll(M1) : 0u);
                            for (uint32_t m = emsk & php; m; m &= m - 1u) {
                                const uint32_t q = (uint32_t)__builtin_ctz(m);
                                const uint32_t tb = byteq(t8[0], t8[1], q) & 1u;
                                const bool gm = (!inBe(q) || !spl) && (tb ? M1 : M0) != 0ull;
                                const uint32_t key = (inB(q) ? kB : kA) * K2 + 2u * byteq(r8[0], r8[1], q) + tb;
                                phw |= (gm ? (tb ? f1 : f0) : (uint32_t)(elab[key] >> 4)) << (4u * q);
                            }
                            /* each (segment, type)'s last edge in the chunk carries the state out: a
                             * later edge of the lane, or the first edge of that type in the next lane
                             * holding one, in the same segment means it is not the last */
                            const uint64_t above = ~((2ull << lane) - 1ull);
                            const uint64_t N0 = ballot(g0 != 0xFFFFFFFFu) & above, N1 = ballot(g1 != 0xFFFFFFFFu) & above;
                            uint32_t nx0 = shfl(g0, N0 ? (uint32_t)__builtin_ctzll(N0) : lane);
                            uint32_t nx1 = shfl(g1, N1 ? (uint32_t)__builtin_ctzll(N1) : lane);
                            nx0 = N0 ? nx0 : 0xFFFFFFFFu;
                            nx1 = N1 ? nx1 : 0xFFFFFFFFu;
                            for (uint32_t m = emsk; m;) {
                                const uint32_t q = 31u - (uint32_t)__builtin_clz(m);
                                m &= ~(1u << q);
                                const uint32_t tb = byteq(t8[0], t8[1], q) & 1u;
                                const uint32_t sg = inBe(q) ? segB : segA;
                                if ((tb ? nx1 : nx0) != sg) {
                                    const uint32_t cb = byteq(c0, c1, q);
                                    const uint32_t key = (inB(q) ? kB : kA) * K2 + 2u * byteq(r8[0], r8[1], q) + tb;
                                    elab[key] = (unsigned char)((cb & 0xFu) | ((cb >> 4) ? (cb & 0xF0u) : (((phw >> (4u * q)) & 0xFu) << 4)));
                                }
                                if (tb) nx1 = sg;
                                else nx0 = sg;
                            }
                        } else {
                            /* rounds revisited in the chunk: the edges one key at a time */
                            uint32_t todo = emsk;
                            for (;;) {
                                const uint64_t lm = ballot(todo != 0u);
                                if (!lm) break;
                                const uint32_t kl = (uint32_t)__builtin_ctzll(lm);
                                const uint32_t ks = (uint32_t)__builtin_ctz(rdl(todo, kl));
                                uint32_t mykey = key_of(0u);
#pragma unroll
                                for (uint32_t q = 1; q < LV; ++q) mykey = ks == q ? key_of(q) : mykey;
                                const uint32_t KY = rdl(mykey, kl);
                                bool hm = false;
                                uint32_t lmx = 0u, inb = 0u, fin = 0u;
#pragma unroll
                                for (uint32_t q = 0; q < LV; ++q) {
                                    if (!((todo >> q) & 1u) || key_of(q) != KY) continue;
                                    inb |= 1u << q;
                                    const uint32_t cb = ((q < 4u ? c0 : c1) >> (8u * (q & 3u))) & 0xFFu;
                                    phw &= ~(0xFu << (4u * q));
                                    php &= ~(1u << q);
                                    if (hm) phw |= lmx << (4u * q);
                                    else php |= 1u << q;
                                    if (cb >> 4) { hm = true; lmx = cb >> 4; }
                                }
                                todo &= ~inb;
                                const uint64_t M = ballot(hm) & ((1ull << lane) - 1ull);
                                const uint32_t fm = shfl(lmx, M ? 63u - (uint32_t)__builtin_clzll(M) : 0u);
                                const uint32_t car = elab[KY] >> 4;
#pragma unroll
                                for (uint32_t q = 0; q < LV; ++q) {
                                    if (!((inb >> q) & 1u)) continue;
                                    if ((php >> q) & 1u) phw |= (M ? fm : car) << (4u * q);
                                    const uint32_t cb = ((q < 4u ? c0 : c1) >> (8u * (q & 3u))) & 0xFFu;
                                    fin = (cb & 0xFu) | ((cb >> 4) ? (cb & 0xF0u) : (((phw >> (4u * q)) & 0xFu) << 4));
                                }
                                const uint64_t H2 = ballot(inb != 0u);
                                const uint32_t fv = rdl(fin, 63u - (uint32_t)__builtin_clzll(H2));
                                __builtin_amdgcn_wave_barrier();
                                if (lane == 0u) elab[KY] = (unsigned char)fv;
                                __builtin_amdgcn_wave_barrier();
                            }
                        }
                        __builtin_amdgcn_wave_barrier();
                        /* the records at the instance's segment: rank = the instance's edges before
                         * the chunk (etab) + the edges before it in the chunk */
                        const uint32_t Tn = split ? nB : nA + nB;
                        const uint32_t En = scan(Tn) - Tn;
                        const uint32_t rA = etab[kA] + En - (multi ? shfl(En, sA) : 0u);
                        const uint32_t rB = split ? etab[kB] : rA + nA;
                        const uint64_t gA = Sa + shfl(rl, kA), gB = Sa + shfl(rl, kB);
                        /* (U) the instance's unit B: votes spI .. 7 */
                        const uint32_t mIq = U ? (spI < 8u ? (0xFFu << spI) & 0xFFu : 0u) : 0xF0u;
                        for (uint32_t m = emsk; m; m &= m - 1u) {
                            const uint32_t q = (uint32_t)__builtin_ctz(m);
                            const uint32_t k = (inB(q) ? rB : rA) + (uint32_t)__builtin_popcount(emsk & ((1u << q) - 1u) &
                                                                                                  (inB(q) ? mIq : ~mIq));
                            const uint32_t cb = byteq(c0, c1, q), rq = byteq(r8[0], r8[1], q), tq = byteq(t8[0], t8[1], q) & 1u;
                            const uint32_t prev = (byteq(cbf0, cbf1, q) & 0xFu) | (((phw >> (4u * q)) & 0xFu) << 4);
                            const uint64_t j = c + o8 + q;
                            const uint4 rec = make_uint4((uint32_t)j, (uint32_t)(j >> 32), H.s0 + (inB(q) ? kB : kA),
                                                         rq | (tq << 8) | (cb << 16) | (prev << 24));
                            reinterpret_cast<uint4*>(a.rec_out)[(inB(q) ? gB : gA) + k] = rec;
                        }
                        __builtin_amdgcn_wave_barrier();
                        atomicAdd(etab + kA, kA == kB ? nA + nB : nA);
                        atomicAdd(etab + kB, kA == kB ? 0u : nB);
                    }
                }

                if (EVC && !EDG) { /* records per unit: the votes whose event is Some (codes 1..5) */
                    auto recs = [](uint32_t cw4) -> uint32_t {
                        const uint32_t e = cw4 & 0x07070707u;
                        const uint32_t nz = (e + 0x7F7F7F7Fu) & 0x80808080u; /* event != None        */
                        const uint32_t iv = (e + 0x7A7A7A7Au) & 0x80808080u; /* INVALID / REJECTED   */
                        return (uint32_t)__builtin_popcount(nz & ~iv);
                    };
                    uint32_t nA, nB;
                    if (U) { /* (U) the units split at the instance start spI */
                        const uint32_t m0 = below_bytes((int32_t)spI), m1 = below_bytes((int32_t)spI - 4);
                        nA = recs(c0 & act0 & m0) + recs(c1 & act1 & m1);
                        nB = recs(c0 & act0 & ~m0) + recs(c1 & act1 & ~m1);
                    } else {
                        nA = actA ? recs(c0) : 0u;
                        nB = actB ? recs(c1) : 0u;
                    }
                    atomicAdd(etab + kA, kA == kB ? nA + nB : nA);
                    atomicAdd(etab + kB, kA == kB ? 0u : nB);
                }

                /* codes (deferred) */
                dc0 = c0;
                dc1 = c1;
                if (U) {
                    dc_act = (act0 & act1) == 0xFFFFFFFFu ? 3u : 0u;
                    dcm0 = act0;
                    dcm1 = act1;
                } else {
                    dc_act = (actA ? 1u : 0u) | (actB ? 2u : 0u);
                }
                dc_at = c;
                dc_u = U;
                __builtin_amdgcn_wave_barrier();
            }
            };
            if constexpr (RG) {
                if (H.rag) chunks(std::true_type{});
                else chunks(std::false_type{});
            } else {
                chunks(std::false_type{});
            }
        }
        /* batch end: the record counts and the States out (a walk-list batch's are the
         * walk kernel's) */
        if (EVC && m && H.go) {
            __builtin_amdgcn_wave_barrier();
            const uint32_t Le = rdl(H.olo, m) - rdl(H.olo, 0u) + (rdl(H.olo, 0u) & 127u);
            if (lane < m) a.ev_counts[H.s0 + lane] = Le ? (uint64_t)etab[lane] : 0ull;
        }
        if (SM && m && H.go) {
            if (smf) { /* no vote: the States as they came */
                dma_wait();
                for (uint32_t j = lane; j < 4u * m; j += 64u)
                    st_out(reinterpret_cast<uint4*>(a.states + H.s0) + j, *reinterpret_cast<const uint4*>(sbh + 16u * j));
            } else {
                finalize(m, H.s0, sbh);
            }
        }
        FDIAG(if (lane == 0) {
                  if (dg_b < 30u) {
                      const uint64_t nvb = u64of(rdl(H.olo, m), rdl(H.ohi, m)) - u64of(rdl(H.olo, 0u), rdl(H.ohi, 0u));
                      dg[4u + 2u * dg_b] = dg_t;
                      dg[5u + 2u * dg_b] = (unsigned long long)m | ((unsigned long long)(dg_c - dg_c0) << 16) | (nvb << 32);
                  }
              }
              ++dg_b;)
        if (AGNES_FLOW_AHEAD == 1 && N.stage == 0u) { /* a batch without chunks: N's slot now */
            range_of(rdl(tq, 0u), N.s0, N.e0);
            hdr1(N);
        }
        if (N.s0 >= N.e0) break;
        if (N.stage < 3u) { /* a short batch: the rest of the header now */
            if (N.stage == 1u) hdr2(N);
            hdr3(N);
            if (N.go) dma_states(N, spar ^ 1u);
        }
        H = N;
        spar ^= 1u;
#if AGNES_FLOW_AHEAD == 1
        /* one batch ahead only: the next slot is claimed now and read at the next chunk's
         * top, so at the queue's end a wave holds no claimed batch beyond the next one */
        if (lane == 0) tq = atomicAdd(ctr, 1u) + 2u * qS;
        N.stage = 0u;
        N.s0 = 0u;
        N.e0 = 1u; /* (pending: not empty) */
#else
        range_of(rdl(tq, 0u), N.s0, N.e0); /* the batch after, grabbed one batch ago */
        if (lane == 0) tq = atomicAdd(ctr, 1u) + 2u * qS;
        hdr1(N);
#endif
    }
    flush();
    const uint32_t nb = rdl(scan(bad), 63u);
    if (lane == 0 && nb) add_invalid(a.n_invalid, (unsigned long long)nb);
    FDIAG(if (lane == 0) {
        dg[1] = __builtin_amdgcn_s_memrealtime();
        dg[2] = dg_b;
        dg[3] = dg_c;
    })
}

} // namespace flow
} // namespace agnes

/* ------------------------------------------------------------------ */
/* launcher                                                            */

/* One flow kernel (RG: with the unaligned-stream loop) */
template <bool SM, bool R1, bool EVC, bool W64, bool REC = false, bool EDG = false, bool U = false>
static hipError_t launch_flow_k(const agnes_tally_args* a, int num_cus, hipStream_t st) {
    const uint32_t n = a->vb.n_instances;
    if (n == 0) return hipSuccess;
    using agnes::flow::flow;
    const void* fns[2] = {reinterpret_cast<const void*>(&flow<false, SM, R1, EVC, W64, REC, EDG, U>),
                          reinterpret_cast<const void*>(&flow<true, SM, R1, EVC, W64, REC, EDG, U>)};
    const uint32_t lpw = agnes::flow::lds_bytes(SM, a->max_rounds, EVC, W64, EDG, REC);
    const uint64_t wave_lds = (uint64_t)lpw * AGNES_WAVES_PER_BLOCK;
    const uint64_t pcb = agnes::align16((W64 ? 8ull : 4ull) * a->n_sets * a->n_vals);
    /* blocks per CU from the occupancy query; the LDS power table only where it
     * costs no occupancy.  Cached per (kernel, LDS shape). */
    struct Occ { const void* fn; uint64_t wave_lds, pcb; int per_cu; bool pc; };
    static thread_local Occ occ[8];
    static thread_local unsigned occ_next = 0;
    Occ* o = nullptr;
    for (auto& c : occ)
        if (c.per_cu && c.fn == fns[0] && c.wave_lds == wave_lds && c.pcb == pcb) o = &c;
    if (!o) {
        auto per_cu = [&](const void* fn, uint64_t lds) -> int {
            if (lds > 160u * 1024u) return 0;
            if (lds > 48u * 1024u &&
                hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
                return 0;
            int k = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&k, fn, 256, (size_t)lds) != hipSuccess) k = 0;
            return k;
        };
        const int k0 = per_cu(fns[0], wave_lds);
        const int k1 = pcb <= 32u * 1024u ? per_cu(fns[1], wave_lds + pcb) : 0;
        o = &occ[occ_next++ % 8];
        *o = Occ{fns[0], wave_lds, pcb, k0 > 0 ? k0 : 1, false};
        if (k1 > 0 && k1 >= k0) {
            o->per_cu = k1;
            o->pc = true;
        }
    }
    agnes_tally_args b = *a;
    b.set_cache = 0;
    b.power_cache = o->pc ? (uint32_t)pcb : 0u;
    const uint64_t lds = wave_lds + b.power_cache;
    const void* fn = fns[o->pc ? 1 : 0];
    { /* batches of FB, fewer when that leaves a wave under AGNES_FLOW_BATCHES_PER_WAVE */
        const uint64_t waves = (uint64_t)(num_cus > 0 ? num_cus : 256) * (uint64_t)o->per_cu * AGNES_WAVES_PER_BLOCK;
        uint64_t fbx = AGNES_FLOW_BATCHES_PER_WAVE ? (uint64_t)n / (waves * AGNES_FLOW_BATCHES_PER_WAVE) : agnes::flow::FB;
        fbx = fbx < 4u ? 4u : (fbx > agnes::flow::FB ? agnes::flow::FB : fbx);
        b.batch = (uint32_t)fbx;
        /* the tail: batches of about AGNES_FLOW_TAIL_VOTES votes, AGNES_FLOW_TAIL_PER_WAVE
         * per wave, at most a quarter of the instances */
        b.tail_batch = 0u;
        b.tail_n = 0u;
        if (AGNES_FLOW_TAIL_VOTES && a->vb.n_votes) {
            const uint64_t avg = (a->vb.n_votes + n - 1u) / n;
            uint64_t tb = ((uint64_t)AGNES_FLOW_TAIL_VOTES + avg - 1u) / avg;
            tb = tb < 1u ? 1u : (tb > fbx ? fbx : tb);
            uint64_t tn = (uint64_t)AGNES_FLOW_TAIL_PER_WAVE * waves * tb;
            if (tn > n / 4u) tn = n / 4u;
            b.tail_batch = (uint32_t)tb;
            b.tail_n = (uint32_t)tn;
        }
    }
    if (lds > 48u * 1024u) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    const uint64_t ncu = (uint64_t)(num_cus > 0 ? num_cus : 256);
    uint64_t blocks = ((uint64_t)n + 4u * AGNES_WAVES_PER_BLOCK - 1u) / (4u * AGNES_WAVES_PER_BLOCK);
    const uint64_t cap = ncu * (uint64_t)o->per_cu;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    if (o->pc) hipLaunchKernelGGL((flow<true, SM, R1, EVC, W64, REC, EDG, U>), dim3((uint32_t)blocks), dim3(256), (size_t)lds, st, b, lpw);
    else hipLaunchKernelGGL((flow<false, SM, R1, EVC, W64, REC, EDG, U>), dim3((uint32_t)blocks), dim3(256), (size_t)lds, st, b, lpw);
    return hipGetLastError();
}

#ifdef AGNES_FLOW_DIAG
/* diagnostics build only: arm the per-wave record buffer (device memory, 64 u64 per wave
 * of the grid; nullptr disarms) */
extern "C" int agnes_flow_diag_arm(unsigned long long* dev_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(agnes::flow::flow_diag_buf), &dev_buf, sizeof(dev_buf)) == hipSuccess ? 0 : -1;
}
#endif

bool agnes_flow_supported(const agnes_tally_args* a) {
    /* rounds 0..14 in the byte checks; the per-wave LDS fits the waves a CU holds (16
     * without the State machine, 12 with it: its VGPRs allow 3 waves per SIMD; the u64
     * kernel's allow 2) */
    const bool sm = (a->flags & AGNES_FLAG_STATE_MACHINE) != 0 && a->states != nullptr;
    const uint32_t waves = a->w64 ? 8u : (sm ? 12u : 16u);
    return a->max_rounds <= 15u && agnes::flow::lds_bytes(sm, a->max_rounds, a->ev_counts != nullptr, a->w64 != 0u,
                                                          a->edges != 0u, a->rec_out && !a->edges) * waves <= 160u * 1024u;
}

bool agnes_flow_counts_events(uint32_t flags, uint32_t max_rounds, bool edges, bool rec) {
    const bool sm = (flags & AGNES_FLAG_STATE_MACHINE) != 0;
    return max_rounds <= 15u &&
           agnes::flow::lds_bytes(sm, max_rounds, true, false, edges, rec && !edges) * (sm ? 12u : 16u) <= 160u * 1024u;
}

template <bool G>
static hipError_t launch_flow_u32(const agnes_tally_args* a, int num_cus, hipStream_t st, bool sm, bool r1) {
    if (a->rec_out && a->edges) { /* agnes_tally_edges: the edge counts and records */
        if (!a->ev_counts) return hipErrorInvalidValue;
        if (r1) return sm ? launch_flow_k<true, true, true, false, false, true, G>(a, num_cus, st)
                          : launch_flow_k<false, true, true, false, false, true, G>(a, num_cus, st);
        return sm ? launch_flow_k<true, false, true, false, false, true, G>(a, num_cus, st)
                  : launch_flow_k<false, false, true, false, false, true, G>(a, num_cus, st);
    }
    if (a->rec_out) { /* agnes_tally_records: counts and the records themselves */
        if (!a->ev_counts) return hipErrorInvalidValue;
        if (r1) return sm ? launch_flow_k<true, true, true, false, true, false, G>(a, num_cus, st)
                          : launch_flow_k<false, true, true, false, true, false, G>(a, num_cus, st);
        return sm ? launch_flow_k<true, false, true, false, true, false, G>(a, num_cus, st)
                  : launch_flow_k<false, false, true, false, true, false, G>(a, num_cus, st);
    }
    if (a->ev_counts) {
        if (r1) return sm ? launch_flow_k<true, true, true, false, false, false, G>(a, num_cus, st)
                          : launch_flow_k<false, true, true, false, false, false, G>(a, num_cus, st);
        return sm ? launch_flow_k<true, false, true, false, false, false, G>(a, num_cus, st)
                  : launch_flow_k<false, false, true, false, false, false, G>(a, num_cus, st);
    }
    if (r1) return sm ? launch_flow_k<true, true, false, false, false, false, G>(a, num_cus, st)
                      : launch_flow_k<false, true, false, false, false, false, G>(a, num_cus, st);
    return sm ? launch_flow_k<true, false, false, false, false, false, G>(a, num_cus, st)
              : launch_flow_k<false, false, false, false, false, false, G>(a, num_cus, st);
}

namespace agnes {
namespace flow {
/* the gate words, one per block (its share of the offsets holds one off a multiple of 4),
 * and the call's counters zeroed (zw words at zb: the memset this launch replaces) */
__global__ __launch_bounds__(256) void flow_prep(const uint64_t* offsets, uint64_t n1, uint32_t* zb, uint32_t zw,
                                                 uint32_t* slots) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t < zw) zb[t] = 0u;
    const uint64_t S = (uint64_t)gridDim.x * 256u;
    uint64_t acc = 0, i = t;
    for (; i + 3u * S < n1; i += 4u * S) /* four independent loads in flight */
        acc |= offsets[i] | offsets[i + S] | offsets[i + 2u * S] | offsets[i + 3u * S];
    for (; i < n1; i += S) acc |= offsets[i];
    const bool odd = __syncthreads_or((acc & 3u) != 0u);
    if (threadIdx.x == 0) slots[blockIdx.x] = odd ? 1u : 0u;
}
} // namespace flow
} // namespace agnes

bool agnes_flow_rg(const agnes_tally_args* a) { return AGNES_FLOW_RG && !a->w64; }

bool agnes_flow_rg_build() { return AGNES_FLOW_RG != 0; }

hipError_t agnes_launch_flow_prep(const agnes_tally_args* a, hipStream_t st) {
    /* the invalid count's stripes and the queue words, up to the gate words */
    constexpr uint32_t ZW = AGNES_ERR_BYTES / 4u + AGNES_PREP_SLOT0;
    static_assert(ZW <= AGNES_PREP_SLOTS * 256u, "one word per thread");
    hipLaunchKernelGGL(agnes::flow::flow_prep, dim3(AGNES_PREP_SLOTS), dim3(256), 0, st, a->vb.offsets,
                       (uint64_t)a->vb.n_instances + 1u, reinterpret_cast<uint32_t*>(a->n_invalid),
                       a->prep_zero ? ZW : 0u, a->list_count + AGNES_PREP_SLOT0);
    return hipGetLastError();
}

hipError_t agnes_launch_flow(const agnes_tally_args* a, int num_cus, hipStream_t st, bool rg) {
    const bool sm = (a->flags & AGNES_FLAG_STATE_MACHINE) != 0 && a->states != nullptr;
    const bool r1 = a->max_rounds == 1u;
    if (a->w64) { /* the u64 domain: no record counts (agnes_sweep_supported); unaligned streams to the walk */
        if (a->ev_counts || rg) return hipErrorInvalidValue;
        if (r1) return sm ? launch_flow_k<true, true, false, true>(a, num_cus, st) : launch_flow_k<false, true, false, true>(a, num_cus, st);
        return sm ? launch_flow_k<true, false, false, true>(a, num_cus, st) : launch_flow_k<false, false, false, true>(a, num_cus, st);
    }
#if AGNES_FLOW_FORCE_U
    { /* (A/B builds) every stream through the RG kernel's unaligned-stream loop, ungated */
        if (!rg) return hipSuccess;
        agnes_tally_args b = *a;
        b.gate = 0u;
        return launch_flow_u32<true>(&b, num_cus, st, sm, r1);
    }
#endif
    if (rg) return launch_flow_u32<AGNES_FLOW_RG != 0>(a, num_cus, st, sm, r1);
    return launch_flow_u32<false>(a, num_cus, st, sm, r1);
}
