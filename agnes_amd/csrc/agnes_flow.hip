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
#ifndef AGNES_FLOW_RG_ALIGNED
#define AGNES_FLOW_RG_ALIGNED 1 /* the RG kernel walks a call's aligned batches with the aligned loop (0: the U loop) */
#endif
#ifndef AGNES_FLOW_FORCE_U
#define AGNES_FLOW_FORCE_U 0 /* A/B builds only: every stream through the unaligned-stream loop */
#endif
#ifndef AGNES_FLOW_CODE_VMCNT
/* 1: after a whole-chunk code store the next chunk waits vmcnt(1), leaving that store in
 * flight -- which assumes loads and stores retire from vmcnt in issue order, an ordering
 * LLVM's waitcnt pass does not assume for mixed loads and stores.  Measured worth nothing
 * in round 6 (same box: c3shard 0.3672 / 0.3592 ms with it, 0.3634 / 0.3636 without; C3
 * 2.401 / 2.402 vs 2.385 / 2.379), so the exact vmcnt(0) is the default. */
#define AGNES_FLOW_CODE_VMCNT 0
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
        h.rag = (RG && (AGNES_FLOW_FORCE_U || !AGNES_FLOW_RG_ALIGNED)) || ballot(lane <= m && (h.olo & 3u) != 0u) != 0ull;
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
            if constexpr (RG && AGNES_FLOW_RG_ALIGNED && !W64) { /* (W64: its registers hold one loop) */
                if (H.rag) {
                    constexpr bool U = true;
#include "agnes_flow_chunks.inc"
                } else {
                    constexpr bool U = false;
#include "agnes_flow_chunks.inc"
                }
            } else if constexpr (RG) {
                constexpr bool U = true;
#include "agnes_flow_chunks.inc"
            } else {
                constexpr bool U = false;
#include "agnes_flow_chunks.inc"
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
    for (; i + 7u * S < n1; i += 8u * S) /* eight independent loads in flight (C2's 8 MB: two round trips) */
        acc |= offsets[i] | offsets[i + S] | offsets[i + 2u * S] | offsets[i + 3u * S] | offsets[i + 4u * S] |
               offsets[i + 5u * S] | offsets[i + 6u * S] | offsets[i + 7u * S];
    for (; i < n1; i += S) acc |= offsets[i];
    const bool odd = __syncthreads_or((acc & 3u) != 0u);
    if (threadIdx.x == 0) slots[blockIdx.x] = odd ? 1u : 0u;
}
} // namespace flow
} // namespace agnes

bool agnes_flow_rg(const agnes_tally_args*) { return AGNES_FLOW_RG != 0; }

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
    if (a->w64) { /* the u64 domain: no record counts (agnes_sweep_supported); (rg) the unaligned-stream loop */
        if (a->ev_counts) return hipErrorInvalidValue;
        if (rg) { /* the unaligned-stream loop only (every batch of such a call through it) */
            if (r1) return sm ? launch_flow_k<true, true, false, true, false, false, true>(a, num_cus, st)
                              : launch_flow_k<false, true, false, true, false, false, true>(a, num_cus, st);
            return sm ? launch_flow_k<true, false, false, true, false, false, true>(a, num_cus, st)
                      : launch_flow_k<false, false, false, true, false, false, true>(a, num_cus, st);
        }
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
