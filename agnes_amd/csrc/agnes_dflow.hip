/*
 * agnes_dflow.hip — DEDUP and RoundSkip batches (BASELINE C4) as ONE pass over the
 * vote stream: first-vote filter -> weight gather -> ordered tally -> quorum ->
 * event, plus the +1/3 RoundSkip bit (consensus_executor.rs:61-69 with the
 * extensions of SURVEY.md §0 gaps 1 and 4).
 *
 * The flow kernel (agnes_flow.hip) owns REFERENCE batches whose rounds come in runs.
 * A C4 stream breaks both of its assumptions: 20 % of the votes are duplicates or
 * equivocations that must not count (the first vote of (instance, round, type,
 * validator) wins, SURVEY.md gap 1, ahead of round_votes.rs:48-56), and 5 % are
 * early votes of the next round sprinkled through the current one, so one 8-vote
 * lane holds votes of several (round, type) executors.  The per-instance kernel
 * (agnes_fast.hip) answers that with one full pass over the chunk per (round, type)
 * key present (~5 per C4 chunk).  Here every chunk takes ONE tally pass whatever
 * the interleaving: the chunk's accepted votes are counting-sorted by (round, type)
 * in LDS, which makes every executor's votes contiguous in stream order, and the
 * ordered tally becomes a segmented scan over the sorted chunk.
 *
 * Work: a queue hands a wave batches of up to FB consecutive instances, walked as
 * one vote stream in 512-vote chunks (lane l: votes 8l .. 8l+7), every column by
 * non-temporal LDS-DMA one chunk ahead.  Instance starts may fall anywhere (C4's
 * instances are 375 votes per round): each vote's instance SEGMENT is derived from
 * the starts inside the chunk.  Per chunk:
 *
 *   K1   the boundary's checks (round < R, type <= 1, the vote names its instance,
 *        validator in the set) and the weight gather (power table in block LDS when
 *        it fits, else L2);
 *   F    first-vote flags, one pass per instance of the chunk: an LDS table over
 *        (round, type, validator) takes atomic max of (instance epoch << lb |
 *        LMASK - vote index in the instance), so the earliest vote of a key holds
 *        the entry across chunks without clearing it.  A vote is accepted (DEDUP)
 *        when the entry is its own; it is its round's first vote of its validator
 *        (RoundSkip weight) when moreover the other type's entry is older;
 *   S    the accepted votes of up to NSEG instances counting-sorted by key =
 *        round << 1 | type (nibble counters per lane, one wave scan), scattered to
 *        LDS as {weight, position | nil | first | key | instance};
 *   K2/3 over the sorted chunk, lane-serial prefixes of (value, nil) per run of
 *        equal (instance, key) — a run is one RoundVotes executor's votes in stream
 *        order — and one wave scan of the lanes' last-run totals; is_quorum
 *        (round_votes.rs:31-33) on the running sums plus the carried executor, the
 *        precedence Value > Nil > Any (:58-66) as a level written back to the
 *        vote's stream position;
 *   RS   RoundSkip (+1/3 of the distinct validators voting in the vote's round):
 *        the sorted pass also sums the first-vote weights per run; a (instance,
 *        round) whose carried plus chunk total crosses floor(total/3) in this chunk
 *        is scanned once in stream order for its crossing vote, and every accepted
 *        vote of it from there on carries the SKIP bit (the sum only grows);
 *   codes to_event (vote_executor.rs:26-36) by (type, level) | SKIP, REJECTED for a
 *        later duplicate, INVALID for a vote that fails the checks; one deferred
 *        8-B non-temporal store per lane.
 *
 * Instances whose sums may reach 2^31 are deferred to the i64 LIST kernel (the
 * u32-domain test shared with agnes_fast.hip and agnes_apply.hip).  The State
 * machine runs in the apply pass over the codes (agnes_apply.hip).
 */
#include <type_traits>
#include <vector>
#include <cstdio>

#include "agnes_fast.h"

/* AGNES_DFLOW_CHECK (development builds only): every global access bounds-checked; a
 * violation is printed and the access skipped */
#ifndef AGNES_DFLOW_CHECK
#define AGNES_DFLOW_CHECK 0
#endif
#if AGNES_DFLOW_CHECK
#include <cstdio>
__device__ unsigned agnes_dflow_nbad;
__device__ __noinline__ bool agnes_dflow_bad(int tag, unsigned long long x, unsigned long long y) {
    if (atomicAdd(&agnes_dflow_nbad, 1u) < 48u)
        printf("dflow OOB tag %d x %llu lim %llu block %u thread %u\n", tag, x, y, blockIdx.x, threadIdx.x);
    return false;
}
#define DCHK(c, tag, x, y) ((c) || agnes_dflow_bad(tag, (unsigned long long)(x), (unsigned long long)(y)))
#else
#define DCHK(c, tag, x, y) true
#endif

namespace agnes {
namespace dflow {
using namespace agnes::fast;

constexpr uint32_t LV = 8u, CH = 64u * LV; /* votes per lane, per chunk */
/* DMA slot: each column of the chunk as a contiguous image (the flow kernel's layout) */
constexpr uint32_t F_INST = 0, F_VALUE = 2048, F_VAL = 4096, F_ROUND = 6144, F_TYPE = 6656, F_BYTES = 7168;
constexpr uint32_t FB = 32u;     /* instances per batch (header: one per lane)          */
constexpr uint32_t SMALLB = 4u;  /* batch size of the work queue's tail                 */
constexpr uint32_t NSEG = 4u;    /* instances (segments) per tally pass of a chunk      */
constexpr uint32_t NKEY = 16u;   /* sort keys: round (< 8) << 1 | type                  */
constexpr uint32_t NRUN = NSEG * NKEY;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t DEF = 0x80000000u; /* record nvv: the instance is the LIST kernel's */
/* per-instance record (batch lane k): quorum / RoundSkip thresholds, power row base,
 * validators of its set (| DEF), epoch (0: none yet), instance id */
constexpr uint32_t R_Q2 = 0, R_Q1 = 1, R_PBASE = 2, R_NV = 3, R_EP = 4, R_ID = 5;
/* (State machine) the instance's State as vote events see it, and what the batch
 * changed: step, State.round as a u8-comparable (0x100: no u8 round equals it), the
 * round clamped to [-1, 256] (vote round r > RLT <=> State.round < r), the P1 position
 * (| LOCKF: a PolkaValue, :198), the commit position and round (:211), the last
 * set_valid_value position + 1 (:202), whether a RoundSkip moved the round (:210).
 * Positions are stream-relative. */
constexpr uint32_t R_STEP = 6, R_EQ8 = 7, R_RLT = 8, R_P1 = 9, R_C = 10, R_DR = 11, R_VP = 12, R_SK = 13, RECW = 16;
constexpr uint32_t LOCKF = 0x80000000u;
/* per-segment record of the current chunk: id, power row base, nvv | DEF, q2 */
constexpr uint32_t S_ID = 0, S_PBASE = 1, S_NV = 2, S_Q2 = 3, SEGW = 4;

/* to_event by index type * 4 + level (Init, Any, Nil, Value): vote_executor.rs:26-36 */
constexpr uint32_t EV_LO = AGNES_CODE_NONE | (AGNES_CODE_POLKA_ANY << 8) | (AGNES_CODE_POLKA_NIL << 16) |
                           (AGNES_CODE_POLKA_VALUE << 24);
constexpr uint32_t EV_HI = AGNES_CODE_NONE | (AGNES_CODE_PRECOMMIT_ANY << 8) | (AGNES_CODE_NONE << 16) |
                           (AGNES_CODE_PRECOMMIT_VALUE << 24);

/* ALIAS: the sort buffers (6 KB) share the chunk's DMA slot, which the next chunk's
 * prefetch then fills only after the tally: 6 KB less LDS per wave (occupancy) against
 * a shorter prefetch distance */
#ifndef AGNES_DFLOW_ALIAS
#define AGNES_DFLOW_ALIAS 0
#endif
constexpr bool ALIAS = AGNES_DFLOW_ALIAS != 0;
/* AGNES_DFLOW_ABL (timing ablations only, results wrong): bit 0 no F pass, 1 no sort /
 * sorted pass, 2 no RS, 3 no K4, 4 no codes stage */
#ifndef AGNES_DFLOW_ABL
#define AGNES_DFLOW_ABL 0
#endif
constexpr uint32_t ABL = AGNES_DFLOW_ABL;

/* per-wave LDS layout */
struct Lay {
    uint32_t t, sb, lo, rt, re, cr, xs, kx, it, st, et, total;
};
__host__ __device__ inline Lay layout(uint32_t R, uint32_t nv, bool evc, bool sm) {
    Lay L;
    uint32_t o = F_BYTES;
    L.t = o;  o += (uint32_t)align16(8ull * R * nv);   /* first-vote table [R][2][nv] u32    */
    if (ALIAS) { /* the sort buffers in the DMA slot (the next chunk's DMA waits for them) */
        L.sb = 0;
        L.lo = 8u * CH;
    } else {
        L.sb = o; o += 8u * CH;                         /* sorted chunk {w, meta} u64         */
        L.lo = o; o += 64u * 32u;                       /* lane key offsets u16, then levels   */
    }
    L.rt = o; o += 16u * NRUN;                          /* run thresholds {tv, tn, ta, -}      */
    L.re = o; o += 16u * NRUN;                          /* run totals {v, n, s, -}             */
    L.cr = o; o += 2u * (8u * NKEY + 4u * 8u);          /* carried executors, 2 copies         */
    L.xs = o; o += 4u * NSEG * 8u;                      /* RoundSkip crossing per (seg, round) */
    L.kx = o; o += sm ? 2u * FB * 8u : 0u;              /* (State machine) crossings in the chunk */
    L.it = o; o += 4u * (sm ? RECW : R_STEP + 2u) * FB; /* instance records                    */
    L.st = o; o += 4u * SEGW * FB;                      /* segment records of the chunk        */
    L.et = o; o += evc ? 4u * FB : 0u;                  /* (EVC) record counts                 */
    L.total = (uint32_t)align16(o);
    return L;
}

__device__ __forceinline__ uint32_t rep4(uint32_t b) { return __builtin_amdgcn_perm(0u, b, 0u); }
__device__ __forceinline__ uint32_t zero_marks(uint32_t x) { /* 0x80 in the bytes of x that are zero */
    const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    return ((t | x) & 0x80808080u) ^ 0x80808080u;
}
__device__ __forceinline__ uint32_t mark_bytes(uint32_t m) { return (m << 1) - (m >> 7); } /* 0x80 -> 0xFF */
__device__ __forceinline__ uint32_t eq_bytes(uint32_t x, uint32_t b) { return mark_bytes(zero_marks(x ^ rep4(b))); }
/* byte i (0/1) = bit i of x, x < 16 */
__device__ __forceinline__ uint32_t spread4(uint32_t x) { return (x * 0x00204081u) & 0x01010101u; }
/* 0xFF bytes for the set bits of x < 16 */
__device__ __forceinline__ uint32_t bytes_of(uint32_t x) { const uint32_t b = spread4(x); return (b << 8) - b; }
/* 0xFF in the bytes b of x (all < 128) with lo <= b < hi (lo < 128, hi <= 128) */
__device__ __forceinline__ uint32_t range_bytes(uint32_t x, uint32_t lo, uint32_t hi) {
    const uint32_t ge = ((x | 0x80808080u) - rep4(lo)) & 0x80808080u;
    const uint32_t lt = ~((x | 0x80808080u) - rep4(hi)) & 0x80808080u;
    return mark_bytes(ge & lt);
}
/* bit i = byte i of x != 0, for 0x00 / 0xFF bytes */
__device__ __forceinline__ uint32_t bits_of(uint32_t x) { return (((x & 0x01010101u) * 0x01020408u) >> 24) & 0xFu; }
/* byte i = popcount(x & (2 << i) - 1), x < 16 */
__device__ __forceinline__ uint32_t pfx4(uint32_t x) { return spread4(x) * 0x01010101u; }
__device__ __forceinline__ uint32_t bsel(uint32_t w, uint32_t s) { return __builtin_amdgcn_ubfe(w, 8u * (s & 3u), 8u); }
__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
/* four nibbles (16 bits) into the four 16-bit fields of a u64 */
__device__ __forceinline__ uint64_t nib16(uint64_t x) {
    x &= 0xFFFFull;
    x = (x | (x << 24)) & 0x000000FF000000FFull;
    x = (x | (x << 12)) & 0x000F000F000F000Full;
    return x;
}

__device__ __forceinline__ void sdma16(const void* base, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(base), "s"(lds)
                 : "memory");
}
__device__ __forceinline__ void sdma4(const void* base, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(base), "s"(lds)
                 : "memory");
}
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
__device__ __forceinline__ void sstore8(void* base, uint32_t voff, uint32_t d0, uint32_t d1) {
    asm volatile("global_store_dwordx2 %0, %1, %2 nt" ::"v"(voff), "v"(u64of(d0, d1)), "s"(base) : "memory");
}

/* a batch: instances [s0, e0); header built in three stages one chunk apart (as the
 * flow kernel's): offsets + sets requested; lengths, offset checks, set constants;
 * thresholds, the LIST deferral, and whether the batch is one stream */
struct Hdr {
    uint32_t s0, e0;
    uint32_t olo, ohi; /* lanes 0..m: offset (clamped to n_votes)          */
    uint32_t hs;       /* lane k < m: power set                             */
    uint32_t q2, q1, mp, fa, ln;
    uint32_t def;      /* lane k: deferred to the LIST kernel              */
    uint32_t stage;
    uint32_t stream;
};

/* EVC: also each instance's event-record count (Some(Event) votes, a SKIP bit one more:
 * RoundSkip is emitted before the tally event) into a.ev_counts */
template <bool DEDUP, bool SKIP, bool PC, bool EVC, bool SM>
__global__ __launch_bounds__(256) void dflow(agnes_tally_args a, uint32_t lds_per_wave) {
    const uint32_t lane = lane_id();
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint32_t R = a.max_rounds, nv = a.n_vals, ns = a.n_sets, n = a.vb.n_instances;
    const uint64_t NV = a.vb.n_votes;
    const uint32_t o16 = 16u * lane, o8 = 8u * lane, o4 = 4u * lane;
    const Lay L = layout(R, nv, EVC, SM);
    constexpr uint32_t RW = SM ? RECW : R_STEP + 2u; /* record words */

    if (PC) {
        uint32_t* pc = reinterpret_cast<uint32_t*>(agnes_smem);
        const uint32_t np = ns * nv;
        for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) pc[k] = a.power32[k];
        __syncthreads();
    }
    unsigned char* const base = agnes_smem + a.power_cache + wave * lds_per_wave;
    unsigned char* const slot = base;
    const uint32_t slotl = lds_addr(slot);
    uint32_t* const T = reinterpret_cast<uint32_t*>(base + L.t);
    unsigned long long* const SB = reinterpret_cast<unsigned long long*>(base + L.sb);
    unsigned char* const LO = base + L.lo;
    uint4* const RT = reinterpret_cast<uint4*>(base + L.rt);
    uint4* const RE = reinterpret_cast<uint4*>(base + L.re);
    uint32_t* const CR = reinterpret_cast<uint32_t*>(base + L.cr); /* copy c: [c * 40]: v[16] n[16] s[8] */
    uint32_t* const XS = reinterpret_cast<uint32_t*>(base + L.xs);
    uint32_t* const IT = reinterpret_cast<uint32_t*>(base + L.it);
    uint32_t* const ST = reinterpret_cast<uint32_t*>(base + L.st);
    uint32_t* const ET = reinterpret_cast<uint32_t*>(base + L.et);
    uint16_t* const KX = reinterpret_cast<uint16_t*>(base + L.kx);
    const uint32_t tsize = 2u * R * nv;
    fill_u32(T, tsize, 0u, lane);
    const uint32_t lb = a.epoch_shift;
    const uint32_t lmask = lb >= 32u ? 0xFFFFFFFFu : (1u << lb) - 1u;
    const uint32_t emax = lb >= 31u ? 1u : ((1u << (32u - lb)) - 1u);
    uint32_t epc = 0; /* epochs handed out since the table was last cleared */
    uint32_t cpar = 0;
    uint64_t pf_at = ~0ull;
    uint32_t bad = 0;

    /* ---- work queue (the flow kernel's): batches of FB, SMALLB ones for the tail ---- */
    const uint32_t qn = gridDim.x < QN ? gridDim.x : QN;
    const uint32_t qk = blockIdx.x % qn;
    uint32_t* const ctr = a.list_count + 1u + qk;
    const uint64_t NB = (uint64_t)(n / FB) * 15u / 16u;
    auto range_of = [&](uint32_t t, uint32_t& s0, uint32_t& e0) {
        const uint64_t b = (uint64_t)t * qn + qk;
        const uint64_t s = b < NB ? b * FB : NB * FB + (b - NB) * SMALLB;
        const uint64_t e = s + (b < NB ? FB : SMALLB);
        s0 = s < n ? (uint32_t)s : n;
        e0 = e < n ? (uint32_t)e : n;
    };
    auto hdr1 = [&](Hdr& h) {
        const uint32_t m = h.e0 - h.s0;
        uint32_t lo = 0, hi = 0, hs = 0;
        if (m > 0u && lane <= m) {
            const uint64_t o = DCHK(h.s0 + lane <= n, 1, h.s0 + lane, n) ? a.vb.offsets[h.s0 + lane] : 0ull;
            const uint64_t oc = o < NV ? o : NV;
            lo = (uint32_t)oc;
            hi = (uint32_t)(oc >> 32);
        }
        if (lane < m) {
            const uint32_t k = h.s0 + lane;
            hs = a.vb.instance_set ? (DCHK(k < n, 2, k, n) ? a.vb.instance_set[k] : 0u) : (ns ? k % ns : 0u);
        }
        h.olo = lo;
        h.ohi = hi;
        h.hs = hs;
        h.stage = 1;
        h.stream = 0;
    };
    auto hdr2 = [&](Hdr& h) {
        const uint32_t m = h.e0 - h.s0;
        const bool il = lane < m;
        const uint64_t ob = u64of(h.olo, h.ohi);
        const uint64_t oe = u64of(shfl(h.olo, lane + 1u), shfl(h.ohi, lane + 1u));
        const uint64_t len = il && oe > ob ? oe - ob : 0ull;
        h.ln = len < (1ull << 31) ? (uint32_t)len : (1u << 31);
        uint32_t q2 = 0, q1 = 0, mp = 0, fa = 2;
        if (il && h.hs < ns && DCHK(h.hs < ns, 3, h.hs, ns)) {
            const agnes_set_info* const si = a.sets + h.hs;
            q2 = si->q2;
            q1 = si->q1;
            mp = si->maxpow;
            fa = si->fast;
        }
        h.q2 = q2;
        h.q1 = q1;
        h.mp = mp;
        h.fa = fa;
        /* one stream: offsets non-decreasing, the whole batch < 2^30 votes */
        const bool badl = lane < m && oe < ob;
        const uint64_t O0 = u64of(rdl(h.olo, 0u), rdl(h.ohi, 0u)), Om = u64of(rdl(h.olo, m), rdl(h.ohi, m));
        h.stream = m > 0u && !ballot(badl) && Om - O0 < (1ull << 30);
        h.stage = 2;
    };
    auto hdr3 = [&](Hdr& h) {
        const uint32_t m = h.e0 - h.s0;
        uint32_t def = 0;
        if (lane < m && h.fa != 2u && h.ln != 0u) def = defer_to_list(h.fa, h.mp, h.ln) ? 1u : 0u;
        h.def = def;
        h.q2 = h.q2 < 0x7FFFFFFFu ? h.q2 : 0x7FFFFFFFu;
        h.q1 = h.q1 < 0x7FFFFFFFu ? h.q1 : 0x7FFFFFFFu;
        h.stage = 3;
    };
    /* a batch that is not one stream: each instance alone (a one-instance header) */
    auto hdr_one = [&](const Hdr& h, uint32_t k, Hdr& o) {
        o.s0 = h.s0 + k;
        o.e0 = o.s0 + 1u;
        const uint32_t blo = rdl(h.olo, k), bhi = rdl(h.ohi, k);
        const uint64_t b = u64of(blo, bhi), e = b + rdl(h.ln, k);
        o.olo = lane == 0u ? blo : (uint32_t)e;
        o.ohi = lane == 0u ? bhi : (uint32_t)(e >> 32);
        o.hs = rdl(h.hs, k);
        o.q2 = rdl(h.q2, k);
        o.q1 = rdl(h.q1, k);
        o.mp = rdl(h.mp, k);
        o.fa = rdl(h.fa, k);
        o.ln = rdl(h.ln, k);
        o.def = rdl(h.def, k);
        o.stage = 3;
        o.stream = o.ln < (1u << 30);
    };
    auto dma_chunk = [&](uint64_t c, uint32_t lo, uint32_t lim) { /* votes lo..lim of the chunk at c */
        c = rfl64(c); /* uniform: the LDS-DMA takes scalar base addresses */
        lo = rfl(lo);
        lim = rfl(lim);
        __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): the slot's LDS reads are done */
        if (lo == 0u && lim >= CH && c + CH <= NV && DCHK(c + CH <= NV, 4, c + CH, NV)) {
            sdma_chunk(a.vb.instance + c, a.vb.value + c, a.vb.validator + c, a.vb.round + c, a.vb.type + c, o16, o4,
                       slotl);
        } else { /* a stream's first or last chunk: the 4-vote groups that hold active votes;
                  * a group running past the columns' end is read vote by vote */
            for (uint32_t hf = 0; hf < 2u; ++hf) {
                const uint32_t g = 256u * hf + 4u * lane;
                if (g + 4u > lo && g < lim) {
                    if (c + g + 4u <= NV && DCHK(c + g + 4u <= NV, 5, c + g + 4u, NV)) {
                        sdma16(a.vb.instance + c + 256u * hf, o16, slotl + F_INST + 1024u * hf);
                        sdma16(a.vb.value + c + 256u * hf, o16, slotl + F_VALUE + 1024u * hf);
                        sdma16(a.vb.validator + c + 256u * hf, o16, slotl + F_VAL + 1024u * hf);
                        sdma4(a.vb.round + c + 256u * hf, o4, slotl + F_ROUND + 256u * hf);
                        sdma4(a.vb.type + c + 256u * hf, o4, slotl + F_TYPE + 256u * hf);
                    } else {
                        uint32_t iv[4] = {0, 0, 0, 0}, vv[4] = {0, 0, 0, 0}, dv[4] = {0, 0, 0, 0}, rr = 0, tt = 0;
                        for (uint32_t q = 0; q < 4u; ++q) {
                            const uint64_t j = c + g + q;
                            if (j < NV) {
                                iv[q] = a.vb.instance[j];
                                vv[q] = a.vb.value[j];
                                dv[q] = a.vb.validator[j];
                                rr |= (uint32_t)a.vb.round[j] << (8u * q);
                                tt |= (uint32_t)a.vb.type[j] << (8u * q);
                            }
                        }
                        const uint32_t u = 256u * hf;
                        *reinterpret_cast<uint4*>(slot + F_INST + 4u * u + o16) = make_uint4(iv[0], iv[1], iv[2], iv[3]);
                        *reinterpret_cast<uint4*>(slot + F_VALUE + 4u * u + o16) = make_uint4(vv[0], vv[1], vv[2], vv[3]);
                        *reinterpret_cast<uint4*>(slot + F_VAL + 4u * u + o16) = make_uint4(dv[0], dv[1], dv[2], dv[3]);
                        *reinterpret_cast<uint32_t*>(slot + F_ROUND + u + o4) = rr;
                        *reinterpret_cast<uint32_t*>(slot + F_TYPE + u + o4) = tt;
                    }
                }
            }
        }
    };

    /* deferred code stores: the previous chunk's, issued behind the next DMA */
    uint64_t dc_at = ~0ull;
    uint32_t dc0 = 0, dc1 = 0, dc_act = 0; /* dc_act: byte mask (bit s: vote s) of the lane's votes to write */
    auto flush = [&]() {
        if (dc_at != ~0ull) {
            if (dc_act == 0xFFu && DCHK(dc_at + o8 + 8u <= NV, 6, dc_at + o8 + 8u, NV)) {
                sstore8(a.codes + rfl64(dc_at), o8, dc0, dc1);
            } else if (dc_act) {
                for (uint32_t s = 0; s < LV; ++s)
                    if (((dc_act >> s) & 1u) && DCHK(dc_at + o8 + s < NV, 7, dc_at + o8 + s, NV)) a.codes[dc_at + o8 + s] = (uint8_t)bsel(s < 4u ? dc0 : dc1, s);
            }
            dc_at = ~0ull;
        }
    };

    Hdr H, N;
    uint32_t tq = 0;
    {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(ctr, 2u);
        t = rdl(t, 0u);
        range_of(t, H.s0, H.e0);
        range_of(t + 1u, N.s0, N.e0);
        if (lane == 0) tq = atomicAdd(ctr, 1u);
    }
    if (H.s0 >= H.e0) return;
    hdr1(H);
    hdr2(H);
    hdr3(H);
    hdr1(N);

    /* One stream: the instances of header S ([S.s0, S.e0), offsets in lanes 0..m).
     * `last`: no other stream of this batch follows (the next batch's first chunk
     * may be prefetched). */
    auto run_stream = [&](const Hdr& S, bool last) {
        const uint32_t m = S.e0 - S.s0;
        const uint64_t S0 = u64of(rdl(S.olo, 0u), rdl(S.ohi, 0u));
        const uint64_t Sa = S0 & ~127ull;
        const uint32_t lead = (uint32_t)(S0 - Sa);
        const uint32_t s0lo = (uint32_t)S0;
        const uint32_t Lend = rdl(S.olo, m) - s0lo + lead;
        const uint32_t rl = S.olo - s0lo + lead; /* lane k <= m: instance k's start, stream-relative */
        const uint32_t rn = shfl(rl, lane + 1u);
        const uint64_t mm64 = m >= 64u ? ~0ull : (1ull << m) - 1ull;
        const uint64_t NE = ballot(lane < m && rn > rl) & mm64; /* instances with votes */
        const uint32_t relv = lane <= m ? rl : 0x7FFFFFFFu;
        /* the instance records */
        if (lane < m && DCHK(S.s0 + lane < n, 8, S.s0 + lane, n)) {
            uint32_t* const rk = IT + RW * lane;
            const bool set_ok = S.hs < ns;
            rk[R_Q2] = S.q2;
            rk[R_Q1] = S.q1;
            rk[R_PBASE] = set_ok ? S.hs * nv : 0u;
            rk[R_NV] = (set_ok ? nv : 0u) | (S.def ? DEF : 0u);
            rk[R_EP] = 0u;
            rk[R_ID] = S.s0 + lane;
            if (SM) { /* the State as vote events see it (state_machine.rs:184) */
                const uint32_t* const sp = reinterpret_cast<const uint32_t*>(a.states + S.s0 + lane);
                const int64_t rnd = (int64_t)u64of(sp[2], sp[3]);
                rk[R_STEP] = sp[13] & 0xFFu;
                rk[R_EQ8] = (rnd >= 0 && rnd <= 255) ? (uint32_t)rnd : 0x100u;
                rk[R_RLT] = (uint32_t)(rnd < -1 ? -1 : (rnd > 256 ? 256 : (int32_t)rnd));
                rk[R_P1] = NONE;
                rk[R_C] = NONE;
                rk[R_DR] = 0u;
                rk[R_VP] = 0u;
                rk[R_SK] = 0u;
            }
            if (S.def && rn > rl) {
                const uint32_t li = atomicAdd(a.list_count, 1u);
                if (DCHK(li < n, 9, li, n)) a.list[li] = S.s0 + lane;
                /* (agnes_tally_events) its records are counted after the LIST kernel's codes */
                if (EVC) a.walk[atomicAdd(a.list_count + AGNES_WALK_COUNT, 1u)] = S.s0 + lane;
            }
            if (EVC) ET[lane] = 0u;
        }
        __builtin_amdgcn_wave_barrier();
        if (Lend <= lead) {
            if (EVC && lane < m) a.ev_counts[S.s0 + lane] = 0ull;
            return;
        }

        for (uint32_t rc = 0; rc < Lend; rc += CH) {
            /* the lane's offsets recomputed per chunk from an opaque lane id: otherwise the
             * compiler hoists dozens of lane-derived constants out of the chunk loop and keeps
             * them in VGPRs across it */
            uint32_t lane = lane_id();
            asm volatile("" : "+v"(lane));
            const uint32_t o32 = 32u * lane, o16 = 16u * lane, o8 = 8u * lane, o4 = 4u * lane;
            (void)o16;
            (void)o4;
            const uint64_t c = Sa + rc;
            const uint32_t lo_r = rc == 0u ? lead : 0u;
            const uint32_t left = Lend - rc;
            const uint32_t hi_r = left < CH ? left : CH;
            if (pf_at != c) dma_chunk(c, lo_r, hi_r);
            dma_wait();
            __builtin_amdgcn_s_setprio(1);
            /* the next batch's header, one stage per chunk */
            if (last && N.s0 < N.e0) {
                if (N.stage == 1u) hdr2(N);
                else if (N.stage == 2u) hdr3(N);
            }

            /* ---- segments: the instances the chunk holds ---- */
            const uint32_t tj = relv - rc; /* lane k: instance k's start, chunk-relative */
            const uint32_t k0 = 63u - (uint32_t)__builtin_clzll((ballot((int32_t)tj <= (int32_t)lo_r) & mm64) | 1ull);
            uint64_t bk = ballot(lane < m && tj - lo_r - 1u < hi_r - lo_r - 1u) & NE; /* starting inside */
            const bool cont0 = (int32_t)rdl(tj, k0) < (int32_t)lo_r; /* k0 began in an earlier chunk */
            const uint32_t nseg = 1u + (uint32_t)__builtin_popcountll(bk);
            /* segment i -> instance (lane i of segk); per lane: segment of vote 0 and the
             * in-lane starts (bit o: a start at vote o, o >= 1) */
            uint32_t segk = lane == 0u ? k0 : 0u, segA = 0, sm = 0;
            {
                uint32_t i = 1;
                while (bk) {
                    const uint32_t k = (uint32_t)__builtin_ctzll(bk);
                    bk &= bk - 1ull;
                    const uint32_t u = rdl(tj, k);
                    segk = lane == i ? k : segk;
                    segA += u <= o8 ? 1u : 0u;
                    sm |= (u > o8 && u < o8 + 8u) ? 1u << (u - o8) : 0u;
                    ++i;
                }
            }
            /* segment of each vote, a byte per vote */
            const uint32_t sg0c = rep4(segA) + pfx4(sm & 0xFu);
            const uint32_t sg1c = rep4(segA + (uint32_t)__builtin_popcount(sm & 0xFu)) + pfx4(sm >> 4);
            const uint32_t sg0 = sg0c, sg1 = sg1c;
            /* the chunk's segment records */
            if (lane < nseg) {
                const uint32_t* const rk = IT + RW * segk;
                uint32_t* const sr = ST + SEGW * lane;
                const uint4 r0 = *reinterpret_cast<const uint4*>(rk);
                const uint2 r1 = *reinterpret_cast<const uint2*>(rk + 4);
                sr[S_ID] = r1.y;
                sr[S_PBASE] = r0.z;
                sr[S_NV] = r0.w;
                sr[S_Q2] = r0.x;
            }
            __builtin_amdgcn_wave_barrier();
            /* the lane's active votes (bit s: vote s in [lo_r, hi_r)) */
            const uint32_t actb = (o8 + 8u <= lo_r || o8 >= hi_r)
                                      ? 0u
                                      : ((hi_r - o8 >= 8u ? 0xFFu : (1u << (hi_r - o8)) - 1u) &
                                         ~(lo_r > o8 ? (1u << (lo_r - o8)) - 1u : 0u));

            /* ---- K1: columns, checks, weights ---- */
            uint32_t w[LV], kd[LV], r8[2], t8[2];
            uint32_t okb = 0, defb = 0, nilbc = 0; /* bit s: vote s passes the checks / is a deferred instance's / nil */
            {
                uint32_t inst[LV], value[LV], val[LV];
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
                /* a lane's votes lie in its segment segA and (one start inside) the next; two or
                 * more starts inside a lane (instances under 8 votes) take the per-vote records */
                const uint4 recA = *reinterpret_cast<const uint4*>(ST + SEGW * segA); /* id, pbase, nvv, q2 */
                const uint4 recB = *reinterpret_cast<const uint4*>(ST + SEGW * (segA + 1u < nseg ? segA + 1u : segA));
                const bool many = ballot(__builtin_popcount(sm) >= 2) != 0ull;
#pragma unroll
                for (uint32_t s = 0; s < LV; ++s) {
                    const uint32_t sg = bsel(s < 4u ? sg0 : sg1, s);
                    uint4 sr = sg == segA ? recA : recB;
                    if (many && sg > segA + 1u) sr = *reinterpret_cast<const uint4*>(ST + SEGW * (sg < nseg ? sg : 0u));
                    const uint32_t r = bsel(s < 4u ? r8[0] : r8[1], s), t = bsel(s < 4u ? t8[0] : t8[1], s);
                    const bool act = ((actb >> s) & 1u) != 0u;
                    const bool dfr = (sr.z & DEF) != 0u;
                    const bool ok = act && !dfr && inst[s] == sr.x && r < R && t <= 1u && val[s] < (sr.z & ~DEF);
                    okb |= ok ? 1u << s : 0u;
                    defb |= (act && dfr) ? 1u << s : 0u;
                    const uint32_t idx = ok ? sr.y + val[s] : 0u;
                    const uint32_t x = PC ? reinterpret_cast<const uint32_t*>(agnes_smem)[idx]
                                          : (DCHK(idx < ns * nv, 10, idx, ns * nv) ? a.power32[idx] : 0u);
                    w[s] = ok ? x : 0u;
                    nilbc |= value[s] == AGNES_NIL ? 1u << s : 0u;
                    /* first-vote table index (checked-out votes: entry 0, a no-op max) */
                    kd[s] = ok ? ((r << 1) | t) * nv + val[s] : 0u;
                }
                bad += (uint32_t)__builtin_popcount(actb & ~okb & ~defb);
            }
            if (!PC) asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]),
                                  "v"(w[6]), "v"(w[7]));
            /* the next chunk by LDS-DMA (this stream's, or the next batch's first) */
            auto issue_next = [&]() {
                uint64_t nc = ~0ull;
                uint32_t nl = 0, nlo = 0;
                if (rc + CH < Lend) {
                    nc = c + CH;
                    nl = Lend - rc - CH;
                } else if (last && N.s0 < N.e0 && N.stage == 3u && N.stream) {
                    const uint32_t mN = N.e0 - N.s0;
                    const uint64_t n0 = u64of(rdl(N.olo, 0u), rdl(N.ohi, 0u));
                    nc = n0 & ~127ull;
                    nlo = (uint32_t)(n0 - nc);
                    nl = rdl(N.olo, mN) - (uint32_t)n0 + nlo;
                }
                if (nc != ~0ull && nl > nlo) {
                    dma_chunk(nc, nlo, nl < CH ? nl : CH);
                    pf_at = nc;
                } else {
                    pf_at = ~0ull;
                }
            };
            if (!ALIAS) issue_next();
            flush();
            __builtin_amdgcn_s_setprio(0);

            /* per-vote key bytes (round << 1 | type) and nil bytes */
            const uint32_t kb0c = ((r8[0] & 0x07070707u) << 1) | (t8[0] & 0x01010101u);
            const uint32_t kb1c = ((r8[1] & 0x07070707u) << 1) | (t8[1] & 0x01010101u);

            /* the last segment runs into the next chunk (when the next instance starts right
             * at the chunk end, the carry written is simply not read) */
            const bool lastc = rc + CH < Lend;
            uint32_t* const CA = CR + cpar * 40u;        /* carried into this chunk    */
            uint32_t* const CB = CR + (cpar ^ 1u) * 40u; /* carried out of this chunk */
            uint32_t c0 = 0, c1 = 0; /* codes of the lane's votes */

            /* ---- per group of up to NSEG segments ---- */
            /* F: first-vote flags, one pass per segment */
            uint32_t accb = 0, sfbc = 0; /* bits per vote: accepted, first of (round, validator) */
            if ((DEDUP || SKIP) && !(ABL & 1u)) {
                for (uint32_t i = 0; i < nseg; ++i) {
                    const uint32_t k = rdl(segk, i);
                    const uint32_t mok = (bits_of(eq_bytes(sg0, i)) | (bits_of(eq_bytes(sg1, i)) << 4)) & okb;
                    if (!ballot(mok != 0u)) continue;
                    uint32_t ep = rfl(IT[RW * k + R_EP]);
                    if (ep == 0u) { /* the instance's first pass: its epoch */
                        if (epc == emax) {
                            __builtin_amdgcn_wave_barrier();
                            fill_u32(T, tsize, 0u, lane);
                            epc = 0;
                        }
                        ep = ++epc;
                        if (lane == 0) IT[RW * k + R_EP] = ep;
                    }
                    /* enc of vote s = (ep << lb | LMASK) - (its index in the instance) */
                    const uint32_t G = ((ep << lb) | lmask) + rdl(tj, k) - o8;
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) atomicMax(T + kd[s], ((mok >> s) & 1u) ? G - s : 0u);
                    __builtin_amdgcn_wave_barrier();
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        if ((mok >> s) & 1u) {
                            const uint32_t e = G - s;
                            const uint32_t own = *(volatile uint32_t*)(T + kd[s]);
                            const bool first = own == e;
                            if (DEDUP) accb |= first ? 1u << s : 0u;
                            if (SKIP) {
                                const uint32_t t = bsel(s < 4u ? t8[0] : t8[1], s);
                                const uint32_t oth = *(volatile uint32_t*)(T + (t ? kd[s] - nv : kd[s] + nv));
                                sfbc |= (first && oth < e) ? 1u << s : 0u;
                            }
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
            if (!DEDUP) accb = okb;
            const uint32_t accall = accb;

            for (uint32_t g0 = 0; g0 < nseg; g0 += NSEG) {
                const uint32_t gn = nseg - g0 < NSEG ? nseg - g0 : NSEG;
                /* (opaque per pass: keeps the compiler from hoisting per-vote values derived
                 * from them out of this loop and holding them in registers across it) */
                uint32_t sg0 = sg0c, sg1 = sg1c, kb0 = kb0c, kb1 = kb1c, nilb = nilbc, sfb = sfbc, lane = lane_id();
                asm volatile("" : "+v"(sg0), "+v"(sg1), "+v"(kb0), "+v"(kb1), "+v"(nilb), "+v"(sfb), "+v"(lane));
                const uint32_t o8 = 8u * lane;
                /* the group's votes: segments g0 .. g0 + gn - 1 (segment bytes minus g0 < gn) */
                const uint32_t inb = bits_of(range_bytes(sg0, g0, g0 + gn)) | (bits_of(range_bytes(sg1, g0, g0 + gn)) << 4);
                accb = accall & inb;

                if (!(ABL & 2u)) {
                /* S: counting sort of the group's accepted votes by key */
                uint64_t Cn = 0;
                uint32_t rk0 = 0, rk1 = 0; /* rank of each vote among the lane's votes of its key, bytes */
#pragma unroll
                for (uint32_t s = 0; s < LV; ++s) {
                    const uint32_t sh = bsel(s < 4u ? kb0 : kb1, s) << 2;
                    const uint32_t rnk = (uint32_t)(Cn >> sh) & 0xFu;
                    if (s < 4u) rk0 |= rnk << (8u * s);
                    else rk1 |= rnk << (8u * (s - 4u));
                    Cn += (uint64_t)((accb >> s) & 1u) << sh;
                }
                /* per word j (keys 4j .. 4j+3, 16-bit fields): the lane's exclusive counts plus
                 * the keys' bases (exclusive prefix of the key totals) -> LO[lane][key] */
                uint32_t nacc;
                {
                    uint64_t run = 0;
#pragma unroll
                    for (uint32_t j = 0; j < 4u; ++j) {
                        const uint64_t E = nib16(Cn >> (16u * j));
                        const uint64_t I = scan(E);
                        const uint64_t tot = rdl(I, 63u);                 /* the 4 keys' totals      */
                        const uint64_t incl = tot * 0x0001000100010001ull; /* prefix inside the word */
                        const uint64_t O = I - E + (incl - tot) + run * 0x0001000100010001ull;
                        *reinterpret_cast<uint2*>(LO + 32u * lane + 8u * j) = make_uint2((uint32_t)O, (uint32_t)(O >> 32));
                        run += incl >> 48;
                    }
                    nacc = (uint32_t)run;
                }
                /* the run table: per (segment of the group, key) the thresholds on the run's
                 * own sums (the carried executor's sums folded in); run totals zeroed */
                {
                    const uint32_t sr = lane >> 4, key = lane & 15u;
                    uint32_t q2 = 0x7FFFFFFFu, cv = 0, cn = 0;
                    if (sr < gn) {
                        q2 = ST[SEGW * (g0 + sr) + S_Q2];
                        if (g0 + sr == 0u && cont0) {
                            cv = CA[key];
                            cn = CA[16u + key];
                        }
                    }
                    RT[lane] = make_uint4(q2 - cv, q2 - cn, q2 - cv - cn, 0u);
                    RE[lane] = make_uint4(0u, 0u, 0u, 0u);
                }
                __builtin_amdgcn_wave_barrier();
                /* scatter: {weight, position | nil << 9 | first << 10 | (key | segment << 4) << 16} */
#pragma unroll
                for (uint32_t s = 0; s < LV; ++s) {
                    if ((accb >> s) & 1u) {
                        const uint32_t key = bsel(s < 4u ? kb0 : kb1, s);
                        const uint32_t sg = bsel(s < 4u ? sg0 : sg1, s) - g0;
                        const uint32_t off = *reinterpret_cast<const uint16_t*>(LO + 32u * lane + 2u * key);
                        const uint32_t slotn = off + bsel(s < 4u ? rk0 : rk1, s);
                        const uint32_t hi = (o8 + s) | (((nilb >> s) & 1u) << 9) | (((sfb >> s) & 1u) << 10) |
                                            ((key | (sg << 4)) << 16);
                        SB[slotn] = u64of(w[s], hi);
                    }
                }
                __builtin_amdgcn_wave_barrier();

                /* K2/K3 over the sorted chunk: runs of equal (segment, key) */
                {
                    uint32_t ew[LV], eh[LV];
                    {
                        const uint4* const sp = reinterpret_cast<const uint4*>(SB + o8);
                        const uint4 x0 = sp[0], x1 = sp[1], x2 = sp[2], x3 = sp[3];
                        ew[0] = x0.x; eh[0] = x0.y; ew[1] = x0.z; eh[1] = x0.w;
                        ew[2] = x1.x; eh[2] = x1.y; ew[3] = x1.z; eh[3] = x1.w;
                        ew[4] = x2.x; eh[4] = x2.y; ew[5] = x2.z; eh[5] = x2.w;
                        ew[6] = x3.x; eh[6] = x3.y; ew[7] = x3.z; eh[7] = x3.w;
                    }
                    /* run id of slot s: (key | segment << 4), 0x100 past the accepted votes */
                    auto rid = [&](uint32_t s) -> uint32_t { return o8 + s < nacc ? (eh[s] >> 16) & 0x3Fu : 0x100u; };
                    const uint32_t rp = shfl(rid(LV - 1u), lane - 1u);
                    const uint32_t rprev = lane == 0u ? 0x200u : rp;
                    uint32_t stb = 0; /* bit s: a run starts at slot s */
                    /* pass 1: the lane's last-run totals */
                    uint64_t P = 0;
                    uint32_t Sx = 0;
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        const bool st = rid(s) != (s ? rid(s - 1u) : rprev);
                        stb |= st ? 1u << s : 0u;
                        P = (st ? 0ull : P) + ((uint64_t)ew[s] << ((eh[s] >> 4) & 32u));
                        if (SKIP) Sx = (st ? 0u : Sx) + ((eh[s] & 0x400u) ? ew[s] : 0u);
                    }
                    const uint32_t Tv = (uint32_t)P, Tn = (uint32_t)(P >> 32), Ts = Sx;
                    const uint32_t Iv = scan(Tv), In = scan(Tn), Is = SKIP ? scan(Ts) : 0u;
                    const uint32_t Ev = Iv - Tv, En = In - Tn, Es = Is - Ts;
                    /* the run holding the lane's first slots started in lane h (its last start):
                     * their sums before the lane are the scan from there */
                    const uint64_t hs = ballot(stb != 0u) & ((1ull << lane) - 1ull);
                    const uint32_t h = hs ? 63u - (uint32_t)__builtin_clzll(hs) : 0u;
                    const uint32_t Bv = Ev - shfl(Ev, h), Bn = En - shfl(En, h), Bs = SKIP ? Es - shfl(Es, h) : 0u;
                    const uint32_t nst0 = shfl(stb & 1u, lane + 1u); /* the next lane starts a run */
                    /* pass 2: every slot's sums from its run's start, the level, the run ends */
                    uint32_t sv = Bv, sn = Bn, ss = Bs;
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        const bool st = (stb >> s) & 1u;
                        const uint32_t x = ew[s], nl = eh[s] & 0x200u;
                        sv = (st ? 0u : sv) + (nl ? 0u : x);
                        sn = (st ? 0u : sn) + (nl ? x : 0u);
                        if (SKIP) ss = (st ? 0u : ss) + ((eh[s] & 0x400u) ? x : 0u);
                        if (o8 + s < nacc) {
                            const uint32_t r = rid(s);
                            const uint4 t = RT[r];
                            uint32_t l = (int32_t)(sv + sn) > (int32_t)t.z ? 1u : 0u;
                            l = (int32_t)sn > (int32_t)t.y ? 2u : l;
                            l = (int32_t)sv > (int32_t)t.x ? 3u : l;
                            LO[eh[s] & 0x1FFu] = (unsigned char)l;
                            const bool end = s < LV - 1u ? ((stb >> (s + 1u)) & 1u) != 0u
                                                         : (nst0 != 0u || o8 + LV >= nacc);
                            if (end || o8 + s + 1u == nacc) RE[r] = make_uint4(sv, sn, ss, 0u);
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();

                }
                /* RS: the RoundSkip crossing of every (segment, round) of the group */
                if (SKIP && !(ABL & 4u)) {
                    const uint32_t sr = lane >> 3, r = lane & 7u;
                    uint32_t xpos = NONE;
                    bool cross = false;
                    uint32_t cs = 0, q1 = 0;
                    const uint32_t ksr = shfl(segk, g0 + (sr < NSEG ? sr : 0u)); /* (all lanes active) */
                    if (lane < 8u * NSEG && sr < gn && r < R) {
                        const uint32_t tot = RE[16u * sr + 2u * r].z + RE[16u * sr + 2u * r + 1u].z;
                        cs = (g0 + sr == 0u && cont0) ? CA[32u + r] : 0u;
                        q1 = IT[RW * ksr + R_Q1];
                        if (cs > q1) xpos = 0u;                /* crossed in an earlier chunk */
                        else if (cs + tot > q1) cross = true;  /* in this one */
                    }
                    uint64_t cm = ballot(cross);
                    while (cm) { /* the exact crossing vote, in stream order */
                        const uint32_t j = (uint32_t)__builtin_ctzll(cm);
                        cm &= cm - 1ull;
                        const uint32_t gsr = g0 + (j >> 3), gr = j & 7u;
                        const uint32_t cj = rdl(cs, j), qj = rdl(q1, j);
                        const uint32_t ms0 = eq_bytes(sg0, gsr) & eq_bytes(kb0 >> 1 & 0x07070707u, gr);
                        const uint32_t ms1 = eq_bytes(sg1, gsr) & eq_bytes(kb1 >> 1 & 0x07070707u, gr);
                        const uint32_t mm = accb & sfb;
                        uint32_t pre[LV], acc = 0;
#pragma unroll
                        for (uint32_t s = 0; s < LV; ++s) {
                            const bool in = ((mm >> s) & 1u) && bsel(s < 4u ? ms0 : ms1, s) != 0u;
                            acc += in ? w[s] : 0u;
                            pre[s] = acc;
                        }
                        const uint32_t ex = scan(acc) - acc + cj;
                        uint32_t f = 8u;
#pragma unroll
                        for (int s = LV - 1; s >= 0; --s)
                            if (ex + pre[s] > qj) f = (uint32_t)s;
                        const uint64_t lm = ballot(f < 8u);
                        const uint32_t L0 = lm ? (uint32_t)__builtin_ctzll(lm) : 0u;
                        const uint32_t xp = lm ? 8u * L0 + rdl(f, L0) : NONE;
                        xpos = lane == j ? xp : xpos;
                    }
                    if (lane < 8u * NSEG) XS[lane] = xpos;
                    /* (State machine) the crossings inside this chunk: the RoundSkip candidates */
                    if (SM && lane < 8u * gn) KX[8u * g0 + lane] = (uint16_t)(cross && xpos != NONE ? xpos : 0xFFFFu);
                    /* the last segment's round sums into the next chunk */
                    if (lastc && nseg - 1u >= g0 && nseg - 1u < g0 + gn && lane < 8u) {
                        const uint32_t srl = nseg - 1u - g0;
                        const uint32_t base_s = (nseg == 1u && cont0) ? CA[32u + lane] : 0u;
                        CB[32u + lane] = base_s + RE[16u * srl + 2u * lane].z + RE[16u * srl + 2u * lane + 1u].z;
                    }
                }
                /* the last segment's executors into the next chunk */
                if (lastc && nseg - 1u >= g0 && nseg - 1u < g0 + gn && lane < NKEY) {
                    const uint32_t srl = nseg - 1u - g0;
                    const bool same = nseg == 1u && cont0;
                    const uint4 e = RE[16u * srl + lane];
                    CB[lane] = (same ? CA[lane] : 0u) + e.x;
                    CB[16u + lane] = (same ? CA[16u + lane] : 0u) + e.y;
                }
                __builtin_amdgcn_wave_barrier();

                /* codes of the group's votes: to_event by (type, level), SKIP, REJECTED */
                if (!(ABL & 16u)) {
                    const uint2 lv = *reinterpret_cast<const uint2*>(LO + o8);
                    const uint32_t ev0 = __builtin_amdgcn_perm(EV_HI, EV_LO,
                                                               (lv.x & 0x03030303u) | ((t8[0] & 0x01010101u) << 2));
                    const uint32_t ev1 = __builtin_amdgcn_perm(EV_HI, EV_LO,
                                                               (lv.y & 0x03030303u) | ((t8[1] & 0x01010101u) << 2));
                    const uint32_t am0 = bytes_of(accb & 0xFu), am1 = bytes_of(accb >> 4);
                    uint32_t x0 = ev0 & am0, x1 = ev1 & am1;
                    if (SKIP) {
#pragma unroll
                        for (uint32_t s = 0; s < LV; ++s) {
                            if ((accb >> s) & 1u) {
                                const uint32_t sr = bsel(s < 4u ? sg0 : sg1, s) - g0;
                                const uint32_t r = bsel(s < 4u ? kb0 : kb1, s) >> 1;
                                const uint32_t xp = XS[8u * sr + r];
                                if (o8 + s >= xp) {
                                    if (s < 4u) x0 |= AGNES_CODE_SKIP << (8u * s);
                                    else x1 |= AGNES_CODE_SKIP << (8u * (s - 4u));
                                }
                            }
                        }
                    }
                    const uint32_t rej = inb & okb & ~accb;
                    x0 |= bytes_of(rej & 0xFu) & (AGNES_CODE_REJECTED * 0x01010101u);
                    x1 |= bytes_of(rej >> 4) & (AGNES_CODE_REJECTED * 0x01010101u);
                    c0 |= x0;
                    c1 |= x1;
                    if (EVC) { /* records per segment: Some(Event) votes, + 1 with the SKIP bit */
                        auto recs = [](uint32_t cw, uint32_t m4) -> uint32_t {
                            const uint32_t e = cw & 0x07070707u;
                            const uint32_t nz = (e + 0x7F7F7F7Fu) & 0x80808080u;
                            return (uint32_t)__builtin_popcount(nz & m4) + (uint32_t)__builtin_popcount(cw & 0x08080808u & m4);
                        };
                        for (uint32_t i = g0; i < g0 + gn; ++i) {
                            const uint32_t m0b = eq_bytes(sg0, i) & am0, m1b = eq_bytes(sg1, i) & am1;
                            const uint32_t nrec = recs(x0, m0b) + recs(x1, m1b);
                            const uint32_t tot = rdl(scan(nrec), 63u);
                            if (lane == 0 && tot) ET[rdl(segk, i)] += tot;
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
            if (lastc) cpar ^= 1u;
            /* (ALIAS: the sort buffers live in the DMA slot, free again only now) */
            if (ALIAS) {
                __builtin_amdgcn_s_setprio(1);
                issue_next();
                __builtin_amdgcn_s_setprio(0);
            }

            /* ---- K4: State::apply(v.round, event) in stream order, per instance of the chunk
             * (consensus_executor.rs:64-68 -> state_machine.rs:196-211).  Vote events move the
             * State only at a few votes: P1 (the first PolkaNil / PolkaValue at State.round in
             * Prevote, :197-198), C (the first PrecommitValue, any round, :211) and RoundSkips
             * to a higher round (:210; the first SKIP vote of a round is its crossing).  Those
             * breakpoints are resolved in order on the scalar path; every other vote's message
             * follows from the State between them: TimeoutPrevote (PolkaAny at State.round in
             * Prevote, :196), TimeoutPrecommit (PrecommitAny at State.round, :208) ---- */
            if (SM && !(ABL & 8u)) {
                uint32_t lane = lane_id();
                asm volatile("" : "+v"(lane));
                const uint32_t o8 = 8u * lane;
                const uint32_t e0 = c0 & 0x07070707u, e1 = c1 & 0x07070707u;
                const uint32_t nn0 = ~bytes_of(nilbc & 0xFu), nn1 = ~bytes_of(nilbc >> 4); /* non-nil votes */
                /* the first / last chunk position whose byte is set in (m0, m1), NONE if none */
                auto first_pos = [&](uint32_t m0, uint32_t m1) -> uint32_t {
                    const uint32_t f = m0 ? ((uint32_t)__builtin_ctz(m0) >> 3) : (m1 ? 4u + ((uint32_t)__builtin_ctz(m1) >> 3) : 8u);
                    const uint64_t b = ballot(f < 8u);
                    if (!b) return NONE;
                    const uint32_t L0 = (uint32_t)__builtin_ctzll(b);
                    return 8u * L0 + rdl(f, L0);
                };
                auto last_pos = [&](uint32_t m0, uint32_t m1) -> uint32_t {
                    const uint32_t f = m1 ? 4u + ((31u - (uint32_t)__builtin_clz(m1)) >> 3)
                                          : (m0 ? (31u - (uint32_t)__builtin_clz(m0)) >> 3 : 8u);
                    const uint64_t b = ballot(f < 8u);
                    if (!b) return NONE;
                    const uint32_t L0 = 63u - (uint32_t)__builtin_clzll(b);
                    return 8u * L0 + rdl(f, L0);
                };
                /* the event / round byte at chunk position p (uniform) */
                auto ev_at = [&](uint32_t p) -> uint32_t {
                    const uint32_t lo = rdl(c0, p >> 3), hi = rdl(c1, p >> 3);
                    return bsel((p & 7u) < 4u ? lo : hi, p & 3u) & 7u;
                };
                auto round_at = [&](uint32_t p) -> uint32_t {
                    const uint32_t lo = rdl(r8[0], p >> 3), hi = rdl(r8[1], p >> 3);
                    return bsel((p & 7u) < 4u ? lo : hi, p & 3u);
                };
                for (uint32_t i = 0; i < nseg; ++i) {
                    const uint32_t k = rdl(segk, i);
                    uint32_t* const rk = IT + RW * k;
                    uint32_t step = rfl(rk[R_STEP]);
                    if (step == AGNES_STEP_COMMIT) continue; /* :205 every later event: None */
                    const uint32_t mb = accall & (bits_of(eq_bytes(sg0c, i)) | (bits_of(eq_bytes(sg1c, i)) << 4));
                    if (!ballot(mb != 0u)) continue;
                    const uint32_t mb0 = bytes_of(mb & 0xFu), mb1 = bytes_of(mb >> 4);
                    uint32_t eq8 = rfl(rk[R_EQ8]);
                    int32_t rlt = (int32_t)rfl(rk[R_RLT]);
                    const uint32_t step0 = step, eq80 = eq8;
                    /* candidates: C, P1 (from the chunk's starting State), the RoundSkip crossings */
                    const uint32_t cpos = first_pos(eq_bytes(e0, 5u) & mb0, eq_bytes(e1, 5u) & mb1);
                    uint32_t ppos = NONE;
                    if (step == AGNES_STEP_PREVOTE && eq8 < 0x100u) {
                        const uint32_t q0 = eq_bytes(r8[0], eq8) & mb0, q1 = eq_bytes(r8[1], eq8) & mb1;
                        ppos = first_pos((eq_bytes(e0, 2u) | eq_bytes(e0, 3u)) & q0, (eq_bytes(e1, 2u) | eq_bytes(e1, 3u)) & q1);
                    }
                    uint32_t kxv = 0xFFFFu; /* lane r: round r's crossing in this chunk */
                    if (SKIP && lane < R) kxv = KX[8u * i + lane];
                    if (ABL && kxv >= CH) kxv = 0xFFFFu; /* (ablations: stale crossings) */
                    /* breakpoints in order: lane j of bpp / bps = position / State after it */
                    uint32_t nbp = 0, bpp = NONE, bps = 0;
                    uint32_t p1_at = NONE, c_at = NONE, dr = 0, sk = 0;
                    /* breakpoint messages: lane j of mat / mv (at most P1, a RoundSkip per round, C) */
                    uint32_t mat = NONE, mv = 0, nmsg = 0;
                    for (;;) {
                        uint32_t kpos = NONE, kr = 0;
                        if (SKIP) {
                            uint64_t kb = ballot(lane < R && (int32_t)lane > rlt && kxv != 0xFFFFu);
                            while (kb) {
                                const uint32_t r = (uint32_t)__builtin_ctzll(kb);
                                kb &= kb - 1ull;
                                const uint32_t x = rdl(kxv, r);
                                if (x < kpos) { kpos = x; kr = r; }
                            }
                        }
                        const uint32_t pc = step == AGNES_STEP_PREVOTE ? ppos : NONE;
                        const uint32_t nx = min(kpos, min(pc, cpos));
                        if (nx == NONE) break;
                        uint32_t m;
                        if (kpos == nx) { /* :210 round_skip, then the vote's tally event at the new State */
                            eq8 = kr;
                            rlt = (int32_t)kr;
                            step = AGNES_STEP_NEW_ROUND;
                            sk = 1u;
                            const uint32_t e = ev_at(kpos);
                            if (cpos == kpos) {
                                m = AGNES_VMSG_NEW_ROUND_DECISION;
                                step = AGNES_STEP_COMMIT;
                                c_at = kpos;
                                dr = kr;
                            } else {
                                m = e == AGNES_CODE_PRECOMMIT_ANY ? AGNES_VMSG_NEW_ROUND_TIMEOUT_PRECOMMIT : AGNES_VMSG_NEW_ROUND;
                            }
                        } else if (pc == nx) { /* P1: :197 precommit nil / :198 lock, precommit */
                            const bool pv = ev_at(ppos) == AGNES_CODE_POLKA_VALUE;
                            m = pv ? AGNES_VMSG_PRECOMMIT_VALUE : AGNES_VMSG_PRECOMMIT_NIL;
                            step = AGNES_STEP_PRECOMMIT;
                            p1_at = ppos | (pv ? LOCKF : 0u);
                        } else { /* C: :211 commit */
                            m = AGNES_VMSG_DECISION;
                            step = AGNES_STEP_COMMIT;
                            c_at = cpos;
                            dr = round_at(cpos);
                        }
                        bpp = lane == nbp ? nx : bpp;
                        bps = lane == nbp ? (eq8 | (step << 16)) : bps;
                        ++nbp;
                        mat = lane == nmsg ? nx : mat;
                        mv = lane == nmsg ? m : mv;
                        ++nmsg;
                        if (step == AGNES_STEP_COMMIT) break;
                    }
                    /* every vote's message from the State before it; the last set_valid_value */
                    uint32_t x0 = 0, x1 = 0, vpos = NONE;
                    if (nbp == 0u) { /* one State over the whole chunk: bytewise */
                        if (eq8 < 0x100u) {
                            const uint32_t q0 = eq_bytes(r8[0], eq8) & mb0, q1 = eq_bytes(r8[1], eq8) & mb1;
                            if (step == AGNES_STEP_PREVOTE) {
                                x0 |= eq_bytes(e0, 1u) & q0 & (AGNES_VMSG_TIMEOUT_PREVOTE * 0x10101010u);
                                x1 |= eq_bytes(e1, 1u) & q1 & (AGNES_VMSG_TIMEOUT_PREVOTE * 0x10101010u);
                            }
                            x0 |= eq_bytes(e0, 4u) & q0 & (AGNES_VMSG_TIMEOUT_PRECOMMIT * 0x10101010u);
                            x1 |= eq_bytes(e1, 4u) & q1 & (AGNES_VMSG_TIMEOUT_PRECOMMIT * 0x10101010u);
                            if (step == AGNES_STEP_PRECOMMIT)
                                vpos = last_pos(eq_bytes(e0, 3u) & q0 & nn0, eq_bytes(e1, 3u) & q1 & nn1);
                        }
                    } else {
                        uint32_t vl = 8u; /* the lane's last set_valid_value vote */
#pragma unroll
                        for (uint32_t s = 0; s < LV; ++s) {
                            if ((mb >> s) & 1u) {
                                uint32_t st = eq80 | (step0 << 16);
                                for (uint32_t j = 0; j < nbp; ++j) {
                                    const uint32_t bj = rdl(bpp, j);
                                    st = o8 + s > bj ? rdl(bps, j) : st;
                                }
                                const uint32_t e = bsel(s < 4u ? e0 : e1, s);
                                const uint32_t r = bsel(s < 4u ? r8[0] : r8[1], s);
                                const uint32_t sp = st >> 16;
                                const bool eqv = (st & 0x1FFu) == r;
                                uint32_t mm = 0;
                                if (eqv && e == AGNES_CODE_POLKA_ANY && sp == AGNES_STEP_PREVOTE) mm = AGNES_VMSG_TIMEOUT_PREVOTE;
                                if (eqv && e == AGNES_CODE_PRECOMMIT_ANY && sp != AGNES_STEP_COMMIT) mm = AGNES_VMSG_TIMEOUT_PRECOMMIT;
                                if (s < 4u) x0 |= mm << (8u * s + 4u);
                                else x1 |= mm << (8u * (s - 4u) + 4u);
                                if (eqv && e == AGNES_CODE_POLKA_VALUE && sp == AGNES_STEP_PRECOMMIT && !((nilbc >> s) & 1u)) vl = s;
                            }
                        }
                        const uint64_t b = ballot(vl < 8u);
                        if (b) {
                            const uint32_t L0 = 63u - (uint32_t)__builtin_clzll(b);
                            vpos = 8u * L0 + rdl(vl, L0);
                        }
                        if (p1_at != NONE && (p1_at & LOCKF) && (vpos == NONE || (p1_at & ~LOCKF) > vpos)) vpos = p1_at & ~LOCKF; /* :198 set_valid */
                    }
                    /* the breakpoint votes' own messages */
                    for (uint32_t j = 0; j < nmsg; ++j) {
                        const uint32_t p = rdl(mat, j), mj = rdl(mv, j);
                        if (lane == (p >> 3)) {
                            const uint32_t sh = 8u * (p & 3u) + 4u;
                            if ((p & 7u) < 4u) x0 |= mj << sh;
                            else x1 |= mj << sh;
                        }
                    }
                    c0 |= x0;
                    c1 |= x1;
                    /* the instance's record: the State after the chunk and its change points */
                    if (lane == 0) {
                        rk[R_STEP] = step;
                        rk[R_EQ8] = eq8;
                        rk[R_RLT] = (uint32_t)rlt;
                        if (p1_at != NONE) rk[R_P1] = (p1_at & LOCKF) | (rc + (p1_at & ~LOCKF));
                        if (c_at != NONE) {
                            rk[R_C] = rc + c_at;
                            rk[R_DR] = dr;
                        }
                        if (vpos != NONE) rk[R_VP] = rc + vpos + 1u;
                        if (sk) rk[R_SK] = 1u;
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
            /* INVALID for the votes that failed the checks (a deferred instance's: left to
             * the LIST kernel, which writes them) */
            const uint32_t inv = actb & ~okb & ~defb;
            c0 |= bytes_of(inv & 0xFu) & (AGNES_CODE_INVALID * 0x01010101u);
            c1 |= bytes_of(inv >> 4) & (AGNES_CODE_INVALID * 0x01010101u);
            dc0 = c0;
            dc1 = c1;
            dc_act = actb;
            dc_at = c;
            __builtin_amdgcn_wave_barrier();
        }
        if (EVC) {
            __builtin_amdgcn_wave_barrier();
            if (lane < m) a.ev_counts[S.s0 + lane] = (uint64_t)ET[lane];
        }
        if (SM) { /* the States back: round (RoundSkip), locked, valid, decision, step */
            __builtin_amdgcn_wave_barrier();
            if (lane < m && !S.def && DCHK(S.s0 + lane < n, 11, S.s0 + lane, n)) {
                const uint32_t* const rk = IT + RW * lane;
                const uint32_t p1 = rk[R_P1], cc = rk[R_C], vp = rk[R_VP], sk = rk[R_SK], step = rk[R_STEP];
                uint4* const sp = reinterpret_cast<uint4*>(a.states + S.s0 + lane);
                const uint4 s0 = sp[0], s3 = sp[3];
                if (p1 != NONE || cc != NONE || vp != 0u || sk != 0u || step != (s3.y & 0xFFu)) {
                    uint4 s1 = sp[1], s2 = sp[2];
                    uint4 n0 = s0, n3 = s3;
                    uint32_t flags = s3.y;
                    if (sk) { /* the last RoundSkip's round */
                        n0.z = rk[R_EQ8];
                        n0.w = 0u;
                    }
                    if (p1 != NONE && (p1 & LOCKF)) { /* locked = {round, v} at P1 */
                        s1.x = s0.z;
                        s1.y = s0.w;
                        s2.z = (!ABL || (Sa + (p1 & ~LOCKF) < NV)) && DCHK(Sa + (p1 & ~LOCKF) < NV, 12, Sa + (p1 & ~LOCKF), NV) ? a.vb.value[Sa + (p1 & ~LOCKF)] : 0u;
                        flags |= 1u << 8;
                    }
                    if (vp != 0u) { /* valid = {round, v} of the last set_valid_value */
                        s1.z = s0.z;
                        s1.w = s0.w;
                        s2.w = (!ABL || (Sa + vp - 1u < NV)) && DCHK(Sa + vp - 1u < NV, 13, Sa + vp - 1u, NV) ? a.vb.value[Sa + vp - 1u] : 0u;
                        flags |= 1u << 16;
                    }
                    if (cc != NONE) { /* the decision */
                        s2.x = rk[R_DR];
                        s2.y = 0u;
                        n3.x = (!ABL || (Sa + cc < NV)) && DCHK(Sa + cc < NV, 14, Sa + cc, NV) ? a.vb.value[Sa + cc] : 0u;
                        flags |= 1u << 24;
                    }
                    n3.y = (flags & ~0xFFu) | step;
                    sp[0] = n0;
                    sp[1] = s1;
                    sp[2] = s2;
                    sp[3] = n3;
                }
            }
        }
    };

    for (;;) {
        const uint32_t m = H.e0 - H.s0;
        if (H.stream) {
            run_stream(H, true);
        } else {
            pf_at = ~0ull;
            for (uint32_t k = 0; k < m; ++k) {
                Hdr O;
                hdr_one(H, k, O);
                if (!O.stream) { /* >= 2^30 votes: the LIST kernel's */
                    if (lane == 0 && O.ln) {
                        const uint32_t li = atomicAdd(a.list_count, 1u);
                        if (DCHK(li < n, 15, li, n)) a.list[li] = O.s0;
                        if (EVC) a.walk[atomicAdd(a.list_count + AGNES_WALK_COUNT, 1u)] = O.s0;
                    }
                    continue;
                }
                run_stream(O, false);
                pf_at = ~0ull;
            }
        }
        if (N.s0 >= N.e0) break;
        if (N.stage < 3u) {
            if (N.stage == 1u) hdr2(N);
            hdr3(N);
        }
        H = N;
        range_of(rdl(tq, 0u), N.s0, N.e0);
        if (lane == 0) tq = atomicAdd(ctr, 1u);
        hdr1(N);
    }
    flush();
    const uint32_t nb = rdl(scan(bad), 63u);
    if (lane == 0 && nb) add_invalid(a.n_invalid, (unsigned long long)nb);
}

} // namespace dflow
} // namespace agnes

/* ------------------------------------------------------------------ */
/* launcher                                                            */

template <bool DEDUP, bool SKIP, bool EVC, bool SM>
static hipError_t launch_dflow_k(const agnes_tally_args* a, int num_cus, hipStream_t st) {
    const uint32_t n = a->vb.n_instances;
    if (n == 0) return hipSuccess;
    using agnes::dflow::dflow;
    const void* fns[2] = {reinterpret_cast<const void*>(&dflow<DEDUP, SKIP, false, EVC, SM>),
                          reinterpret_cast<const void*>(&dflow<DEDUP, SKIP, true, EVC, SM>)};
    const uint32_t lpw = agnes::dflow::layout(a->max_rounds, a->n_vals, EVC, SM).total;
    const uint64_t wave_lds = (uint64_t)lpw * AGNES_WAVES_PER_BLOCK;
    const uint64_t pcb = agnes::align16(4ull * a->n_sets * a->n_vals);
    /* blocks per CU from the occupancy query; the LDS power table only where it costs no
     * occupancy.  Cached per (kernel, LDS shape). */
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
    if (lds > 48u * 1024u) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    const uint64_t ncu = (uint64_t)(num_cus > 0 ? num_cus : 256);
    uint64_t blocks = ((uint64_t)n + 4u * AGNES_WAVES_PER_BLOCK - 1u) / (4u * AGNES_WAVES_PER_BLOCK);
    const uint64_t cap = ncu * (uint64_t)o->per_cu;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    if (o->pc) hipLaunchKernelGGL((dflow<DEDUP, SKIP, true, EVC, SM>), dim3((uint32_t)blocks), dim3(256), (size_t)lds, st, b, lpw);
    else hipLaunchKernelGGL((dflow<DEDUP, SKIP, false, EVC, SM>), dim3((uint32_t)blocks), dim3(256), (size_t)lds, st, b, lpw);
#if AGNES_DFLOW_CHECK
    {
        hipError_t e = hipStreamSynchronize(st);
        fprintf(stderr, "dflow check: DEDUP %d SKIP %d EVC %d SM %d n %u votes %llu R %u nv %u ns %u lpw %u blocks %llu pc %d: %s\n",
                (int)DEDUP, (int)SKIP, (int)EVC, (int)SM, n, (unsigned long long)a->vb.n_votes, a->max_rounds,
                a->n_vals, a->n_sets, lpw, (unsigned long long)blocks, (int)o->pc, hipGetErrorString(e));
        if (e != hipSuccess) return e;
        unsigned nbad = 0;
        (void)hipMemcpyFromSymbol(&nbad, HIP_SYMBOL(agnes_dflow_nbad), sizeof(nbad));
        uint32_t cnt[1 + AGNES_QUEUE_WORDS] = {0};
        (void)hipMemcpy(cnt, a->list_count, sizeof(uint32_t) * 2, hipMemcpyDeviceToHost);
        fprintf(stderr, "dflow check: %u violations, list %u\n", nbad, cnt[0]);
        if (cnt[0] > n) return hipErrorInvalidValue;
        if (cnt[0]) {
            std::vector<uint32_t> L(cnt[0]);
            (void)hipMemcpy(L.data(), a->list, sizeof(uint32_t) * cnt[0], hipMemcpyDeviceToHost);
            for (uint32_t i = 0; i < cnt[0]; ++i)
                if (L[i] >= n) {
                    fprintf(stderr, "dflow check: list[%u] = %u >= n\n", i, L[i]);
                    return hipErrorInvalidValue;
                }
        }
        if (nbad) return hipErrorInvalidValue;
    }
#endif
    return hipGetLastError();
}

bool agnes_dflow_supported(const agnes_tally_args* a) {
    /* rounds < 8 (the sort keys), the first-vote table in the wave's LDS, the columns
     * aligned for 16-B / 4-B LDS-DMA and the 8-B code stores of 128-vote chunks */
    const uintptr_t al16 = reinterpret_cast<uintptr_t>(a->vb.instance) | reinterpret_cast<uintptr_t>(a->vb.value) |
                           reinterpret_cast<uintptr_t>(a->vb.validator);
    const uintptr_t al4 = reinterpret_cast<uintptr_t>(a->vb.round) | reinterpret_cast<uintptr_t>(a->vb.type);
    const bool gathered = a->vb.weight == nullptr && a->carry == nullptr && !a->w64; /* u32 sums */
    return gathered && a->max_rounds >= 1u && a->max_rounds <= 8u && a->n_vals > 0u &&
           agnes::dflow::layout(a->max_rounds, a->n_vals, true, true).total <= 40u * 1024u && (al16 & 15u) == 0u &&
           (al4 & 3u) == 0u && (reinterpret_cast<uintptr_t>(a->codes) & 7u) == 0u && a->vb.validator != nullptr;
}

/* the stream kernel on the AUTO route when asked for (AGNES_FLAG_ROUTE_STREAM); a build
 * with AGNES_DFLOW_AUTO=1 takes it for every supported batch (A/B experiments) */
#ifndef AGNES_DFLOW_AUTO
#define AGNES_DFLOW_AUTO 0
#endif
bool agnes_dflow_route(const agnes_tally_args* a) {
    const uint32_t route = (a->flags >> AGNES_ROUTE_SHIFT) & AGNES_ROUTE_MASK;
    return (AGNES_DFLOW_AUTO || (a->flags & AGNES_FLAG_ROUTE_STREAM) != 0u) && route == AGNES_ROUTE_AUTO &&
           agnes_dflow_supported(a);
}

template <bool DEDUP, bool SKIP>
static hipError_t launch_dflow_m(const agnes_tally_args* a, int num_cus, hipStream_t st) {
    const bool sm = (a->flags & AGNES_FLAG_STATE_MACHINE) != 0 && a->states != nullptr;
    if (a->ev_counts) return sm ? launch_dflow_k<DEDUP, SKIP, true, true>(a, num_cus, st)
                                : launch_dflow_k<DEDUP, SKIP, true, false>(a, num_cus, st);
    return sm ? launch_dflow_k<DEDUP, SKIP, false, true>(a, num_cus, st) : launch_dflow_k<DEDUP, SKIP, false, false>(a, num_cus, st);
}

hipError_t agnes_launch_dflow(const agnes_tally_args* a, uint32_t mode, int num_cus, hipStream_t st) {
    const bool skip = (a->flags & AGNES_FLAG_ROUND_SKIP) != 0;
    if (mode == AGNES_MODE_DEDUP) return skip ? launch_dflow_m<true, true>(a, num_cus, st) : launch_dflow_m<true, false>(a, num_cus, st);
    return launch_dflow_m<false, true>(a, num_cus, st);
}
