/*
 * agnes_sieve.hip — the DEDUP / RoundSkip tally (BASELINE C4: duplicates,
 * equivocations, Zipf powers, +1/3 round skips), codes only; the State machine
 * runs after it in the one-instance-per-lane apply pass (agnes_apply.hip).
 *
 * One wave walks one instance at a time (work queue of instance batches) in
 * 512-vote chunks, lane l holding votes 8l .. 8l+7.  Per chunk:
 *   K1   loads (16-B / 4-B lanes), the boundary's checks, the weight gather;
 *   DEDUP the first vote of each (round, type, validator) of the instance wins
 *        (SURVEY.md gap 1: the reference run on the first-vote-filtered stream);
 *        RoundSkip's first vote of each (round, validator): LDS tables of
 *        (instance epoch << lb | LMASK - local index) lowered by atomic max, so
 *        the earliest vote wins whatever order the lanes' atomics land in;
 *   K2+3 ONE pass per round present for BOTH vote types: each vote adds its weight
 *        to its type's half of two u64 lane accumulators (all votes / nil votes,
 *        32-bit halves: Zipf powers up to 2^20 do not fit flow's 16-bit fields),
 *        five DPP wave scans (prevote / precommit x all / nil, the distinct-
 *        validator RoundSkip sum), then per vote is_quorum on its own type's sums
 *        (round_votes.rs:31-33) with precedence Value > Nil > Any > Init (:58-66)
 *        as a level, to_event (vote_executor.rs:26-36) by one byte lookup, and the
 *        RoundSkip bit (3 * distinct > total, applied before the vote's event,
 *        state_machine.rs:210).
 * tally_fast (agnes_fast.hip) did one pass per (round, type) key over 256-vote
 * chunks: ~5 passes per 256 votes on C4 against ~2 per 512 here.
 *
 * Domain (else the instance goes to the i64 LIST kernel, as tally_fast): a u32
 * power set with every sum of the instance < 2^31 (len * maxpow < 2^31); instances
 * of at most 2^lb votes (lb = the launcher's epoch shift).
 */
#include "agnes_fast.h"

namespace agnes {
namespace sieve {
using namespace agnes::fast;

constexpr uint32_t LV = 8u, CH = 64u * LV; /* votes per lane, per chunk */
constexpr uint32_t SB = 4u;                 /* instances per work-queue batch */

/* to_event by index type * 4 + level (Init, Any, Nil, Value): vote_executor.rs:26-36 */
constexpr uint32_t EV_LO = AGNES_CODE_NONE | (AGNES_CODE_POLKA_ANY << 8) | (AGNES_CODE_POLKA_NIL << 16) |
                           (AGNES_CODE_POLKA_VALUE << 24);
constexpr uint32_t EV_HI = AGNES_CODE_NONE | (AGNES_CODE_PRECOMMIT_ANY << 8) | (AGNES_CODE_NONE << 16) |
                           (AGNES_CODE_PRECOMMIT_VALUE << 24);

/* DMA slot: each column of the next chunk as a contiguous image */
constexpr uint32_t F_INST = 0, F_VALUE = 2048, F_VAL = 4096, F_ROUND = 6144, F_TYPE = 6656, F_BYTES = 7168;

/* per-wave LDS: carried executors ca[2R] (all votes), cn[2R] (nil), cs[R] (distinct
 * RoundSkip weight) | DEDUP table [2R][nv] | RoundSkip table [R][nv] | DMA slot */
__host__ __device__ inline void layout(uint32_t mode, bool skip, uint32_t R, uint32_t nv, uint32_t* o_fv,
                                       uint32_t* o_fs, uint32_t* o_slot, uint32_t* total) {
    uint32_t o = (uint32_t)align16(20ull * R);
    *o_fv = o;
    if (mode == AGNES_MODE_DEDUP) o = (uint32_t)align16(o + 8ull * R * nv);
    *o_fs = o;
    if (skip) o = (uint32_t)align16(o + 4ull * R * nv);
    *o_slot = o;
    *total = o + F_BYTES;
}

/* LDS-DMA, saddr form (uniform 64-bit base + 32-bit lane offset), non-temporal: the
 * vote columns are read once */
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

__device__ __forceinline__ uint32_t wave_or(uint32_t x) { /* every lane active */
    x |= dpp<0x111, 0xf>(x);
    x |= dpp<0x112, 0xf>(x);
    x |= dpp<0x114, 0xf>(x);
    x |= dpp<0x118, 0xf>(x);
    x |= dpp<0x142, 0xa>(x);
    x |= dpp<0x143, 0xc>(x);
    return rdl(x, 63u);
}
__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }

template <uint32_t MODE, bool SKIP, bool PC>
__global__ __launch_bounds__(256) void sieve(agnes_tally_args a, uint32_t lds_per_wave) {
    const uint32_t lane = lane_id();
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint32_t R = a.max_rounds, nv = a.n_vals, ns = a.n_sets, n = a.vb.n_instances;
    const uint64_t NV = a.vb.n_votes;
    const uint32_t p0 = LV * lane;

    if (PC) { /* block-shared u32 power table (launcher-staged only when it costs no occupancy) */
        uint32_t* pc = reinterpret_cast<uint32_t*>(agnes_smem);
        const uint32_t np = ns * nv;
        for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) pc[k] = a.power32[k];
        __syncthreads();
    }
    uint32_t o_fv, o_fs, o_slot, o_tot;
    layout(MODE, SKIP, R, nv, &o_fv, &o_fs, &o_slot, &o_tot);
    unsigned char* const base = agnes_smem + a.power_cache + wave * lds_per_wave;
    uint32_t* const ca = reinterpret_cast<uint32_t*>(base); /* [2R] all-vote weight carried */
    uint32_t* const cn = ca + 2u * R;                        /* [2R] nil weight              */
    uint32_t* const cs = cn + 2u * R;                        /* [R]  distinct RoundSkip weight */
    uint32_t* const first_v = reinterpret_cast<uint32_t*>(base + o_fv);
    uint32_t* const first_s = reinterpret_cast<uint32_t*>(base + o_fs);
    unsigned char* const slot = base + o_slot;
    const uint32_t slotl = lds_addr(slot);
    const uint32_t o16 = 16u * lane, o4 = 4u * lane;
    uint64_t pf_at = ~0ull; /* the chunk held (or in flight) in the slot */
    /* the full chunk at c into the slot (c + CH <= NV, c a multiple of 4) */
    auto dma_chunk = [&](uint64_t c) {
        __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): the slot's LDS reads are done */
        sdma16(a.vb.instance + c, o16, slotl + F_INST);
        sdma16(a.vb.instance + c + 256u, o16, slotl + F_INST + 1024u);
        sdma16(a.vb.value + c, o16, slotl + F_VALUE);
        sdma16(a.vb.value + c + 256u, o16, slotl + F_VALUE + 1024u);
        sdma16(a.vb.validator + c, o16, slotl + F_VAL);
        sdma16(a.vb.validator + c + 256u, o16, slotl + F_VAL + 1024u);
        sdma4(a.vb.round + c, o4, slotl + F_ROUND);
        sdma4(a.vb.round + c + 256u, o4, slotl + F_ROUND + 256u);
        sdma4(a.vb.type + c, o4, slotl + F_TYPE);
        sdma4(a.vb.type + c + 256u, o4, slotl + F_TYPE + 256u);
        pf_at = c;
    };
    if (MODE == AGNES_MODE_DEDUP) fill_u32(first_v, 2ull * R * nv, 0u, lane);
    if (SKIP) fill_u32(first_s, (uint64_t)R * nv, 0u, lane);
    const uint32_t lb = a.epoch_shift, lmask = (1u << lb) - 1u;
    const uint32_t emax = lb >= 31u ? 1u : ((1u << (32u - lb)) - 1u);
    uint32_t ep = 0, bad = 0;

    /* work queue: batches of SB consecutive instances, many counters (same-address
     * device atomics serialise) */
    const uint32_t qn = gridDim.x < QN ? gridDim.x : QN;
    const uint32_t qk = blockIdx.x % qn;
    uint32_t* const ctr = a.list_count + 1u + qk;
    auto range_of = [&](uint32_t t, uint32_t& s0, uint32_t& e0) {
        const uint64_t b0 = ((uint64_t)t * qn + qk) * SB;
        s0 = b0 < n ? (uint32_t)b0 : n;
        e0 = b0 + SB < n ? (uint32_t)(b0 + SB) : n;
    };
    uint32_t q, qe, nS, nE, tq = 0;
    {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(ctr, 2u);
        t = rdl(t, 0u);
        range_of(t, q, qe);
        range_of(t + 1u, nS, nE);
        if (lane == 0) tq = atomicAdd(ctr, 1u);
    }
    /* instance header in lanes: 0, 1 offsets[i] lo / hi, 2, 3 offsets[i + 1], 4 its set */
    auto load_hdr = [&](uint32_t i) -> uint32_t {
        uint32_t h = 0;
        if (i < n) {
            if (lane < 4u) h = reinterpret_cast<const uint32_t*>(a.vb.offsets + i)[lane];
            else if (lane == 4u) h = a.vb.instance_set ? a.vb.instance_set[i] : (ns ? i % ns : 0u);
        }
        return h;
    };
    auto succ = [&]() -> uint32_t { return q + 1u < qe ? q + 1u : (nS < nE ? nS : n); };
    uint32_t hq = q < qe ? load_hdr(q) : 0u;

    while (q < qe) {
        const uint32_t hn = load_hdr(succ()); /* the next instance's header, one ahead */
        const uint32_t i = q;
        uint64_t beg = u64of(rdl(hq, 0u), rdl(hq, 1u)), end = u64of(rdl(hq, 2u), rdl(hq, 3u));
        beg = beg < NV ? beg : NV;
        end = end < NV ? end : NV;
        end = end > beg ? end : beg;
        const uint32_t set = rdl(hq, 4u);
        const bool set_ok = set < ns;
        uint32_t q2 = 0, q1 = 0;
        bool run = end > beg;
        if (set_ok) {
            const agnes_set_info si = a.sets[set];
            const uint64_t len = end - beg;
            /* sums provably < 2^31 (u32 arithmetic), else the i64 LIST kernel */
            if (!si.fast || len >= (1ull << 31) || len * (uint64_t)si.maxpow >= (1ull << 31)) {
                if (run && lane == 0) a.list[atomicAdd(a.list_count, 1u)] = i;
                run = false;
            }
            q2 = si.q2 < 0x7FFFFFFFu ? si.q2 : 0x7FFFFFFFu;
            q1 = si.q1 < 0x7FFFFFFFu ? si.q1 : 0x7FFFFFFFu;
        }
        if (run) {
            if (MODE == AGNES_MODE_DEDUP || SKIP) {
                if (++ep > emax) { /* epoch space used up: recycle the tables */
                    if (MODE == AGNES_MODE_DEDUP) fill_u32(first_v, 2ull * R * nv, 0u, lane);
                    if (SKIP) fill_u32(first_s, (uint64_t)R * nv, 0u, lane);
                    ep = 1;
                }
            }
            const uint32_t pbase = set_ok ? set * nv : 0u, nvs = set_ok ? nv : 0u;
            const uint64_t c0 = beg & ~3ull;
            if (end - c0 > CH) { /* RoundVotes::new per round (round_votes.rs:83-90) */
                for (uint32_t k = lane; k < 5u * R; k += 64u) ca[k] = 0u;
                __builtin_amdgcn_wave_barrier();
            }
            for (uint64_t c = c0; c < end; c += CH) {
                const uint32_t lo_r = (uint32_t)(beg > c ? beg - c : 0ull);
                const uint32_t hi_r = end - c < CH ? (uint32_t)(end - c) : CH;
                const uint64_t j0 = c + p0;
                /* ---- K1 ---- */
                uint32_t inst[LV], value[LV], val[LV], r8[2], t8[2];
                if (pf_at == c) { /* prefetched by LDS-DMA */
                    dma_wait();
                    const uint32_t o32 = 32u * lane, o8 = 8u * lane;
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
                } else if (j0 + LV <= NV) {
                    const uint4 i0 = *reinterpret_cast<const uint4*>(a.vb.instance + j0);
                    const uint4 i1 = *reinterpret_cast<const uint4*>(a.vb.instance + j0 + 4u);
                    const uint4 v0 = *reinterpret_cast<const uint4*>(a.vb.value + j0);
                    const uint4 v1 = *reinterpret_cast<const uint4*>(a.vb.value + j0 + 4u);
                    const uint4 d0 = *reinterpret_cast<const uint4*>(a.vb.validator + j0);
                    const uint4 d1 = *reinterpret_cast<const uint4*>(a.vb.validator + j0 + 4u);
                    r8[0] = *reinterpret_cast<const uint32_t*>(a.vb.round + j0);
                    r8[1] = *reinterpret_cast<const uint32_t*>(a.vb.round + j0 + 4u);
                    t8[0] = *reinterpret_cast<const uint32_t*>(a.vb.type + j0);
                    t8[1] = *reinterpret_cast<const uint32_t*>(a.vb.type + j0 + 4u);
                    inst[0] = i0.x; inst[1] = i0.y; inst[2] = i0.z; inst[3] = i0.w;
                    inst[4] = i1.x; inst[5] = i1.y; inst[6] = i1.z; inst[7] = i1.w;
                    value[0] = v0.x; value[1] = v0.y; value[2] = v0.z; value[3] = v0.w;
                    value[4] = v1.x; value[5] = v1.y; value[6] = v1.z; value[7] = v1.w;
                    val[0] = d0.x; val[1] = d0.y; val[2] = d0.z; val[3] = d0.w;
                    val[4] = d1.x; val[5] = d1.y; val[6] = d1.z; val[7] = d1.w;
                } else {
                    r8[0] = r8[1] = t8[0] = t8[1] = 0u;
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        const bool in = j0 + s < NV;
                        inst[s] = in ? a.vb.instance[j0 + s] : 0u;
                        value[s] = in ? a.vb.value[j0 + s] : 0u;
                        val[s] = in ? a.vb.validator[j0 + s] : 0u;
                        r8[s >> 2] |= (in ? (uint32_t)a.vb.round[j0 + s] : 0u) << (8u * (s & 3u));
                        t8[s >> 2] |= (in ? (uint32_t)a.vb.type[j0 + s] : 0u) << (8u * (s & 3u));
                    }
                }
                /* the boundary's checks: the vote names its instance, round < R, type in
                 * {0, 1}, validator in the set; in: inside [beg, end) */
                uint32_t inm = 0, okm = 0; /* bit s (bitwise tests: no per-vote branches) */
#pragma unroll
                for (uint32_t s = 0; s < LV; ++s) {
                    const uint32_t r = byte_of(r8[s >> 2], s & 3u), t = byte_of(t8[s >> 2], s & 3u);
                    const uint32_t in = (uint32_t)(p0 + s >= lo_r) & (uint32_t)(p0 + s < hi_r);
                    const uint32_t ok = in & (uint32_t)(inst[s] == i) & (uint32_t)(r < R) & (uint32_t)(t <= 1u) &
                                        (uint32_t)(val[s] < nvs);
                    inm |= in << s;
                    okm |= ok << s;
                }
                /* K1: w = power[set][validator] (consensus_executor.rs:62-63 -> validators.rs:7);
                 * a vote that checked out reads entry 0 and weighs 0 */
                uint32_t w[LV];
#pragma unroll
                for (uint32_t s = 0; s < LV; ++s) {
                    const uint32_t idx = pbase + (((okm >> s) & 1u) ? val[s] : 0u);
                    w[s] = PC ? reinterpret_cast<const uint32_t*>(agnes_smem)[idx] : a.power32[idx];
                }
#pragma unroll
                for (uint32_t s = 0; s < LV; ++s) w[s] = ((okm >> s) & 1u) ? w[s] : 0u;
                bad += (uint32_t)__builtin_popcount(inm & ~okm);
                uint32_t nilm = 0; /* bit s: a nil vote */
#pragma unroll
                for (uint32_t s = 0; s < LV; ++s) nilm |= (uint32_t)(value[s] == AGNES_NIL) << s;
                /* a gather from HBM retires before the DMA below is issued (vmcnt retires in
                 * issue order); then the next chunk: this instance's, or the next one's first */
                if (!PC) asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]), "v"(w[5]),
                                      "v"(w[6]), "v"(w[7]));
                {
                    uint64_t nc = c + CH;
                    if (nc >= end) {
                        nc = ~0ull;
                        if (succ() < n) {
                            const uint64_t nb = u64of(rdl(hn, 0u), rdl(hn, 1u)), ne = u64of(rdl(hn, 2u), rdl(hn, 3u));
                            if (ne > nb && nb < NV) nc = nb & ~3ull;
                        }
                    }
                    if (nc != ~0ull && nc + CH <= NV) dma_chunk(nc);
                    else pf_at = ~0ull;
                }

                /* first-vote tables: the earliest vote of the instance wins (DEDUP: per (round,
                 * type, validator); RoundSkip: per (round, validator)) */
                uint32_t acc = okm, sfirst = 0;
                if (MODE == AGNES_MODE_DEDUP || SKIP) {
                    const uint32_t loc0 = (uint32_t)(c - beg) + p0; /* (wraps before beg: never ok) */
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        if ((okm >> s) & 1u) {
                            const uint32_t r = byte_of(r8[s >> 2], s & 3u), t = byte_of(t8[s >> 2], s & 3u);
                            const uint32_t enc = (ep << lb) | (lmask - (loc0 + s));
                            if (MODE == AGNES_MODE_DEDUP) atomicMax(&first_v[(r * 2u + t) * nv + val[s]], enc);
                            if (SKIP) atomicMax(&first_s[r * nv + val[s]], enc);
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    /* opaque copies: the read-back recomputes its addresses instead of keeping
                     * the atomics' 16 addresses live (register pressure) */
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) asm volatile("" : "+v"(val[s]));
                    asm volatile("" : "+v"(r8[0]), "+v"(r8[1]), "+v"(t8[0]), "+v"(t8[1]));
                    if (MODE == AGNES_MODE_DEDUP) acc = 0u;
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        if ((okm >> s) & 1u) {
                            const uint32_t r = byte_of(r8[s >> 2], s & 3u), t = byte_of(t8[s >> 2], s & 3u);
                            const uint32_t enc = (ep << lb) | (lmask - (loc0 + s));
                            if (MODE == AGNES_MODE_DEDUP)
                                acc |= (uint32_t)(*(volatile uint32_t*)&first_v[(r * 2u + t) * nv + val[s]] == enc) << s;
                            if (SKIP)
                                sfirst |= (uint32_t)(*(volatile uint32_t*)&first_s[r * nv + val[s]] == enc) << s;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                }

                /* ---- K2 + K3: one pass per round present, both vote types ---- */
                const bool ld_carry = c != c0, st_carry = c + CH < end;
                uint32_t rb = 0;
#pragma unroll
                for (uint32_t s = 0; s < LV; ++s) rb |= ((acc >> s) & 1u) << (byte_of(r8[s >> 2], s & 3u) & 31u);
                uint32_t rset = wave_or(rb);
                uint32_t lv[2] = {0u, 0u}, skb[2] = {0u, 0u}; /* levels / RoundSkip bits, byte per vote */
                while (rset) {
                    const uint32_t r = (uint32_t)__builtin_ctz(rset);
                    rset &= rset - 1u;
                    uint32_t am = 0; /* bit s: an accepted vote of round r */
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s)
                        am |= ((acc >> s) & 1u & (uint32_t)(byte_of(r8[s >> 2], s & 3u) == r)) << s;
                    /* the lane's totals: all-vote and nil weights per type (prevote in the low,
                     * precommit in the high half), distinct-validator weight */
                    uint64_t PA = 0, PN = 0;
                    uint32_t PS = 0;
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        const uint32_t wm = ((am >> s) & 1u) ? w[s] : 0u;
                        const uint32_t sh = (byte_of(t8[s >> 2], s & 3u) & 1u) << 5; /* 32 * type */
                        PA += (uint64_t)wm << sh;
                        PN += (uint64_t)(((nilm >> s) & 1u) ? wm : 0u) << sh;
                        if (SKIP) PS += ((sfirst >> s) & 1u) ? wm : 0u;
                    }
                    const uint32_t Tpa = (uint32_t)PA, Tca = (uint32_t)(PA >> 32);
                    const uint32_t Tpn = (uint32_t)PN, Tcn = (uint32_t)(PN >> 32);
                    const uint32_t Ipa = scan(Tpa), Ica = scan(Tca), Ipn = scan(Tpn), Icn = scan(Tcn);
                    uint32_t Is = 0;
                    if (SKIP) Is = scan(PS);
                    /* the sums before the lane: carry + exclusive wave prefix */
                    const uint32_t K = 2u * r;
                    const uint32_t bpa = (ld_carry ? ca[K] : 0u) + Ipa - Tpa;
                    const uint32_t bca = (ld_carry ? ca[K + 1u] : 0u) + Ica - Tca;
                    const uint32_t bpn = (ld_carry ? cn[K] : 0u) + Ipn - Tpn;
                    const uint32_t bcn = (ld_carry ? cn[K + 1u] : 0u) + Icn - Tcn;
                    /* thresholds on the lane prefixes, per type (prevote low, precommit high):
                     * value > q2 <=> (Da - Dn) > q2 - (ba - bn); nil > q2 <=> Dn > q2 - bn;
                     * value + nil > q2 <=> Da > q2 - ba */
                    const uint64_t TV = u64of(q2 - (bpa - bpn), q2 - (bca - bcn));
                    const uint64_t TN = u64of(q2 - bpn, q2 - bcn);
                    const uint64_t TA = u64of(q2 - bpa, q2 - bca);
                    uint32_t csr = 0, ts = 0;
                    if (SKIP) {
                        csr = ld_carry ? cs[r] : 0u;
                        ts = q1 - csr - (Is - PS);
                    }
                    /* a quiet round: even its sums after the chunk stay at or below the
                     * thresholds (every vote of it Init, no RoundSkip) -- the usual case for the
                     * few early next-round votes.  Uniform; sums < 2^31 in this domain. */
                    const uint32_t ktot = (ld_carry ? ca[K] : 0u) + rdl(Ipa, 63u), ktc = (ld_carry ? ca[K + 1u] : 0u) + rdl(Ica, 63u);
                    const bool quiet = ktot <= q2 && ktc <= q2 && (!SKIP || csr + rdl(Is, 63u) <= q1);
                    /* per vote (the lane prefixes again, fewer live registers): is_quorum on
                     * its own type's sums, precedence as a level; RoundSkip (3 * distinct >
                     * total <=> distinct > q1) */
                    uint64_t QA = 0, QN = 0;
                    uint32_t QS = 0;
                    if (!quiet)
#pragma unroll
                    for (uint32_t s = 0; s < LV; ++s) {
                        const uint32_t wm = ((am >> s) & 1u) ? w[s] : 0u;
                        const uint32_t sh = (byte_of(t8[s >> 2], s & 3u) & 1u) << 5;
                        QA += (uint64_t)wm << sh;
                        QN += (uint64_t)(((nilm >> s) & 1u) ? wm : 0u) << sh;
                        const uint32_t Da = (uint32_t)(QA >> sh), Dn = (uint32_t)(QN >> sh);
                        const int32_t tv = (int32_t)(uint32_t)(TV >> sh);
                        const int32_t tn = (int32_t)(uint32_t)(TN >> sh);
                        const int32_t ta = (int32_t)(uint32_t)(TA >> sh);
                        uint32_t l = (int32_t)Da > ta ? 1u : 0u;
                        l = (int32_t)Dn > tn ? 2u : l;
                        l = (int32_t)(Da - Dn) > tv ? 3u : l;
                        l = ((am >> s) & 1u) ? l : 0u;
                        lv[s >> 2] |= l << (8u * (s & 3u));
                        if (SKIP) {
                            QS += ((sfirst >> s) & 1u) ? wm : 0u;
                            skb[s >> 2] |= ((am >> s) & 1u & (uint32_t)((int32_t)QS > (int32_t)ts)) << (8u * (s & 3u) + 3u);
                        }
                    }
                    if (SKIP && st_carry && lane == 63u) cs[r] = csr + Is;
                    if (st_carry && lane == 63u) { /* the round's executors after the chunk */
                        ca[K] = bpa + Tpa;
                        ca[K + 1u] = bca + Tca;
                        cn[K] = bpn + Tpn;
                        cn[K + 1u] = bcn + Tcn;
                    }
                    __builtin_amdgcn_wave_barrier();
                }
                /* codes: to_event by (type, level) for accepted votes; INVALID / REJECTED */
#pragma unroll
                for (uint32_t u = 0; u < 2u; ++u) {
                    const uint32_t ix = lv[u] | ((t8[u] & 0x01010101u) << 2);
                    uint32_t code = __builtin_amdgcn_perm(EV_HI, EV_LO, ix & 0x07070707u) | skb[u];
                    uint32_t inb = 0;
#pragma unroll
                    for (uint32_t s = 0; s < 4u; ++s) {
                        const uint32_t b = 4u * u + s;
                        const uint32_t sft = 8u * s;
                        /* not tallied: INVALID, or REJECTED (DEDUP) */
                        const uint32_t x = ((okm >> b) & 1u) ? AGNES_CODE_REJECTED : AGNES_CODE_INVALID;
                        const uint32_t mk = ((acc >> b) & 1u) ? 0u : 0xFFu << sft;
                        code = (code & ~mk) | ((x << sft) & mk);
                        inb |= ((inm >> b) & 1u) << s;
                    }
                    const uint64_t at = j0 + 4u * u;
                    if (inb == 0xFu) {
                        *reinterpret_cast<uint32_t*>(a.codes + at) = code;
                    } else if (inb) {
#pragma unroll
                        for (uint32_t s = 0; s < 4u; ++s)
                            if ((inb >> s) & 1u) a.codes[at + s] = (uint8_t)(code >> (8u * s));
                    }
                }
            }
        }
        /* the next instance */
        if (q + 1u < qe) {
            ++q;
        } else {
            q = nS;
            qe = nE;
            if (q >= qe) break;
            range_of(rdl(tq, 0u), nS, nE); /* the batch after, grabbed one batch ago */
            if (lane == 0) tq = atomicAdd(ctr, 1u);
        }
        hq = hn;
    }
    dma_wait(); /* no LDS-DMA may land after the wave's LDS is handed on */
    const uint32_t nb = rdl(scan(bad), 63u);
    if (lane == 0 && nb) atomicAdd(a.n_invalid, (unsigned long long)nb);
}

} // namespace sieve
} // namespace agnes

/* ------------------------------------------------------------------ */
/* launcher                                                            */

static uint32_t sieve_lds(uint32_t mode, uint32_t flags, uint32_t R, uint32_t nv) {
    uint32_t fv, fs, sl, tot;
    agnes::sieve::layout(mode, (flags & AGNES_FLAG_ROUND_SKIP) != 0, R, nv, &fv, &fs, &sl, &tot);
    return tot;
}

bool agnes_sieve_supported(const agnes_tally_args* a, uint32_t mode) {
    /* rounds 0..31 in the rounds-present mask; the tables fit a wave's LDS share */
    return a->max_rounds <= 31u && sieve_lds(mode, a->flags, a->max_rounds, a->n_vals) <= AGNES_MAX_LDS_PER_WAVE;
}

template <uint32_t MODE, bool SKIP>
static hipError_t launch_sieve_k(const agnes_tally_args* a, int num_cus, hipStream_t st) {
    const uint32_t n = a->vb.n_instances;
    if (n == 0) return hipSuccess;
    using agnes::sieve::sieve;
    const void* fns[2] = {reinterpret_cast<const void*>(&sieve<MODE, SKIP, false>),
                          reinterpret_cast<const void*>(&sieve<MODE, SKIP, true>)};
    const uint32_t lpw = sieve_lds(MODE, a->flags, a->max_rounds, a->n_vals);
    const uint64_t wave_lds = (uint64_t)lpw * AGNES_WAVES_PER_BLOCK;
    const uint64_t pcb = agnes::align16(4ull * a->n_sets * a->n_vals);
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
    if (lds > 48u * 1024u) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    const uint64_t ncu = (uint64_t)(num_cus > 0 ? num_cus : 256);
    uint64_t blocks = ((uint64_t)n + agnes::sieve::SB * AGNES_WAVES_PER_BLOCK - 1u) /
                      (agnes::sieve::SB * AGNES_WAVES_PER_BLOCK);
    const uint64_t cap = ncu * (uint64_t)o->per_cu;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    if (o->pc) hipLaunchKernelGGL((sieve<MODE, SKIP, true>), dim3((uint32_t)blocks), dim3(256), (size_t)lds, st, b, lpw);
    else hipLaunchKernelGGL((sieve<MODE, SKIP, false>), dim3((uint32_t)blocks), dim3(256), (size_t)lds, st, b, lpw);
    return hipGetLastError();
}

hipError_t agnes_launch_sieve(const agnes_tally_args* a, uint32_t mode, int num_cus, hipStream_t st) {
    const bool skip = (a->flags & AGNES_FLAG_ROUND_SKIP) != 0;
    if (mode == AGNES_MODE_DEDUP)
        return skip ? launch_sieve_k<1, true>(a, num_cus, st) : launch_sieve_k<1, false>(a, num_cus, st);
    return skip ? launch_sieve_k<0, true>(a, num_cus, st) : launch_sieve_k<0, false>(a, num_cus, st);
}
