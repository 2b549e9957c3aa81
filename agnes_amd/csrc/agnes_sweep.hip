/*
 * agnes_sweep.hip — the walk kernel of the REFERENCE route without RoundSkip
 * (BASELINE C2/C3): the instances the flow kernel (agnes_flow.hip) hands off
 * through the walk list (unaligned offsets, long instances, power sets outside
 * the flow domain): ingest -> weight gather -> ordered tally -> quorum -> event
 * -> State::apply, ONE pass over the votes (consensus_executor.rs:61-69).
 *
 * The walk list is statically split over the waves: each instance is a stream of
 * its own, in 256-vote chunks (lane l = votes 4l..4l+3), starting at its first
 * vote rounded down to 4 (the votes before it masked); an instance whose sums may
 * reach 2^31 goes to the i64 LIST kernel.
 * The vote columns arrive by non-temporal LDS-DMA one chunk ahead; every address
 * is a uniform 64-bit base plus a 32-bit lane offset (saddr forms: no 64-bit
 * vector arithmetic per chunk).
 *
 * Per chunk:
 *   K1   validation (bit tests, SWAR on the round/type bytes), weight gather from
 *        the power table (block LDS copy when it fits, else L2);
 *   K2+3 per (round, type) key present: one stream-order scan of the value and
 *        nil weights (lane-local 4-vote prefix + DPP wave scan); a segment's
 *        running sum is scan - base + carry, so is_quorum (round_votes.rs:31-33)
 *        is one signed compare of the lane prefix against a per-lane threshold;
 *        Value > Nil > Any > Init (:58-66) and to_event (vote_executor.rs:26-36)
 *        by three selects;
 *   K4   State::apply for the vote events (state_machine.rs:196-211), lane
 *        parallel.  Without RoundSkip the step only moves Prevote -> Precommit at
 *        P1 (the first PolkaNil / PolkaValue at the State's round while in
 *        Prevote, :197-198) and -> Commit at C (the first PrecommitValue, any
 *        round, :211).  Per vote a v_perm table maps the event to its roles (P1
 *        candidate, commit, TimeoutPrevote :196, TimeoutPrecommit :208, PolkaValue
 *        :202); two ballots restricted to the vote's segment find P1 and C; every
 *        message nibble follows from the vote's position relative to them.
 *        Values reach the State at P1 (locked = valid, :198), at the last
 *        PolkaValue at the State's round before C (valid, :202) and at C (the
 *        decision).  In this domain (weights >= 0, executors fresh per call) the
 *        P1 and C votes carry their own value (a value quorum is crossed by a
 *        non-nil vote) and valid's value is that of the last NON-NIL PolkaValue
 *        vote before C (the label of a later nil PolkaValue vote is that value,
 *        round_votes.rs:50-54), so no label is ever searched.
 *
 * States: in place in states_out (the flow kernel copied the walked instances'
 * States through), staged in LDS by DMA when an instance starts, updated through
 * per-instance shadow records, written back when it ends.
 */
#include "agnes_fast.h"

namespace agnes {
namespace sweep {
using namespace agnes::fast;

constexpr uint32_t SB = 16u;    /* instances per batch (header offsets in lanes 0..SB) */
constexpr uint32_t HI = 32u;    /* header lanes HI + k: per-instance data of instance k */
constexpr uint32_t REC = 32u;   /* bytes of an instance record                          */
/* instance record words: quorum threshold, row base in the power table, validators
 * of its set (0: the set does not exist), State view (State.round if in 0..255 else
 * 0x100 | step << 16), shadow flags and values */
constexpr uint32_t R_Q2 = 0, R_PBASE = 1, R_NV = 2, R_SMW = 3, R_FLAGS = 4, R_LOCK = 5, R_VALID = 6, R_DEC = 7;
constexpr uint32_t F_LOCK = 1u, F_VALID = 2u, F_DEC = 4u; /* R_FLAGS bits; bits 8..15: decision round */

/* K4 roles of a vote event (byte lookup by v_perm, index = event code 0..7) */
constexpr uint32_t X_P1 = 0x01u, X_C = 0x02u, X_TP = 0x04u, X_TC = 0x08u, X_PV = 0x10u;
constexpr uint32_t XT_LO = (0u) | (X_TP << 8) | (X_P1 << 16) | ((X_P1 | X_PV) << 24); /* None, PolkaAny, PolkaNil, PolkaValue */
constexpr uint32_t XT_HI = (X_TC) | (X_C << 8);                                      /* PrecommitAny, PrecommitValue, -, - */
/* roles kept per step (byte lookup by step 0..7): NewRound / Propose: TimeoutPrecommit
 * and commit only (:208, :211); Prevote: all; Precommit: no P1 / TimeoutPrevote; Commit: none (:205) */
constexpr uint32_t SM_LO = (X_C | X_TC) | ((X_C | X_TC) << 8) | (0x1Fu << 16) | ((X_C | X_TC | X_PV) << 24);
constexpr uint32_t SM_HI = 0u;

__host__ __device__ inline uint32_t carry_bytes(uint32_t R) { return (uint32_t)align16(32ull * R); }
/* per-wave LDS: DMA chunk slot | carried executors (2 copies x (vw[2R], vn[2R]) u32) |
 * instance records | (State machine) the batch's staged States */
__host__ __device__ inline uint32_t lds_bytes(bool sm, uint32_t R) {
    return PF_BYTES + carry_bytes(R) + SB * REC + (sm ? SB * 64u : 0u);
}

/* 0x80 in the bytes of x that are zero (exact, no borrow) */
__device__ __forceinline__ uint32_t zero_marks(uint32_t x) {
    const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    return ((t | x) & 0x80808080u) ^ 0x80808080u;
}
/* 0xFF in the bytes below byte i (i <= 4) */
__device__ __forceinline__ uint32_t below_bytes(uint32_t i) { return i >= 4u ? 0xFFFFFFFFu : (1u << (8u * i)) - 1u; }
__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
/* wave-wide OR of x (every lane active) */
__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
    x |= dpp<0x111, 0xf>(x);
    x |= dpp<0x112, 0xf>(x);
    x |= dpp<0x114, 0xf>(x);
    x |= dpp<0x118, 0xf>(x);
    x |= dpp<0x142, 0xa>(x);
    x |= dpp<0x143, 0xc>(x);
    return rdl(x, 63u);
}

/* saddr forms: address = uniform 64-bit base + 32-bit lane offset.  The LDS-DMAs
 * are non-temporal (each vote byte is read once). */
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
__device__ __forceinline__ void sstore4(void* base, uint32_t voff, uint32_t data) {
    asm volatile("global_store_dword %0, %1, %2" ::"v"(voff), "v"(data), "s"(base) : "memory");
}

/* a batch: instances [s0, e0); header VGPRs: lanes 0..m the offsets (clamped to
 * n_votes), lane HI + k the set (olo) and, after phase 2, the quorum threshold (q2)
 * of instance k */
struct Hdr {
    uint32_t s0, e0;
    uint32_t olo, ohi, q2;
    uint32_t f31;    /* bit k: instance k in the u32 domain (else the i64 LIST kernel) */
    uint32_t stream; /* walked by this kernel                                          */
    uint32_t ready;  /* phase 2 done                                                    */
};

template <bool PC, bool SM>
__global__ __launch_bounds__(256) void sweep(agnes_tally_args a, uint32_t lds_per_wave) {
    const uint32_t lane = lane_id();
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint32_t R = a.max_rounds, nv = a.n_vals, ns = a.n_sets, n = a.vb.n_instances;
    const uint64_t NV = a.vb.n_votes;
    const uint32_t p0 = 4u * lane, o16 = 16u * lane;
    /* nothing walked (every batch streamed): leave before staging anything */
    if (*(volatile const uint32_t*)(a.list_count + AGNES_WALK_COUNT) == 0u) return;

    /* block-shared u32 power table (launcher-staged only when it costs no occupancy) */
    if (PC) {
        uint32_t* pc = reinterpret_cast<uint32_t*>(agnes_smem);
        const uint32_t np = ns * nv;
        for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) pc[k] = a.power32[k];
        __syncthreads();
    }
    unsigned char* const base = agnes_smem + a.power_cache + wave * lds_per_wave;
    unsigned char* const pfb = base;
    const uint32_t pfl = lds_addr(pfb);
    uint32_t* const crow = reinterpret_cast<uint32_t*>(base + PF_BYTES);
    const uint32_t cw = 4u * R; /* one carry copy: vw[2R] then vn[2R] */
    uint32_t* const itab = reinterpret_cast<uint32_t*>(base + PF_BYTES + carry_bytes(R));
    unsigned char* const sb = base + PF_BYTES + carry_bytes(R) + SB * REC;
    /* in place: the flow kernel copied the walked instances' States */
    const agnes_state* const st_in = a.states;
    uint32_t cpar = 0;
    uint64_t pf_at = ~0ull;
    uint32_t bad = 0;
    /* r < R <=> ((r & 0x7F) + 128 - R) < 128 and r < 128 (R <= 15) */
    const uint32_t RK = (128u - R) * 0x01010101u;

    /* ---- work: this wave's slice of the walk list, one instance at a time ---- */
    uint32_t wl = 0, wend = 0;
    {
        const uint32_t L = rfl(*(volatile uint32_t*)(a.list_count + AGNES_WALK_COUNT));
        const uint32_t W = gridDim.x * AGNES_WAVES_PER_BLOCK, gw = blockIdx.x * AGNES_WAVES_PER_BLOCK + wave;
        wl = (uint32_t)((uint64_t)L * gw / W);
        wend = (uint32_t)((uint64_t)L * (gw + 1u) / W);
    }
    auto range_of = [&](uint32_t t, uint32_t& s0, uint32_t& e0) {
        const uint32_t e = wl + t;
        s0 = e < wend ? rfl(a.walk[e]) : n;
        e0 = e < wend ? s0 + 1u : n;
    };
    /* header phase 1: offsets and sets */
    auto hdr1 = [&](Hdr& h) {
        const uint32_t m = h.e0 - h.s0;
        uint32_t lo = 0, hi = 0;
        if (m > 0u && lane <= m) {
            const uint64_t o = a.vb.offsets[h.s0 + lane];
            const uint64_t oc = o < NV ? o : NV;
            lo = (uint32_t)oc;
            hi = (uint32_t)(oc >> 32);
        } else if (lane >= HI && lane < HI + m) {
            const uint32_t k = h.s0 + lane - HI;
            lo = a.vb.instance_set ? a.vb.instance_set[k] : (ns ? k % ns : 0u);
        }
        h.olo = lo;
        h.ohi = hi;
        h.q2 = 0;
        h.f31 = h.stream = h.ready = 0;
    };
    /* header phase 2 (needs phase 1): per instance its quorum threshold and domain,
     * per batch whether this kernel walks it */
    auto hdr2 = [&](Hdr& h) {
        const uint32_t m = h.e0 - h.s0;
        const bool il = lane >= HI && lane < HI + m;
        const uint32_t k = il ? lane - HI : 0u;
        const uint64_t ob = u64of(shfl(h.olo, k), shfl(h.ohi, k));
        const uint64_t oe = u64of(shfl(h.olo, k + 1u), shfl(h.ohi, k + 1u));
        const uint64_t len = oe > ob ? oe - ob : 0ull;
        bool f31 = false;
        uint32_t q2 = 0;
        if (il) {
            const uint32_t set = h.olo;
            if (set < ns) {
                const agnes_set_info si = a.sets[set];
                const uint64_t wmax = len * (uint64_t)si.maxpow; /* no sum of the instance exceeds it */
                f31 = si.fast && len < (1ull << 30) && wmax < (1ull << 31);
                /* 3s > 2t <=> s > q2; a q2 >= wmax is never crossed, so min(q2, wmax) */
                const uint64_t qq = (uint64_t)si.q2 < wmax ? (uint64_t)si.q2 : wmax;
                q2 = (uint32_t)(qq < 0x7FFFFFFFull ? qq : 0x7FFFFFFFull);
            } else {
                f31 = len < (1ull << 30); /* no such set: every vote INVALID */
            }
        }
        h.q2 = q2;
        const uint32_t full = (uint32_t)((1ull << m) - 1ull);
        h.f31 = (uint32_t)(ballot(f31) >> HI) & full;
        h.stream = m == 1u && h.f31 == 1u;
        h.ready = 1;
    };
    /* the batch's States into LDS (64 B each, lane l's 16 B at 16 l) */
    auto dma_states = [&](const Hdr& h) {
        const uint32_t m = h.e0 - h.s0;
        if (!SM || m == 0u) return;
        const unsigned char* src = reinterpret_cast<const unsigned char*>(st_in + h.s0) + 16u * (lane < 4u * m ? lane : 0u);
        glds16(src, sb);
    };
    /* the next chunk of the stream into the DMA slot (c: its first vote) */
    auto dma_chunk = [&](uint64_t c) {
        __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): the slot's LDS reads are done */
        sdma16(a.vb.instance + c, o16, pfl + PF_INST);
        sdma16(a.vb.value + c, o16, pfl + PF_VALUE);
        sdma16(a.vb.validator + c, o16, pfl + PF_VAL);
        sdma4(a.vb.round + c, p0, pfl + PF_ROUND);
        sdma4(a.vb.type + c, p0, pfl + PF_TYPE);
    };

    /* deferred code stores (vmcnt retires in issue order: issued behind the next
     * chunk's gather and DMA) */
    uint64_t dc_at = ~0ull;
    uint32_t dc_code = 0, dc_pos = 0; /* dc_pos: byte mask of the lane's votes to store */
    auto flush = [&]() {
        if (dc_at != ~0ull) {
            if (dc_pos == 0xFFFFFFFFu) {
                sstore4(a.codes + dc_at, p0, dc_code);
            } else if (dc_pos) {
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s)
                    if ((dc_pos >> (8u * s)) & 1u) a.codes[dc_at + p0 + s] = (uint8_t)(dc_code >> (8u * s));
            }
            dc_at = ~0ull;
        }
    };

    Hdr H, N;
    uint32_t tq = 0; /* lane 0: slot of the batch after N (atomic in flight) */
    {
        range_of(0u, H.s0, H.e0);
        range_of(1u, N.s0, N.e0);
        tq = 2u;
    }
    if (H.s0 >= H.e0) return;
    hdr1(H);
    dma_states(H);
    hdr1(N);
    hdr2(H);

    for (;;) { /* batches: H current, N next */
        const uint32_t m = H.e0 - H.s0;
        bool smf = SM; /* the State views are not yet set up from the staged States */
        if (!H.stream) {
            if (lane == 0) { /* sums may reach 2^31: the i64 LIST kernel */
                if (rdl(H.olo, 1u) != rdl(H.olo, 0u) || rdl(H.ohi, 1u) != rdl(H.ohi, 0u))
                    a.list[atomicAdd(a.list_count, 1u)] = H.s0;
            }
        } else {
            /* instance records */
            {
                const uint32_t q2k = shfl(H.q2, HI + lane);
                const uint32_t setk = shfl(H.olo, HI + lane);
                if (lane < m) {
                    uint32_t* const rk = itab + 8u * lane;
                    rk[R_Q2] = q2k;
                    rk[R_PBASE] = setk < ns ? setk * nv : 0u;
                    rk[R_NV] = setk < ns ? nv : 0u;
                    rk[R_SMW] = (uint32_t)AGNES_STEP_COMMIT << 16; /* no State machine: no role survives */
                    rk[R_FLAGS] = 0u;
                }
            }
            /* the stream: starts relative to its first chunk */
            const uint64_t O0 = u64of(rdl(H.olo, 0u), rdl(H.ohi, 0u));
            const uint64_t S0 = O0 & ~3ull;
            const uint32_t s0lo = (uint32_t)S0;
            const uint32_t lo0 = (uint32_t)O0 - s0lo; /* votes before the instance in its first chunk */
            const uint32_t Lend = rdl(H.olo, m) - s0lo;
            const uint32_t rl = lane == 0u ? 0u : H.olo - s0lo;
            const uint32_t rn = shfl(rl, lane + 1u);
            const uint64_t NE = ballot(lane < m && rn > rl);
            const uint32_t relv = lane <= m ? rl : 0x7FFFFFFFu;
            const uint64_t mm64 = (1ull << m) - 1ull;

            for (uint32_t rc = 0; rc < Lend; rc += CHUNK) {
                const uint64_t c = S0 + rc;
                /* this chunk's DMA (and a new batch's States) have landed */
                dma_wait();
                if (SM && smf) { /* the State machine's view of each instance (state_machine.rs:184) */
                    if (lane < m) {
                        const uint32_t* const sp = reinterpret_cast<const uint32_t*>(sb + 64u * lane);
                        const int64_t rnd = (int64_t)u64of(sp[2], sp[3]);
                        const uint32_t eq8 = (rnd >= 0 && rnd <= 255) ? (uint32_t)rnd : 0x100u;
                        itab[8u * lane + R_SMW] = eq8 | ((sp[13] & 0xFFu) << 16);
                    }
                    smf = false;
                }

                /* ---- segments: the instances the chunk straddles ---- */
                const uint32_t tj = relv - rc; /* instance start relative to the chunk */
                const uint32_t k0 = 63u - (uint32_t)__builtin_clzll(ballot((int32_t)tj <= 0) & mm64);
                uint64_t bk = ballot(tj - 1u < CHUNK - 1u) & NE; /* non-empty, starting inside */
                const bool multi = bk != 0ull;
                const bool cont0 = ((ballot((int32_t)tj < 0) >> k0) & 1ull) != 0ull;
                const uint32_t left = Lend - rc;
                const bool lastc = left > CHUNK && !ballot(tj == CHUNK);
                const uint32_t hi_r = left < CHUNK ? left : CHUNK;
                const uint32_t lo_r = rc == 0u ? lo0 : 0u;
                uint32_t kln = k0, ss = 0;
                uint64_t BL = 0;
                if (multi) {
                    uint32_t segw = k0, D = 0;
                    while (bk) {
                        const uint32_t k = (uint32_t)__builtin_ctzll(bk);
                        bk &= bk - 1ull;
                        ++D;
                        const uint32_t L = rdl(tj, k) >> 2; /* its first lane */
                        BL |= 1ull << L;
                        segw = lane == D ? (k | (L << 8)) : segw;
                    }
                    const uint32_t sw = shfl(segw, mbcnt64(BL >> 1));
                    kln = sw & 0xFFu;
                    ss = sw >> 8;
                }
                const uint32_t* const rk = itab + 8u * kln;
                const uint4 rec = *reinterpret_cast<const uint4*>(rk); /* q2, pbase, nv of its set, smw */
                /* the lane's votes in the stream (byte mask) */
                uint32_t posb;
                {
                    const uint32_t bh = hi_r > p0 ? (hi_r - p0 < 4u ? hi_r - p0 : 4u) : 0u;
                    const uint32_t bl = lo_r > p0 ? (lo_r - p0 < 4u ? lo_r - p0 : 4u) : 0u;
                    posb = below_bytes(bh) & ~below_bytes(bl);
                }

                /* ---- K1: votes of the chunk + validation + weight gather ---- */
                uint32_t value[VPL], val[VPL], r4, t4;
                uint32_t key4, okb;
                bool all_ok;
                {
                    uint32_t inst[VPL];
                    if (pf_at == c) { /* prefetched by LDS-DMA */
                        const uint4 ia = *reinterpret_cast<const uint4*>(pfb + PF_INST + o16);
                        const uint4 va = *reinterpret_cast<const uint4*>(pfb + PF_VALUE + o16);
                        const uint4 da = *reinterpret_cast<const uint4*>(pfb + PF_VAL + o16);
                        inst[0] = ia.x; inst[1] = ia.y; inst[2] = ia.z; inst[3] = ia.w;
                        value[0] = va.x; value[1] = va.y; value[2] = va.z; value[3] = va.w;
                        val[0] = da.x; val[1] = da.y; val[2] = da.z; val[3] = da.w;
                        r4 = *reinterpret_cast<const uint32_t*>(pfb + PF_ROUND + p0);
                        t4 = *reinterpret_cast<const uint32_t*>(pfb + PF_TYPE + p0);
                    } else { /* not prefetched (a wave's first chunk, the columns' end) */
                        const uint64_t j = c + p0;
                        r4 = t4 = 0;
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s) {
                            const bool in = j + s < NV;
                            inst[s] = in ? a.vb.instance[j + s] : 0u;
                            value[s] = in ? a.vb.value[j + s] : 0u;
                            val[s] = in ? a.vb.validator[j + s] : 0u;
                            r4 |= (in ? (uint32_t)a.vb.round[j + s] : 0u) << (8u * s);
                            t4 |= (in ? (uint32_t)a.vb.type[j + s] : 0u) << (8u * s);
                        }
                    }
                    /* the boundary's checks (round < R, type in {0, 1}, the vote names its
                     * instance, validator in the set); keys round * 2 + type */
                    const uint32_t id = H.s0 + kln;
                    const uint32_t rt_bad = R == 1u ? (t4 & 0xFEFEFEFEu) | r4
                                                    : (t4 & 0xFEFEFEFEu) | ((r4 | ((r4 & 0x7F7F7F7Fu) + RK)) & 0x80808080u);
                    key4 = ((r4 << 1) & 0xFEFEFEFEu) | t4;
                    all_ok = false; /* the exact per-vote checks */
                    okb = posb;
                    {
                        okb = 0;
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s) {
                            const bool o = ((rt_bad >> (8u * s)) & 0xFFu) == 0u && inst[s] == id && val[s] < rec.z;
                            okb |= o ? 0xFFu << (8u * s) : 0u;
                        }
                        okb &= posb;
                        bad += (uint32_t)__builtin_popcount(posb & ~okb) >> 3;
                    }
                    key4 |= ~okb; /* no key: 0xFF */
                }
                uint32_t w[VPL];
                {
                    /* K1: w = power[set][validator] (consensus_executor.rs:62-63 ->
                     * validators.rs:7); a vote that checked out reads entry 0 */
                    const uint32_t pb = rec.y;
                    if (all_ok && hi_r == CHUNK) { /* every vote of the chunk checked in: val < n_vals */
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s)
                            w[s] = PC ? reinterpret_cast<const uint32_t*>(agnes_smem)[pb + val[s]] : a.power32[pb + val[s]];
                    } else {
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s) {
                            const uint32_t idx = ((okb >> (8u * s)) & 1u) ? pb + val[s] : 0u;
                            w[s] = PC ? reinterpret_cast<const uint32_t*>(agnes_smem)[idx] : a.power32[idx];
                        }
                    }
                }
                /* a gather from HBM retires before the DMA below is issued: a wait on it
                 * behind the DMA would wait for the DMA too (in-order vmcnt) */
                if (!PC) asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));
                /* the next chunk by LDS-DMA (this stream's, or the next batch's first),
                 * then the previous chunk's codes */
                {
                    uint64_t nc = ~0ull;
                    if (rc + CHUNK < Lend) nc = c + CHUNK;
                    if (nc != ~0ull && nc + CHUNK <= NV) {
                        dma_chunk(nc);
                        pf_at = nc;
                    } else {
                        pf_at = ~0ull;
                    }
                }
                flush();

                /* per-vote code: INVALID for a vote that checked out, else the tally event below */
                uint32_t c4 = (posb & ~okb) & (AGNES_CODE_INVALID * 0x01010101u);
                bool nil[VPL];
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s) nil[s] = value[s] == AGNES_NIL;

                /* carried executors: read row A (segment 0, when it continues from the
                 * previous chunk), write row B (the segment running into the next chunk) */
                uint32_t* const A = crow + cpar * cw;
                uint32_t* const B = crow + (cpar ^ 1u) * cw;
                if (lastc) {
                    const bool keep = !multi && cont0;
                    for (uint32_t k = lane; k < cw; k += 64u) B[k] = keep ? A[k] : 0u;
                    __builtin_amdgcn_wave_barrier();
                }
                const uint32_t q2 = rec.x;
                const uint32_t srcl = (ss ? ss : 1u) - 1u; /* the lane before my segment's first */

                /* K2+K3 per (round, type) key present: one stream-order scan of its value
                 * and nil weights over the chunk (VoteCount::add_vote, round_votes.rs:48-56)
                 * and, per vote, is_quorum with precedence Value > Nil > Any > Init
                 * (:31-33, :58-66) and to_event (vote_executor.rs:26-36) */
                uint32_t kset;
                if (R == 1u) {
                    kset = 3u;
                } else {
                    uint32_t kb = 0;
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s) kb |= 1u << (((key4 >> (8u * s)) & 0xFFu) & 31u);
                    kset = wave_or(kb & 0x7FFFFFFFu);
                }
                while (kset) {
                    const uint32_t K = (uint32_t)__builtin_ctz(kset);
                    kset &= kset - 1u;
                    uint32_t av[VPL], an[VPL];
                    bool in[VPL];
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s) {
                        in[s] = ((key4 >> (8u * s)) & 0xFFu) == K;
                        av[s] = (in[s] && !nil[s]) ? w[s] : 0u;
                        an[s] = (in[s] && nil[s]) ? w[s] : 0u;
                    }
                    av[1] += av[0]; av[2] += av[1]; av[3] += av[2];
                    an[1] += an[0]; an[2] += an[1]; an[3] += an[2];
                    const uint32_t iv = scan(av[3]), inn = scan(an[3]);
                    const uint32_t exv = iv - av[3], exn = inn - an[3];
                    /* segment 0's carry-in (uniform LDS reads) */
                    const uint32_t cv = cont0 ? A[K] : 0u, cn = cont0 ? A[2u * R + K] : 0u;
                    /* running sum of vote s = (lane prefix) + exclusive - base + carry, so
                     * sum > q2  <=>  lane prefix > q2 + base - carry - exclusive */
                    uint32_t bv = 0, bn = 0;
                    if (multi) {
                        /* the shuffles run in every lane (a lane outside a ds_bpermute's exec
                         * mask reads as 0 to the others) */
                        const uint32_t xv = shfl(iv, srcl), xn = shfl(inn, srcl);
                        bv = ss ? xv : 0u;
                        bn = ss ? xn : 0u;
                    }
                    const uint32_t ccv = ss ? 0u : cv, ccn = ss ? 0u : cn;
                    const int32_t tv = (int32_t)(q2 + bv - ccv - exv);
                    const int32_t tn = (int32_t)(q2 + bn - ccn - exn);
                    /* value + nil > q2: the two thresholds' sum less one q2 (mod 2^32) */
                    const int32_t ta = (int32_t)((uint32_t)tv + (uint32_t)tn - q2);
                    /* to_event: (Any, Nil, Value) codes of the key's vote type */
                    const bool pc = (K & 1u) != 0u;
                    const uint32_t eA = pc ? AGNES_CODE_PRECOMMIT_ANY : AGNES_CODE_POLKA_ANY;
                    const uint32_t eN = pc ? AGNES_CODE_NONE : AGNES_CODE_POLKA_NIL;
                    const uint32_t eV = pc ? AGNES_CODE_PRECOMMIT_VALUE : AGNES_CODE_POLKA_VALUE;
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s) {
                        const bool qv = (int32_t)av[s] > tv, qn = (int32_t)an[s] > tn,
                                   qa = (int32_t)(av[s] + an[s]) > ta;
                        uint32_t e = (in[s] && qa) ? eA : 0u;
                        e = (in[s] && qn) ? eN : e;
                        e = (in[s] && qv) ? eV : e;
                        c4 |= e << (8u * s);
                    }
                    if (lastc) { /* the last segment's weights so far (lane 63 is in it) */
                        const uint32_t lv = rdl(iv, 63u) - rdl(bv, 63u), ln = rdl(inn, 63u) - rdl(bn, 63u);
                        if (lane == 0u) {
                            B[K] += lv;
                            B[2u * R + K] += ln;
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                }
                if (lastc) cpar ^= 1u;

                /* ---- K4: State::apply(v.round, event) in stream order ---- */
                uint32_t msg = 0;
                if (SM) {
                    const uint32_t smw = rec.w;
                    const uint32_t step = (smw >> 16) & 0xFFu, eq8 = smw & 0x1FFu;
                    uint32_t smask = __builtin_amdgcn_perm(SM_HI, SM_LO, (step < 7u ? step : 7u) * 0x01010101u);
                    if (eq8 > 255u) smask &= X_C * 0x01010101u; /* no vote round equals State.round */
                    /* roles of each vote's event; the eqr-guarded ones only at State.round */
                    const uint32_t eqb = (zero_marks(r4 ^ (eq8 * 0x01010101u)) >> 7) * (X_P1 | X_TP | X_TC | X_PV);
                    const uint32_t x = __builtin_amdgcn_perm(XT_HI, XT_LO, c4 & 0x07070707u) & smask &
                                       (eqb | (X_C * 0x01010101u));
                    if (ballot(x != 0u)) {
                        const uint64_t MC = ballot((x & (X_C * 0x01010101u)) != 0u);
                        const uint64_t MP = ballot((x & (X_P1 * 0x01010101u)) != 0u);
                        /* lanes before mine in my segment: [ss, lane) */
                        const uint64_t Bm = (1ull << lane) - (1ull << ss);
                        const bool cbf = (MC & Bm) != 0ull, pbf = (MP & Bm) != 0ull;
                        const uint32_t cb = x & (X_C * 0x01010101u);
                        const uint32_t lcb = cb & (0u - cb);
                        const uint32_t lc = cbf ? 0u : lcb;           /* the commit (:211), bit 1 of its byte */
                        const uint32_t alive = cbf ? 0u : lcb - 1u;   /* bits below the commit  */
                        const uint32_t p1b = pbf ? 0u : (x & (X_P1 * 0x01010101u) & alive);
                        const uint32_t lp = p1b & (0u - p1b); /* P1 (:197-198), bit 0 of its byte */
                        const uint32_t pre = alive & (lp - 1u);
                        /* TimeoutPrevote before P1 in Prevote (:196), TimeoutPrecommit before the commit (:208) */
                        msg = (((x & (pbf ? 0u : pre)) & (X_TP * 0x01010101u)) | (x & alive & (X_TC * 0x01010101u)))
                              << 2;
                        /* P1: precommit(r, v) or precommit(r, None) (:197-198); C: Decision */
                        const uint32_t pvb = (x >> 4) & lp;
                        msg |= ((lp * 3u) + pvb) << AGNES_CODE_MSG_SHIFT;
                        msg |= ((lc >> 1) * AGNES_VMSG_DECISION) << AGNES_CODE_MSG_SHIFT;
                        /* the State: step, locked (P1 a PolkaValue), the decision */
                        if (ballot((lp | lc) != 0u)) {
                            uint32_t* const wk = itab + 8u * kln;
                            if (lp) {
                                const uint32_t ps = (uint32_t)__builtin_ctz(lp) >> 3;
                                atomicMax(wk + R_SMW, eq8 | ((uint32_t)AGNES_STEP_PRECOMMIT << 16));
                                if (pvb) {
                                    wk[R_LOCK] = sel4(value, ps);
                                    atomicOr(wk + R_FLAGS, F_LOCK);
                                }
                            }
                            if (lc) {
                                const uint32_t cs = (uint32_t)__builtin_ctz(lc) >> 3;
                                atomicMax(wk + R_SMW, eq8 | ((uint32_t)AGNES_STEP_COMMIT << 16));
                                wk[R_DEC] = sel4(value, cs);
                                atomicOr(wk + R_FLAGS, F_DEC | (byte_of(r4, cs) << 8));
                            }
                        }
                        /* valid (:198, :202): the PolkaValues at State.round while in Precommit
                         * (from P1 on) before the commit; its value is the last non-nil one's */
                        const bool inpc = step == AGNES_STEP_PRECOMMIT || pbf;
                        const uint32_t cand = x & alive & (X_PV * 0x01010101u) & (inpc ? 0xFFFFFFFFu : ~(lp - 1u));
                        if (ballot(cand != 0u)) {
                            uint32_t vnn = cand;
#pragma unroll
                            for (uint32_t s = 0; s < VPL; ++s) vnn &= nil[s] ? ~(0xFFu << (8u * s)) : 0xFFFFFFFFu;
                            const uint64_t MV = ballot(vnn != 0u);
                            /* lanes after mine in my segment */
                            const uint64_t le = lane == 63u ? ~0ull : ((2ull << lane) - 1ull);
                            const uint64_t nsb = BL & ~le;
                            const uint64_t after = (nsb ? (nsb & (0ull - nsb)) - 1ull : ~0ull) & ~le;
                            if (vnn && !(MV & after)) {
                                uint32_t* const wk = itab + 8u * kln;
                                wk[R_VALID] = sel4(value, (31u - (uint32_t)__builtin_clz(vnn)) >> 3);
                                atomicOr(wk + R_FLAGS, F_VALID);
                            }
                        }
                    }
                }

                /* codes (deferred) */
                dc_code = c4 | msg;
                dc_pos = posb;
                dc_at = c;
                __builtin_amdgcn_wave_barrier();
            }
        }
        /* batch end: the shadows into the staged States, the States out, then the next batch */
        if (SM && m) {
            if (smf) dma_wait(); /* no chunk ran: the staged States are still in flight */
            if (!smf && lane < m) {
                const uint32_t* const rk = itab + 8u * lane;
                const uint32_t f = rk[R_FLAGS];
                uint32_t* const sp = reinterpret_cast<uint32_t*>(sb + 64u * lane);
                uint32_t fl = (sp[13] & ~0xFFu) | ((rk[R_SMW] >> 16) & 0xFFu);
                if (f & F_LOCK) { sp[4] = sp[2]; sp[5] = sp[3]; sp[10] = rk[R_LOCK]; fl |= 1u << 8; }
                if (f & F_VALID) { sp[6] = sp[2]; sp[7] = sp[3]; sp[11] = rk[R_VALID]; fl |= 1u << 16; }
                if (f & F_DEC) { sp[8] = (f >> 8) & 0xFFu; sp[9] = 0u; sp[12] = rk[R_DEC]; fl |= 1u << 24; }
                sp[13] = fl;
            }
            __builtin_amdgcn_wave_barrier();
            if (lane < 4u * m) {
                const uint4 v = *reinterpret_cast<const uint4*>(sb + o16);
                reinterpret_cast<uint4*>(a.states + H.s0)[lane] = v;
            }
        }
        if (N.s0 >= N.e0) break;
        if (!N.ready) hdr2(N);
        H = N;
        dma_states(H);
        range_of(rdl(tq, 0u), N.s0, N.e0); /* the batch after, grabbed one batch ago */
        tq += 1u;
        hdr1(N);
    }
    flush();
    const uint32_t nb = rdl(scan(bad), 63u);
    if (lane == 0 && nb) add_invalid(a.n_invalid, (unsigned long long)nb);
}

} // namespace sweep
} // namespace agnes

/* ------------------------------------------------------------------ */
/* launcher                                                            */

bool agnes_sweep_supported(const agnes_tally_args* a) {
    /* keys round * 2 + type < 31: one bit each in a u32; the u64 domain (flow<W64>)
     * without record counts (its walk list goes to the i64 LIST kernel) */
    return a->max_rounds <= 15u && (!a->w64 || a->ev_counts == nullptr);
}

template <bool SM>
static hipError_t launch_sweep_k(const agnes_tally_args* a, int num_cus, hipStream_t st) {
    const uint32_t n = a->vb.n_instances;
    if (n == 0) return hipSuccess;
    using agnes::sweep::sweep;
    const void* fns[2] = {reinterpret_cast<const void*>(&sweep<false, SM>),
                          reinterpret_cast<const void*>(&sweep<true, SM>)};
    const uint32_t lpw = agnes::sweep::lds_bytes(SM, a->max_rounds);
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
    /* one block per CU (the walk list is a fallback, usually empty) */
    uint64_t blocks = ((uint64_t)n + 4u * AGNES_WAVES_PER_BLOCK - 1u) / (4u * AGNES_WAVES_PER_BLOCK);
    const uint64_t cap = ncu;
    if (blocks > cap) blocks = cap;
    if (blocks == 0) blocks = 1;
    if (o->pc)
        hipLaunchKernelGGL((sweep<true, SM>), dim3((uint32_t)blocks), dim3(256), (size_t)lds, st, b, lpw);
    else
        hipLaunchKernelGGL((sweep<false, SM>), dim3((uint32_t)blocks), dim3(256), (size_t)lds, st, b, lpw);
    return hipGetLastError();
}

hipError_t agnes_launch_sweep(const agnes_tally_args* a, int num_cus, hipStream_t st) {
    const bool sm = (a->flags & AGNES_FLAG_STATE_MACHINE) != 0 && a->states != nullptr;
    if (!agnes_flow_supported(a)) return hipErrorInvalidValue; /* max_rounds <= 15 always fits */
    hipError_t e;
    if (agnes_flow_rg(a)) {
        /* the streams: flow_prep's gate picks ONE of the two kernels -- the aligned one when
         * every instance offset is a multiple of 4, else the one that also walks the
         * unaligned streams; every other batch to the walk list */
        {
            AgnesKt kt("flow_prep", st);
            e = agnes_launch_flow_prep(a, st);
        }
        if (e != hipSuccess) return e;
        agnes_tally_args b = *a;
        b.gate = 1u;
        {
            AgnesKt kt("flow", st);
            e = agnes_launch_flow(&b, num_cus, st, false);
        }
        if (e != hipSuccess) return e;
        b.gate = 2u;
        {
            AgnesKt kt("flow_ragged", st);
            e = agnes_launch_flow(&b, num_cus, st, true);
        }
    } else { /* the streams whose offsets are multiples of 4; every other batch to the walk list */
        AgnesKt kt("flow", st);
        e = agnes_launch_flow(a, num_cus, st, false);
    }
    if (e != hipSuccess) return e;
    AgnesKt kt("sweep_walk", st);
    return sm ? launch_sweep_k<true>(a, num_cus, st) : launch_sweep_k<false>(a, num_cus, st);
}
