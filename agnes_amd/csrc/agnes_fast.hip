/*
 * agnes_fast.hip — the u32 fast-path tally kernel (K1-K4 fused), register-lean.
 *
 * Same decomposition as the general kernel (agnes_kernels.hip): one wave64 owns a
 * contiguous range of instances and walks each instance's votes in 256-vote
 * chunks, lane l holding votes 4l..4l+3 of the chunk (16-B column loads).  It runs
 * every instance whose sums provably stay below 2^31 (non-negative powers,
 * len * maxpow < 2^31) and hands every other one to the i64 LIST kernel.  What
 * differs is how it spends registers, so that 8 waves fit on a SIMD:
 *
 *   - no software prefetch: latency is hidden by occupancy, not by a second set
 *     of vote registers;
 *   - per-set constants come through the scalar cache, the instance header and
 *     its State through one VGPR (lane-distributed), prefetched one instance ahead;
 *   - quorum as a signed compare of the lane-local prefix against a per-lane
 *     threshold (q2 - carry - exclusive wave prefix): no per-vote sums;
 *   - K4 (State::apply for vote events, state_machine.rs:196-211) is table driven:
 *     the State seen by a vote event reduces to a 16-entry change mask and a
 *     16-entry message table indexed by (event, vote round == State.round), so a
 *     pass over the chunk is two bit-field extracts per vote; a state-changing
 *     vote is applied on the scalar path straight into the State's lanes.
 *
 * Thresh::Value payloads (round_votes.rs:53, the last value written) are never
 * propagated per vote.  The State needs a payload only at a state change, and in
 * this domain (non-negative weights, executors fresh at the batch start) a
 * PolkaValue from a nil vote can change nothing that the non-nil vote before it
 * in the same bucket did not already set (that vote saw the same value weight,
 * so the same PolkaValue, in the same step or an earlier one); the rare changing
 * nil vote (a PrecommitValue, or a PolkaValue after a round skip) looks its
 * payload up backwards in the instance's stream.
 */

#include <type_traits>

#include "agnes_fast.h"

namespace agnes {
namespace fast {

__host__ __device__ inline void layout(uint32_t mode, bool skip, bool pf, uint32_t R, uint32_t nv,
                                       uint32_t* o_fv, uint32_t* o_fs, uint32_t* o_pf, uint32_t* total,
                                       bool w64 = false) {
    uint32_t o = (uint32_t)align16((w64 ? 40ull : 20ull) * R); /* vw[2R] vn[2R] skw[R] (u32, or u64 sums) */
    *o_fv = o;
    if (mode == AGNES_MODE_DEDUP) o = (uint32_t)align16(o + 8ull * R * nv);
    *o_fs = o;
    if (skip) o = (uint32_t)align16(o + 4ull * R * nv);
    *o_pf = o;
    if (pf) o += PF_BYTES;
    *total = o;
}

/* uniform facts of the instance being tallied */
struct Inst {
    uint64_t beg, end;
    uint32_t i, pbase, q2, q1, ep, set_ok;
};

/* One chunk of the instance, loaded and validated: lane l = votes c+4l .. c+4l+3. */
struct Chunk {
    uint32_t value[VPL];
    uint32_t key[VPL]; /* round * 2 + type of an accepted vote; 0xFFFFFFFF otherwise */
    uint32_t r4;       /* vote rounds, byte s = vote s */
    uint32_t pos;      /* bit s: vote s belongs to the instance (position inside [beg, end)) */
    uint32_t ok;       /* bit s: ... and passes validation */
};

__device__ __forceinline__ uint32_t uni(uint32_t x) { return rfl(x); }
__device__ __forceinline__ uint64_t uni(uint64_t x) { return rfl64(x); }

/* W64: the u64 domain (agnes_fast.h defer_si): the same kernel with u64 sums, weights
 * gathered from the i64 power table (no u32 LDS copy: PC is false) */
template <uint32_t MODE, bool SKIP, bool SM, bool PC, bool PF, bool W64>
__global__ __launch_bounds__(256) void tally_fast(agnes_tally_args a, uint32_t lds_per_wave) {
    static_assert(!(PC && W64), "the LDS power table holds u32 powers");
    using Acc = typename std::conditional<W64, uint64_t, uint32_t>::type;  /* running sums */
    using SAcc = typename std::conditional<W64, int64_t, int32_t>::type;   /* thresholds   */
    const uint32_t lane = lane_id();
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint32_t R = a.max_rounds;
    const uint32_t nv = a.n_vals;
    const uint32_t ns = a.n_sets;
    const uint32_t n = a.vb.n_instances;
    const uint64_t NV = a.vb.n_votes;
    const uint32_t Wn = gridDim.x * AGNES_WAVES_PER_BLOCK;
    const uint32_t gw = blockIdx.x * AGNES_WAVES_PER_BLOCK + wave;

    /* block-shared u32 power table (launcher-staged only when it costs no occupancy) */
    if (PC) {
        uint32_t* pc = reinterpret_cast<uint32_t*>(agnes_smem);
        const uint32_t np = ns * nv;
        for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) pc[k] = a.power32[k];
        __syncthreads();
    }
    /* Work queue: batches of BQ consecutive instances handed out by qn counters
     * (counter k = blockIdx % qn owns batches k, k + qn, ...).  Dynamic, so neither
     * the number of co-resident waves nor the instances' lengths unbalance the
     * grid; many counters, because same-address device atomics serialize
     * (~100 ns each on MI355X). */
    const uint32_t qn = gridDim.x < QN ? gridDim.x : QN; /* every counter has a block */
    const uint32_t qk = blockIdx.x % qn;
    uint32_t* const ctr = a.list_count + 1u + qk;
    auto range_of = [&](uint32_t t, uint32_t& s0, uint32_t& e0) {
        const uint64_t b0 = ((uint64_t)t * qn + qk) * BQ;
        s0 = b0 < n ? (uint32_t)b0 : n;
        e0 = b0 + BQ < n ? (uint32_t)(b0 + BQ) : n;
    };
    uint32_t q, qe, nS, nE;
    {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(ctr, 2u);
        t = rdl(t, 0u);
        range_of(t, q, qe);
        range_of(t + 1u, nS, nE);
    }
    if (q >= qe) return;
    uint32_t tq = 0; /* lane 0: slot of the batch after [nS, nE) (atomic in flight) */
    if (lane == 0) tq = atomicAdd(ctr, 1u);
    (void)Wn;
    (void)gw;

    uint32_t o_fv, o_fs, o_pf, o_tot;
    layout(MODE, SKIP, PF, R, nv, &o_fv, &o_fs, &o_pf, &o_tot, W64);
    unsigned char* base = agnes_smem + a.power_cache + wave * lds_per_wave;
    Acc* vw = reinterpret_cast<Acc*>(base); /* [2R] value weight carried across chunks */
    Acc* vn = vw + 2u * R;                  /* [2R] nil weight                       */
    Acc* skw = vn + 2u * R;                 /* [R]  RoundSkip weight                 */
    uint32_t* first_v = reinterpret_cast<uint32_t*>(base + o_fv);
    uint32_t* first_s = reinterpret_cast<uint32_t*>(base + o_fs);
    unsigned char* const pfb = base + o_pf;
    uint64_t pf_at = ~0ull; /* chunk held (or in flight) in pfb */
    constexpr bool TABLES = MODE == AGNES_MODE_DEDUP || SKIP;
    if (MODE == AGNES_MODE_DEDUP) fill_u32(first_v, 2ull * R * nv, 0u, lane);
    if (SKIP) fill_u32(first_s, (uint64_t)R * nv, 0u, lane);
    const uint32_t lb = a.epoch_shift;
    const uint32_t lmask = (1u << lb) - 1u;
    const uint32_t emax = lb >= 31u ? 1u : ((1u << (32u - lb)) - 1u);
    uint32_t ep = 0;
    uint32_t bad = 0;

    /* header of instance k over lanes: 0..3 offsets[k], offsets[k+1]; 4 its set;
     * SL..SL+13 its State */
    auto load_hdr = [&](uint32_t k) -> uint32_t {
        uint32_t h = 0;
        if (lane < 4u) h = reinterpret_cast<const uint32_t*>(a.vb.offsets + k)[lane];
        else if (lane == 4u) h = a.vb.instance_set ? a.vb.instance_set[k] : (ns ? k % ns : 0u);
        else if (SM && lane >= SL && lane < SL + 14u) h = reinterpret_cast<const uint32_t*>(&a.states[k])[lane - SL];
        return h;
    };

    /* load + validate chunk c of instance I (inst == i, round < R, type <= 1,
     * validator in the set; round_votes.rs has no invalid votes, these are the
     * boundary's checks) and, for DEDUP, its first-vote acceptance is left to the caller */
    auto load_chunk = [&](const Inst& I, uint64_t c, Chunk& x, uint32_t (&val)[VPL], uint32_t& t4) {
        const uint64_t j = c + 4u * lane;
        uint32_t inst[VPL];
        if (PF && pf_at == c) { /* prefetched by LDS-DMA */
            dma_wait();
            const uint4 ia = *reinterpret_cast<const uint4*>(pfb + PF_INST + 16u * lane);
            const uint4 va = *reinterpret_cast<const uint4*>(pfb + PF_VALUE + 16u * lane);
            const uint4 da = *reinterpret_cast<const uint4*>(pfb + PF_VAL + 16u * lane);
            inst[0] = ia.x; inst[1] = ia.y; inst[2] = ia.z; inst[3] = ia.w;
            x.value[0] = va.x; x.value[1] = va.y; x.value[2] = va.z; x.value[3] = va.w;
            val[0] = da.x; val[1] = da.y; val[2] = da.z; val[3] = da.w;
            x.r4 = *reinterpret_cast<const uint32_t*>(pfb + PF_ROUND + 4u * lane);
            t4 = *reinterpret_cast<const uint32_t*>(pfb + PF_TYPE + 4u * lane);
        } else if (c + CHUNK <= NV) {
            const uint4 ia = *reinterpret_cast<const uint4*>(a.vb.instance + j);
            const uint4 va = *reinterpret_cast<const uint4*>(a.vb.value + j);
            const uint4 da = *reinterpret_cast<const uint4*>(a.vb.validator + j);
            inst[0] = ia.x; inst[1] = ia.y; inst[2] = ia.z; inst[3] = ia.w;
            x.value[0] = va.x; x.value[1] = va.y; x.value[2] = va.z; x.value[3] = va.w;
            val[0] = da.x; val[1] = da.y; val[2] = da.z; val[3] = da.w;
            x.r4 = *reinterpret_cast<const uint32_t*>(a.vb.round + j);
            t4 = *reinterpret_cast<const uint32_t*>(a.vb.type + j);
        } else {
            x.r4 = t4 = 0;
#pragma unroll
            for (uint32_t s = 0; s < VPL; ++s) {
                const bool in = j + s < NV;
                inst[s] = in ? a.vb.instance[j + s] : 0u;
                x.value[s] = in ? a.vb.value[j + s] : 0u;
                val[s] = in ? a.vb.validator[j + s] : 0u;
                x.r4 |= (in ? (uint32_t)a.vb.round[j + s] : 0u) << (8u * s);
                t4 |= (in ? (uint32_t)a.vb.type[j + s] : 0u) << (8u * s);
            }
        }
        const uint32_t lo = c < I.beg ? (uint32_t)(I.beg - c) : 0u;
        const uint32_t hi = I.end - c < CHUNK ? (uint32_t)(I.end - c) : CHUNK;
        const uint32_t p0 = 4u * lane;
        x.pos = x.ok = 0;
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s) {
            const uint32_t r = byte_of(x.r4, s), t = byte_of(t4, s);
            const uint32_t in = (uint32_t)(p0 + s >= lo) & (uint32_t)(p0 + s < hi);
            const uint32_t ok = in & (uint32_t)(inst[s] == I.i) & (uint32_t)(r < R) & (uint32_t)(t <= 1u) &
                                (uint32_t)(val[s] < nv) & I.set_ok;
            x.pos |= in << s;
            x.ok |= ok << s;
            x.key[s] = ok ? r * 2u + t : 0xFFFFFFFFu;
        }
    };

    /* the wave's instance stream: [q, qe) then [nS, nE); succ1/succ2 = the next two */
    auto succ1 = [&]() -> uint32_t { return q + 1u < qe ? q + 1u : (nS < nE ? nS : NONE); };
    auto succ2 = [&]() -> uint32_t {
        if (q + 2u < qe) return q + 2u;
        if (q + 1u < qe) return nS < nE ? nS : NONE;
        return nS + 1u < nE ? nS + 1u : NONE;
    };
    /* headers two deep: hq (instance q, arrived), hn (its successor, in flight) */
    uint32_t hq = load_hdr(q);
    uint32_t hn = succ1() != NONE ? load_hdr(succ1()) : 0u;
    /* stores deferred until the next chunk's gather is issued (vmcnt retires in
     * issue order: a store ahead of a load delays every wait on that load) */
    uint64_t dc_at = ~0ull;
    uint32_t dc_code = 0, dc_pos = 0;
    uint32_t ds_i = NONE, ds_word = 0;
    auto flush = [&]() {
        if (dc_at != ~0ull) {
            const uint64_t j = dc_at + 4u * lane;
            if (dc_pos == 0xFu) {
                if (AGNES_FAST_NT) __builtin_nontemporal_store(dc_code, reinterpret_cast<uint32_t*>(a.codes + j));
                else *reinterpret_cast<uint32_t*>(a.codes + j) = dc_code;
            } else {
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s)
                    if ((dc_pos >> s) & 1u) a.codes[j + s] = (uint8_t)(dc_code >> (8u * s));
            }
            dc_at = ~0ull;
        }
        if (SM && ds_i != NONE) {
            if (lane >= SL && lane < SL + 14u) reinterpret_cast<uint32_t*>(&a.states[ds_i])[lane - SL] = ds_word;
            ds_i = NONE;
        }
    };
    uint32_t hnn = 0;
    bool hnn_issued = false;
    auto issue_hnn = [&]() {
        if (!hnn_issued) {
            const uint32_t k = succ2();
            hnn = k != NONE ? load_hdr(k) : 0u;
            hnn_issued = true;
        }
    };

    for (;;) {
        const uint32_t h = hq;
        hnn_issued = false;
        Inst I;
        I.i = q;
        bool run = true;
        uint64_t b = ((uint64_t)rdl(h, 1u) << 32) | rdl(h, 0u);
        uint64_t e = ((uint64_t)rdl(h, 3u) << 32) | rdl(h, 2u);
        b = b < NV ? b : NV;
        e = e < NV ? e : NV;
        I.beg = b;
        I.end = e > b ? e : b;
        const uint32_t set = rdl(h, 4u);
        I.set_ok = set < ns;
        I.pbase = set * nv;
        I.q2 = I.q1 = 0;
        Acc Q2 = 0, Q1 = 0; /* the quorum / +1/3 thresholds in the sums' width */
        const uint64_t len = I.end - I.beg;
        if (I.set_ok) {
            const agnes_set_info si = a.sets[set];
            /* sums provably < 2^31 (u32 arithmetic; W64: < 2^61), else the i64 LIST kernel */
            if (defer_si(si, len, W64)) {
                if (lane == 0) a.list[atomicAdd(a.list_count, 1u)] = I.i;
                run = false;
            }
            if (W64) {
                Q2 = (Acc)si.q2w;
                Q1 = (Acc)si.q1w;
            } else {
                /* sums < 2^31: a threshold >= 2^31 - 1 is never crossed, clamp it so the
                 * per-lane thresholds below stay in int32 range */
                I.q2 = si.q2 < 0x7FFFFFFFu ? si.q2 : 0x7FFFFFFFu;
                I.q1 = si.q1 < 0x7FFFFFFFu ? si.q1 : 0x7FFFFFFFu;
                Q2 = (Acc)I.q2;
                Q1 = (Acc)I.q1;
            }
        }
        if (len == 0) run = false;
        uint32_t evn = 0; /* (a.ev_counts: agnes_tally_events) the lane's records of this instance */
        if (run) {
        if (TABLES) {
            if (++ep > emax) { /* epoch space used up: recycle the tables */
                if (MODE == AGNES_MODE_DEDUP) fill_u32(first_v, 2ull * R * nv, 0u, lane);
                if (SKIP) fill_u32(first_s, (uint64_t)R * nv, 0u, lane);
                ep = 1;
            }
        }
        I.ep = ep;
        const uint64_t c0 = I.beg & ~3ull;
        const bool multi = I.end - c0 > CHUNK;
        if (multi) { /* RoundVotes::new per round (round_votes.rs:83-90) */
            for (uint32_t k = lane; k < 5u * R; k += 64) vw[k] = 0;
            __builtin_amdgcn_wave_barrier();
        }
        uint32_t stv = h;
        View V;
        bool sm_live = false, sm_changed = false;
        if (SM) {
            V = view_of(stv);
            sm_live = (V.flags & 0xFFu) != AGNES_STEP_COMMIT; /* :205 */
        }

        for (uint64_t c = c0; c < I.end; c += CHUNK) {
            Chunk x;
            uint32_t val[VPL], t4;
            /* raised priority while this chunk's loads, the gather and the next chunk's
             * requests go out (same-box A/B: C4 tally_fast 0.797 -> 0.779 ms) */
            __builtin_amdgcn_s_setprio(1);
            load_chunk(I, c, x, val, t4);
            const uint32_t p0 = 4u * lane;
            /* K1: w = power[set][validator] (consensus_executor.rs:62-63 -> validators.rs:7) */
            Acc w[VPL];
#pragma unroll
            for (uint32_t s = 0; s < VPL; ++s) {
                const uint32_t idx = I.pbase + (((x.ok >> s) & 1u) ? val[s] : 0u);
                if (W64) w[s] = (Acc)a.power[idx];
                else w[s] = PC ? reinterpret_cast<const uint32_t*>(agnes_smem)[idx] : a.power32[idx];
            }
            bad += __builtin_popcount(x.pos & ~x.ok);
            /* after the gather: the previous chunk's stores, the header two instances
             * ahead, and the next chunk (this instance's, or the next instance's first)
             * by LDS-DMA — all issued together, all retired by the next chunk's wait */
            flush();
            issue_hnn();
            if (PF) {
                uint64_t nc = c + CHUNK;
                bool has_next = true;
                if (nc >= I.end) {
                    has_next = succ1() != NONE;
                    if (has_next) {
                        const uint64_t nb = ((uint64_t)rdl(hn, 1u) << 32) | rdl(hn, 0u);
                        nc = (nb < NV ? nb : NV) & ~3ull;
                    }
                }
                /* a full chunk inside the columns only (nc <= NV here, no wrap) */
                if (has_next && nc + CHUNK <= NV) {
                    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): this chunk's LDS reads are done */
                    const uint64_t jn = nc + 4u * lane;
                    glds16(a.vb.instance + jn, pfb + PF_INST);
                    glds16(a.vb.value + jn, pfb + PF_VALUE);
                    glds16(a.vb.validator + jn, pfb + PF_VAL);
                    glds4(a.vb.round + jn, pfb + PF_ROUND);
                    glds4(a.vb.type + jn, pfb + PF_TYPE);
                    pf_at = nc;
                } else {
                    pf_at = ~0ull;
                }
            }
            __builtin_amdgcn_s_setprio(0);

            /* first-vote tables: atomic max of (epoch << lb | LMASK - local index), so
             * the earliest vote of the instance wins (DEDUP: per (round, type,
             * validator); RoundSkip: per (round, validator)) */
            uint32_t acc = x.ok, sfirst = 0;
            if (TABLES) {
                const uint32_t loc0 = (uint32_t)(c - I.beg) + p0;
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s) {
                    if ((x.ok >> s) & 1u) {
                        const uint32_t enc = (I.ep << lb) | (lmask - (loc0 + s));
                        if (MODE == AGNES_MODE_DEDUP) atomicMax(&first_v[x.key[s] * nv + val[s]], enc);
                        if (SKIP) atomicMax(&first_s[(x.key[s] >> 1) * nv + val[s]], enc);
                    }
                }
                __builtin_amdgcn_wave_barrier();
                if (MODE == AGNES_MODE_DEDUP) acc = 0;
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s) {
                    if ((x.ok >> s) & 1u) {
                        const uint32_t enc = (I.ep << lb) | (lmask - (loc0 + s));
                        if (MODE == AGNES_MODE_DEDUP)
                            acc |= (uint32_t)(*(volatile uint32_t*)&first_v[x.key[s] * nv + val[s]] == enc) << s;
                        if (SKIP)
                            sfirst |= (uint32_t)(*(volatile uint32_t*)&first_s[(x.key[s] >> 1) * nv + val[s]] == enc) << s;
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }

            /* per-vote code: INVALID / REJECTED, else the tally event filled below */
            uint32_t code[VPL];
            Acc wv[VPL], wn[VPL];
#pragma unroll
            for (uint32_t s = 0; s < VPL; ++s) {
                const bool a_ = (acc >> s) & 1u;
                code[s] = !((x.ok >> s) & 1u) ? AGNES_CODE_INVALID : (a_ ? 0u : AGNES_CODE_REJECTED);
                if (!a_) x.key[s] = 0xFFFFFFFFu;
                const bool isnil = x.value[s] == AGNES_NIL;
                wv[s] = isnil ? (Acc)0 : w[s];
                wn[s] = isnil ? w[s] : (Acc)0;
            }
            const bool ld_carry = c != c0;
            const bool st_carry = c + CHUNK < I.end;

            /* K2+K3 per (round, type) bucket present: one stream-order scan of its value
             * and nil weights (VoteCount::add_vote, round_votes.rs:48-56) and, per vote,
             * is_quorum with precedence Value > Nil > Any > Init (:31-33, :58-66) and
             * to_event (vote_executor.rs:26-36) */
            uint32_t rem = acc;
            for (;;) {
                const uint64_t lm = ballot(rem != 0u);
                if (!lm) break;
                const uint32_t kl = (uint32_t)__builtin_ctzll(lm);
                const uint32_t ks = (uint32_t)__builtin_ctz(rdl(rem, kl));
                const uint32_t K = rdl(sel4(x.key, ks), kl);
                Acc av[VPL], an[VPL];
                uint32_t inb = 0;
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s) {
                    const bool in = x.key[s] == K;
                    inb |= (uint32_t)in << s;
                    av[s] = in ? wv[s] : (Acc)0;
                    an[s] = in ? wn[s] : (Acc)0;
                }
                rem &= ~inb;
                /* lane-local inclusive prefixes and one wave scan of the lane totals */
                av[1] += av[0]; av[2] += av[1]; av[3] += av[2];
                an[1] += an[0]; an[2] += an[1]; an[3] += an[2];
                const Acc iv = scan(av[3]), in_ = scan(an[3]);
                const Acc cv = ld_carry ? vw[K] : (Acc)0, cn = ld_carry ? vn[K] : (Acc)0;
                /* a quiet key: even the bucket's running sums after its last vote of the
                 * chunk stay at or below q2, so every vote of it is Init (code NONE, already
                 * in code[]) -- the common case for the few early next-round votes, and for a
                 * round's first chunk.  Uniform; the sums stay below 2^31 in this domain. */
                if (uni(cv + cn) + rdl(iv, 63u) + rdl(in_, 63u) > Q2) {
                /* sum > q2  <=>  lane-local prefix > q2 - carry - exclusive wave prefix */
                const SAcc tv = (SAcc)(Q2 - cv - (iv - av[3]));
                const SAcc tn = (SAcc)(Q2 - cn - (in_ - an[3]));
                const SAcc ta = (SAcc)(Q2 - cv - cn - (iv - av[3]) - (in_ - an[3]));
                if (K & 1u) { /* precommits: Value -> PrecommitValue, Nil -> None, Any -> PrecommitAny */
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s) {
                        const bool qv = (SAcc)av[s] > tv, qn = (SAcc)an[s] > tn,
                                   qa = (SAcc)(av[s] + an[s]) > ta;
                        const uint32_t ev = qv ? AGNES_CODE_PRECOMMIT_VALUE
                                          : (qn ? AGNES_CODE_NONE : (qa ? AGNES_CODE_PRECOMMIT_ANY : AGNES_CODE_NONE));
                        code[s] = ((inb >> s) & 1u) ? ev : code[s];
                    }
                } else { /* prevotes: PolkaValue / PolkaNil / PolkaAny */
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s) {
                        const bool qv = (SAcc)av[s] > tv, qn = (SAcc)an[s] > tn,
                                   qa = (SAcc)(av[s] + an[s]) > ta;
                        const uint32_t ev = qv ? AGNES_CODE_POLKA_VALUE
                                          : (qn ? AGNES_CODE_POLKA_NIL : (qa ? AGNES_CODE_POLKA_ANY : AGNES_CODE_NONE));
                        code[s] = ((inb >> s) & 1u) ? ev : code[s];
                    }
                }
                }
                if (st_carry && lane == 63u) {
                    vw[K] = cv + iv;
                    vn[K] = cn + in_;
                }
                __builtin_amdgcn_wave_barrier();
            }

            /* RoundSkip (+1/3 of the distinct validators voting in the vote's round,
             * extension): the same scan keyed by round over each validator's first vote */
            if (SKIP) {
                uint32_t rs = acc;
                for (;;) {
                    const uint64_t lm = ballot(rs != 0u);
                    if (!lm) break;
                    const uint32_t kl = (uint32_t)__builtin_ctzll(lm);
                    const uint32_t ks = (uint32_t)__builtin_ctz(rdl(rs, kl));
                    const uint32_t kr = rdl(sel4(x.key, ks), kl) >> 1;
                    Acc as[VPL];
                    uint32_t inb = 0;
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s) {
                        const bool in = (x.key[s] >> 1) == kr && ((rs >> s) & 1u);
                        inb |= (uint32_t)in << s;
                        as[s] = (in && ((sfirst >> s) & 1u)) ? w[s] : (Acc)0;
                    }
                    rs &= ~inb;
                    as[1] += as[0]; as[2] += as[1]; as[3] += as[2];
                    const Acc is = scan(as[3]);
                    const Acc cs = ld_carry ? skw[kr] : (Acc)0;
                    if (uni(cs) + rdl(is, 63u) > Q1) { /* else quiet: no vote of the round crosses +1/3 */
                        const SAcc ts = (SAcc)(Q1 - cs - (is - as[3]));
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s)
                            if (((inb >> s) & 1u) && (SAcc)as[s] > ts) code[s] |= AGNES_CODE_SKIP;
                    }
                    if (st_carry && lane == 63u) skw[kr] = cs + is;
                    __builtin_amdgcn_wave_barrier();
                }
            }

            /* K4: State::apply(v.round, event) in stream order (consensus_executor.rs:64-68) */
            if (SM && sm_live) {
                /* fresh copies: keep the compiler from carrying per-vote values derived
                 * before the slot loop (round bytes, nil tests) across it for this stage */
                asm volatile("" : "+v"(x.r4), "+v"(x.value[0]), "+v"(x.value[1]), "+v"(x.value[2]), "+v"(x.value[3]));
                uint32_t pend = 0;
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s)
                    pend |= (uint32_t)(((acc >> s) & 1u) && (code[s] & 0xFu) != 0u) << s;
                /* the payload of the changing vote (fl, fs) at chunk position `first`:
                 * its own value, or the last value written before it in its bucket
                 * (round_votes.rs:53) for a nil vote */
                auto label_at = [&](uint32_t fl, uint32_t fs, uint32_t first) -> uint32_t {
                    const uint32_t fv = rdl(sel4(x.value, fs), fl);
                    if (fv != AGNES_NIL) return fv;
                    const uint32_t K = rdl(sel4(x.key, fs), fl);
                    uint32_t cand = 0;
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s)
                        cand |= (uint32_t)(x.key[s] == K && x.value[s] != AGNES_NIL && p0 + s < first) << s;
                    const uint64_t cl = ballot(cand != 0u);
                    if (cl) {
                        const uint32_t hl = 63u - (uint32_t)__builtin_clzll(cl);
                        const uint32_t hs = 31u - (uint32_t)__builtin_clz(rdl(cand, hl));
                        return rdl(sel4(x.value, hs), hl);
                    }
                    /* earlier chunks of this instance, newest first: one vote per lane at
                     * a time (rare path, few registers) */
                    for (uint64_t pc = c; pc != c0;) {
                        pc -= CHUNK;
                        uint32_t hit = 0, hv = 0;
#pragma unroll 1
                        for (int s = (int)VPL - 1; s >= 0; --s) {
                            const uint64_t j = pc + p0 + (uint32_t)s;
                            if (!hit && j >= I.beg && j < I.end) {
                                /* opaque bases: keep this rare path's address arithmetic
                                 * from being hoisted into the chunk loop */
                                const uint8_t *br = a.vb.round, *bt = a.vb.type;
                                const uint32_t *bx = a.vb.validator, *bv = a.vb.value, *bi = a.vb.instance;
                                asm volatile("" : "+s"(br), "+s"(bt), "+s"(bx), "+s"(bv), "+s"(bi));
                                const uint32_t vr = br[j], vt = bt[j];
                                const uint32_t vx = bx[j], vv = bv[j];
                                bool ok = bi[j] == I.i && vr < R && vt <= 1u && vx < nv && vr * 2u + vt == K &&
                                          vv != AGNES_NIL;
                                if (MODE == AGNES_MODE_DEDUP && ok)
                                    ok = first_v[K * nv + vx] == ((I.ep << lb) | (lmask - (uint32_t)(j - I.beg)));
                                if (ok) {
                                    hit = 1;
                                    hv = vv;
                                }
                            }
                        }
                        const uint64_t hl = ballot(hit != 0u);
                        if (hl) return rdl(hv, 63u - (uint32_t)__builtin_clzll(hl));
                    }
                    return 0u; /* unreachable in the fast domain (a nil vote at value quorum
                                  always has a value vote before it in its bucket) */
                };
                /* apply the changing vote (fl, fs) on the scalar path; its message into its code */
                auto change_at = [&](uint32_t fl, uint32_t fs) {
                    const uint32_t fcode = rdl(sel4(code, fs), fl);
                    const uint32_t fr = byte_of(rdl(x.r4, fl), fs);
                    const uint32_t ev = fcode & 7u;
                    const uint32_t lab = (ev == AGNES_CODE_POLKA_VALUE || ev == AGNES_CODE_PRECOMMIT_VALUE)
                                             ? label_at(fl, fs, 4u * fl + fs) : 0u;
                    const uint32_t vm = apply_change(stv, V, fcode, fr, lab);
                    sm_changed = true;
                    if (lane == fl) {
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s)
                            if (s == fs) code[s] |= vm << AGNES_CODE_MSG_SHIFT;
                    }
                };
                if (!SKIP && ballot(pend != 0u)) {
                    /* The vote's round never moves State.round here, so eqr is fixed per vote
                     * and vote events drive a tiny automaton: Prevote --PolkaNil/PolkaValue at
                     * eqr--> Precommit --PolkaValue at eqr with another value--> Precommit
                     * (valid), any step --PrecommitValue--> Commit.  Every change is found as
                     * the first set bit of per-sub-vote ballots (lane l, vote s = position
                     * 4l + s) restricted to a position window; the non-changing messages are
                     * PolkaAny at eqr -> TimeoutPrevote before the State leaves Prevote (P1)
                     * and PrecommitAny at eqr -> TimeoutPrecommit before the commit (PC). */
                    /* event of vote s with the eqr bit (event | eqr << 3); 6/7 (invalid /
                     * rejected) match nothing below */
                    auto ev_of = [&](uint32_t s) -> uint32_t {
                        return (code[s] & 7u) | ((uint32_t)(byte_of(x.r4, s) == V.eq8) << 3);
                    };
                    /* one change per pass: the first PrecommitValue (commit), and before it
                     * the first vote that moves the current step (Prevote: PolkaNil /
                     * PolkaValue at eqr; Precommit: PolkaValue at eqr with another value) */
                    const bool prevote0 = (V.flags & 0xFFu) == AGNES_STEP_PREVOTE;
                    uint32_t P1 = prevote0 ? CHUNK : 0u, pc = CHUNK, lo = 0;
                    for (;;) {
                        const uint32_t step = V.flags & 0xFFu;
                        uint64_t b[VPL];
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s) {
                            const uint32_t ix = ev_of(s);
                            const bool pv = ix == (AGNES_CODE_POLKA_VALUE | 8u);
                            const bool mv = step == AGNES_STEP_PREVOTE
                                                ? (pv || ix == (AGNES_CODE_POLKA_NIL | 8u))
                                                : (step == AGNES_STEP_PRECOMMIT && pv &&
                                                   (!V.vsame || (x.value[s] != AGNES_NIL && x.value[s] != V.vval)));
                            b[s] = ballot(mv || (ix & 7u) == AGNES_CODE_PRECOMMIT_VALUE);
                        }
                        const uint32_t f = first_of(b, lo, CHUNK);
                        if (f >= CHUNK) break;
                        change_at(f >> 2, f & 3u);
                        if (step == AGNES_STEP_PREVOTE && P1 == CHUNK) P1 = f; /* left Prevote */
                        if ((V.flags & 0xFFu) == AGNES_STEP_COMMIT) { /* :211; :205 every later event: None */
                            pc = f;
                            sm_live = false;
                            break;
                        }
                        lo = f + 1u;
                    }
                    /* messages of the non-changing events */
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s) {
                        const uint32_t ix = ev_of(s);
                        const bool m1 = ix == (AGNES_CODE_POLKA_ANY | 8u) && ((win(s, 0u, P1) >> lane) & 1u);
                        const bool m2 = ix == (AGNES_CODE_PRECOMMIT_ANY | 8u) && ((win(s, 0u, pc) >> lane) & 1u);
                        code[s] |= (m1 ? AGNES_VMSG_TIMEOUT_PREVOTE : (m2 ? AGNES_VMSG_TIMEOUT_PRECOMMIT : 0u))
                                   << AGNES_CODE_MSG_SHIFT;
                    }
                } else if (SKIP && ballot(pend != 0u)) {
                    /* RoundSkip moves State.round, so eqr changes with the State: each pass
                     * classifies every pending vote against the current State (change mask and
                     * message table indexed by event | eqr << 3), assigns the messages of the
                     * votes before the first change and applies that change */
                    uint32_t idx[VPL];
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s)
                        idx[s] = (code[s] & 7u) | ((uint32_t)(byte_of(x.r4, s) == V.eq8) << 3);
                    for (;;) {
                        uint32_t chb = 0;
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s) {
                            uint32_t ch = (V.chg >> idx[s]) & 1u;
                            if (V.pvchk)
                                ch |= (uint32_t)(idx[s] == (AGNES_CODE_POLKA_VALUE | 8u)) &
                                      (uint32_t)(x.value[s] != V.vval) & (uint32_t)(x.value[s] != AGNES_NIL);
                            ch |= ((code[s] >> 3) & 1u) & (uint32_t)((int32_t)byte_of(x.r4, s) > V.rlt);
                            chb |= ch << s;
                        }
                        chb &= pend;
                        const uint64_t bk = ballot(chb != 0u);
                        uint32_t first = CHUNK, fl = 0, fs = 0;
                        if (bk) {
                            fl = (uint32_t)__builtin_ctzll(bk);
                            fs = (uint32_t)__builtin_ctz(rdl(chb, fl));
                            first = 4u * fl + fs;
                        }
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s) {
                            if (((pend >> s) & 1u) && p0 + s < first)
                                code[s] |= ((V.mt >> (2u * idx[s])) & 3u) << AGNES_CODE_MSG_SHIFT;
                            if (p0 + s <= first) pend &= ~(1u << s);
                        }
                        if (!bk) break;
                        change_at(fl, fs);
                        if ((V.flags & 0xFFu) == AGNES_STEP_COMMIT) { /* :205 every later event: None */
                            sm_live = false;
                            break;
                        }
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s)
                            idx[s] = (code[s] & 7u) | ((uint32_t)(byte_of(x.r4, s) == V.eq8) << 3);
                    }
                }
            }

            /* codes (deferred): one 4-B store when all 4 votes belong to the instance */
            dc_code = code[0] | (code[1] << 8) | (code[2] << 16) | (code[3] << 24);
            dc_pos = x.pos;
            dc_at = c;
            if (a.ev_counts) { /* records: an event 1..5, plus its RoundSkip bit; none for INVALID / REJECTED */
                const uint32_t e = dc_code & 0x07070707u;
                const uint32_t ok = ~(e + 0x7A7A7A7Au) & ((dc_pos * 0x00204081u) & 0x01010101u) << 7;
                evn += (uint32_t)__builtin_popcount((e + 0x7F7F7F7Fu) & ok) +
                       (uint32_t)__builtin_popcount((dc_code << 4) & ok);
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (SM && sm_changed) { /* State back (deferred) */
            ds_i = I.i;
            ds_word = stv;
        }
        } /* run */
        if (a.ev_counts) { /* the instance's record count (a deferred one's is the count pass's) */
            const uint32_t tot = rdl(scan(evn), 63u);
            if (lane == 0) a.ev_counts[I.i] = tot;
        }
        issue_hnn();
        /* advance the stream */
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
        hn = hnn;
    }
    flush();
    const uint32_t nb = rdl(scan(bad), 63u);
    if (lane == 0 && nb) add_invalid(a.n_invalid, (unsigned long long)nb);
}

} // namespace fast
} // namespace agnes

int64_t agnes_fast_lds_per_wave(uint32_t mode, uint32_t flags, uint32_t max_rounds, uint32_t n_vals) {
    uint32_t fv, fs, pf, tot;
    agnes::fast::layout(mode, (flags & AGNES_FLAG_ROUND_SKIP) != 0, true, max_rounds, n_vals, &fv, &fs, &pf,
                        &tot);
    return (int64_t)tot;
}

static uint32_t fast_lds(uint32_t mode, uint32_t flags, bool pf, uint32_t R, uint32_t nv, bool w64 = false) {
    uint32_t fv, fs, o_pf, tot;
    agnes::fast::layout(mode, (flags & AGNES_FLAG_ROUND_SKIP) != 0, pf, R, nv, &fv, &fs, &o_pf, &tot, w64);
    return tot;
}

/* variant v = PC | PF << 1 of the kernel (W64: no PC variant; v & 1 is never chosen) */
template <uint32_t MODE, bool SKIP, bool SM, bool W64, int V>
static const void* fast_fn() {
    return reinterpret_cast<const void*>(&agnes::fast::tally_fast<MODE, SKIP, SM, (V & 1) != 0 && !W64, (V & 2) != 0, W64>);
}

template <uint32_t MODE, bool SKIP, bool SM, bool W64>
static hipError_t launch_fast_k(const agnes_tally_args* a, int num_cus, hipStream_t st) {
    const uint32_t n = a->vb.n_instances;
    if (n == 0) return hipSuccess;
    using agnes::fast::tally_fast;
    const void* fns[4] = {fast_fn<MODE, SKIP, SM, W64, 0>(), fast_fn<MODE, SKIP, SM, W64, 1>(),
                          fast_fn<MODE, SKIP, SM, W64, 2>(), fast_fn<MODE, SKIP, SM, W64, 3>()};
    const uint64_t pcb = agnes::align16(4ull * a->n_sets * a->n_vals);
    /* variant v = PC | PF << 1: blocks per CU from the occupancy query; prefer the
     * LDS-DMA prefetch, then the LDS power table, each only where it costs no
     * occupancy.  Cached per (kernel, LDS shape). */
    struct Occ { const void* fn; uint32_t R, nv, flags; uint64_t pcb; int per_cu; int v; };
    static thread_local Occ occ[8];
    static thread_local unsigned occ_next = 0;
    Occ* o = nullptr;
    for (auto& c : occ)
        if (c.fn == fns[0] && c.R == a->max_rounds && c.nv == a->n_vals && c.flags == a->flags && c.pcb == pcb)
            o = &c;
    auto lds_of = [&](int v) -> uint64_t {
        return (uint64_t)fast_lds(MODE, a->flags, (v & 2) != 0, a->max_rounds, a->n_vals, W64) * AGNES_WAVES_PER_BLOCK +
               ((v & 1) ? pcb : 0u);
    };
    if (!o) {
        auto per_cu = [&](int v) -> int {
            const uint64_t lds = lds_of(v);
            if (lds > 160u * 1024u || ((v & 1) && (W64 || pcb > 32u * 1024u))) return 0;
            if (lds > 48u * 1024u &&
                hipFuncSetAttribute(fns[v], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
                return 0;
            int k = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&k, fns[v], 256, (size_t)lds) != hipSuccess) k = 0;
            return k;
        };
        o = &occ[occ_next++ % 8];
        *o = Occ{fns[0], a->max_rounds, a->n_vals, a->flags, pcb, 0, 0};
        int k[4];
        for (int v = 0; v < 4; ++v) k[v] = per_cu(v);
        const int base = k[0] > 0 ? k[0] : 1;
        int best = 0;
        const int order[3] = {3, 2, 1};
        for (int v : order)
            if (k[v] > 0 && k[v] >= base) { best = v; break; }
        o->v = best;
        o->per_cu = k[best] > 0 ? k[best] : 1;
    }
    agnes_tally_args b = *a;
    b.set_cache = 0;
    b.power_cache = (o->v & 1) ? (uint32_t)pcb : 0u;
    const uint32_t lpw = fast_lds(MODE, a->flags, (o->v & 2) != 0, a->max_rounds, a->n_vals, W64);
    const uint64_t lds = lds_of(o->v);
    if (lds > 48u * 1024u) {
        hipError_t e = hipFuncSetAttribute(fns[o->v], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    const uint64_t ncu = (uint64_t)(num_cus > 0 ? num_cus : 256);
    uint64_t blocks = (n + AGNES_WAVES_PER_BLOCK - 1) / AGNES_WAVES_PER_BLOCK;
    const uint64_t cap = ncu * (uint64_t)o->per_cu;
    if (blocks > cap) blocks = cap;
    const dim3 g((uint32_t)blocks), blk(256);
    constexpr bool P1 = !W64; /* the PC variants (never chosen for W64) */
    switch (o->v) {
    case 0: hipLaunchKernelGGL((tally_fast<MODE, SKIP, SM, false, false, W64>), g, blk, (size_t)lds, st, b, lpw); break;
    case 1: hipLaunchKernelGGL((tally_fast<MODE, SKIP, SM, P1, false, W64>), g, blk, (size_t)lds, st, b, lpw); break;
    case 2: hipLaunchKernelGGL((tally_fast<MODE, SKIP, SM, false, true, W64>), g, blk, (size_t)lds, st, b, lpw); break;
    default: hipLaunchKernelGGL((tally_fast<MODE, SKIP, SM, P1, true, W64>), g, blk, (size_t)lds, st, b, lpw); break;
    }
    return hipGetLastError();
}

template <uint32_t MODE, bool SKIP, bool SM>
static hipError_t launch_fast_w(const agnes_tally_args* a, int num_cus, hipStream_t st) {
    return a->w64 ? launch_fast_k<MODE, SKIP, SM, true>(a, num_cus, st) : launch_fast_k<MODE, SKIP, SM, false>(a, num_cus, st);
}

hipError_t agnes_launch_tally_fast(const agnes_tally_args* a, uint32_t mode, int num_cus, hipStream_t st) {
    const bool skip = (a->flags & AGNES_FLAG_ROUND_SKIP) != 0;
    const bool sm = (a->flags & AGNES_FLAG_STATE_MACHINE) != 0 && a->states != nullptr;
    if (mode == AGNES_MODE_DEDUP) {
        if (skip) return sm ? launch_fast_w<1, true, true>(a, num_cus, st) : launch_fast_w<1, true, false>(a, num_cus, st);
        return sm ? launch_fast_w<1, false, true>(a, num_cus, st) : launch_fast_w<1, false, false>(a, num_cus, st);
    }
    if (skip) return sm ? launch_fast_w<0, true, true>(a, num_cus, st) : launch_fast_w<0, true, false>(a, num_cus, st);
    return sm ? launch_fast_w<0, false, true>(a, num_cus, st) : launch_fast_w<0, false, false>(a, num_cus, st);
}
