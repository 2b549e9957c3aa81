/*
 * agnes_stream.hip — the stream tally kernel: the u32 fast path for REFERENCE
 * batches without RoundSkip (the BASELINE C2/C3 hot path).
 *
 * agnes_fast.hip walks every instance in its own 256-vote chunks, so a 200-vote
 * instance (C2) fills 78 % of its chunk and that chunk's load re-reads the next
 * instance's first votes.  Here a work-queue batch of up to 16 consecutive
 * instances is walked as ONE vote stream: chunks are full, every vote is loaded
 * once, and the instances a chunk straddles are its segments.  A batch is walked
 * this way when its offsets are multiples of 4 — segment boundaries then fall
 * between lanes, so a lane's 4 votes share one instance — and every instance is in
 * the stream domain (u32 power set, len * maxpow < 2^30, maxpow < 2^22: every chunk
 * partial sum, carry and per-lane threshold below stays inside int32).  Any other
 * batch is walked instance by instance through the same chunk body, one segment
 * per chunk (the agnes_fast.hip discipline); instances outside the u32 domain go
 * to the i64 LIST kernel as everywhere else.
 *
 * Per-segment quantities live one per lane (lane d = segment d of the chunk) and
 * reach the votes through one ds_bpermute by the lane's segment index:
 *   quorum     the chunk's value / nil scans are unsegmented; segment d's running
 *              sums are scan - base_d + carry_d, so is_quorum (round_votes.rs:31-33)
 *              becomes  lane-local prefix > q2_d + base_d - carry_d - exclusive wave
 *              prefix, with base_d read from the lane before the segment's first;
 *   executors  only the instance running into the next chunk carries its per-slot
 *              (value, nil) weights over (ping-pong LDS rows; RoundVotes::new is a
 *              zero row, round_votes.rs:83-90);
 *   State      a batch's States are staged in LDS by one DMA issued as the previous
 *              batch ends; State::apply for vote events (state_machine.rs:196-211)
 *              runs per segment with agnes_fast.hip's ballot search restricted to
 *              the segment's positions, and the States go back in one store.
 */
#include <cstdlib>

#include "agnes_fast.h"

namespace agnes {
namespace stream {
using namespace agnes::fast;

constexpr uint32_t SBQ = 16u;  /* instances per batch (header offsets in lanes 0..SBQ) */
constexpr uint32_t HI = 32u;   /* header lanes HI + k: per-instance data of instance k */
constexpr uint32_t SMALL = 4u; /* batch size of the work queue's tail                  */

/* per-wave LDS: DMA chunk buffer | carried executors, 2 copies x (vw[2R], vn[2R]) u32 |
 * (state machine) the current batch's States */
__host__ __device__ inline uint32_t carry_words(uint32_t R) { return (uint32_t)(align16(16ull * R) / 4u); }
__host__ __device__ inline uint32_t lds_bytes(bool sm, uint32_t R) {
    return PF_BYTES + 8u * carry_words(R) + SBQ * 4u + (sm ? SBQ * 64u + SBQ * 32u : 0u);
}

/* State::apply shadow of a batch instance (LDS, 8 dwords): what the votes did to
 * its State, applied to the staged State when the batch ends */
constexpr uint32_t SH_STEP = 0, SH_EQ8 = 1, SH_FLAGS = 2, SH_LOCK = 3, SH_VALID = 4, SH_DEC = 5, SH_DECR = 6;
constexpr uint32_t F_STEP = 1u, F_LOCK = 2u, F_VALID = 4u, F_DEC = 8u;

/* 0xFF in the bytes of x that are zero (exact, no borrow) */
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    const uint32_t z = ~(t | x) & 0x80808080u;
    return z | (z - (z >> 7));
}
/* 0xFF in the bytes below byte i (i <= 4) */
__device__ __forceinline__ uint32_t below_bytes(uint32_t i) { return i >= 4u ? 0xFFFFFFFFu : (1u << (8u * i)) - 1u; }
/* 0xFF in byte i of the result for bit i of x (x < 16) */
__device__ __forceinline__ uint32_t bytes_of(uint32_t x) {
    const uint32_t b = (x * 0x00204081u) & 0x01010101u;
    return (b << 8) - b;
}

__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

/* a batch: instances [s0, e0); header VGPRs: lanes 0..m the offsets (clamped to
 * n_votes), lane HI + k the set (olo) and, after phase 2, the quorum threshold (q2)
 * of instance k */
struct Hdr {
    uint32_t s0, e0;
    uint32_t olo, ohi, q2;
    uint32_t f31;    /* bit k: instance k in the u32 domain (else the i64 LIST kernel) */
    uint32_t stream; /* walked as one stream                                           */
    uint32_t ready;  /* phase 2 done                                                    */
};

template <bool SM, bool PC>
#ifdef AGNES_STREAM_WPE /* development: minimum waves per SIMD the register allocator must allow */
#define AGNES_STREAM_ATTR __attribute__((amdgpu_waves_per_eu(AGNES_STREAM_WPE)))
#else
#define AGNES_STREAM_ATTR
#endif
__global__ __launch_bounds__(256) AGNES_STREAM_ATTR void tally_stream(agnes_tally_args a, uint32_t lds_per_wave) {
    const uint32_t lane = lane_id();
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint32_t R = a.max_rounds, nv = a.n_vals, ns = a.n_sets, n = a.vb.n_instances;
    const uint64_t NV = a.vb.n_votes;
    const uint32_t p0 = 4u * lane;

    /* block-shared u32 power table (launcher-staged only when it costs no occupancy) */
    if (PC) {
        uint32_t* pc = reinterpret_cast<uint32_t*>(agnes_smem);
        const uint32_t np = ns * nv;
        for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) pc[k] = a.power32[k];
        __syncthreads();
    }
    unsigned char* const base = agnes_smem + a.power_cache + wave * lds_per_wave;
    unsigned char* const pfb = base;
    uint32_t* const crow = reinterpret_cast<uint32_t*>(base + PF_BYTES);
    const uint32_t cw = carry_words(R); /* one copy: vw[2R] then vn[2R] */
    uint32_t* const hs = reinterpret_cast<uint32_t*>(base + PF_BYTES + 8u * cw); /* first-event hints */
    unsigned char* const sb = base + PF_BYTES + 8u * cw + SBQ * 4u;
    uint32_t* const shw = reinterpret_cast<uint32_t*>(sb + SBQ * 64u); /* State::apply shadows */
    uint32_t cpar = 0;
    uint64_t pf_at = ~0ull;
    uint32_t bad = 0;

    /* work queue: batches of SBQ, then SMALL ones for the tail (qn counters, as in
     * agnes_fast.hip: same-address device atomics serialize) */
    const uint32_t qn = gridDim.x < QN ? gridDim.x : QN;
    const uint32_t qk = blockIdx.x % qn;
    uint32_t* const ctr = a.list_count + 1u + qk;
    const uint64_t NB = (uint64_t)(n / SBQ) * 7u / 8u;
    auto range_of = [&](uint32_t t, uint32_t& s0, uint32_t& e0) {
        const uint64_t b = (uint64_t)t * qn + qk;
        const uint64_t s = b < NB ? b * SBQ : NB * SBQ + (b - NB) * SMALL;
        const uint64_t e = s + (b < NB ? SBQ : SMALL);
        s0 = s < n ? (uint32_t)s : n;
        e0 = e < n ? (uint32_t)e : n;
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
     * per batch whether it walks as one stream */
    auto hdr2 = [&](Hdr& h) {
        const uint32_t m = h.e0 - h.s0;
        const bool il = lane >= HI && lane < HI + m;
        const uint32_t k = il ? lane - HI : 0u;
        const uint64_t ob = u64of(shfl(h.olo, k), shfl(h.ohi, k));
        const uint64_t oe = u64of(shfl(h.olo, k + 1u), shfl(h.ohi, k + 1u));
        const uint64_t len = oe > ob ? oe - ob : 0ull;
        bool f31 = false, f30 = false;
        uint32_t q2 = 0;
        if (il) {
            const uint32_t set = h.olo;
            if (set < ns) {
                const agnes_set_info si = a.sets[set];
                const uint64_t wmax = len * (uint64_t)si.maxpow; /* no sum of the instance exceeds it */
                f31 = si.fast && len < (1ull << 32) && wmax < (1ull << 31);
                f30 = f31 && wmax < (1ull << 30) && si.maxpow < (1u << 22);
                /* 3s > 2t <=> s > q2; a q2 >= wmax is never crossed, so min(q2, wmax) */
                const uint64_t qq = (uint64_t)si.q2 < wmax ? (uint64_t)si.q2 : wmax;
                q2 = (uint32_t)(qq < 0x7FFFFFFFull ? qq : 0x7FFFFFFFull);
            } else {
                f31 = true; /* no such set: every vote INVALID, on the u32 path */
            }
        }
        h.q2 = q2;
        const uint32_t full = (uint32_t)((1ull << m) - 1ull);
        h.f31 = (uint32_t)(ballot(f31) >> HI) & full;
        const uint32_t f30m = (uint32_t)(ballot(f30) >> HI) & full;
        const uint64_t Ol = u64of(h.olo, h.ohi);
        const uint64_t On = u64of(shfl(h.olo, lane + 1u), shfl(h.ohi, lane + 1u));
        const bool badl = lane <= m && (((h.olo & 3u) != 0u) || (lane < m && On < Ol));
        h.stream = m > 0u && !ballot(badl) && f30m == full;
        h.ready = 1;
    };
    /* the batch's States into LDS (64 B each, lane l's 16 B at 16 l) */
    auto dma_states = [&](const Hdr& h) {
        const uint32_t m = h.e0 - h.s0;
        if (!SM || m == 0u) return;
        const unsigned char* src =
            reinterpret_cast<const unsigned char*>(a.states + h.s0) + 16u * (lane < 4u * m ? lane : 0u);
        glds16(src, sb);
    };
    auto store_states = [&](const Hdr& h) {
        const uint32_t m = h.e0 - h.s0;
        if (!SM || m == 0u) return;
        if (lane < 4u * m) {
            const uint4 v = *reinterpret_cast<const uint4*>(sb + 16u * lane);
            reinterpret_cast<uint4*>(a.states + h.s0)[lane] = v;
        }
    };
    /* the first chunk of a batch's first stream (prefetch target), ~0 if none */
    auto first_chunk = [&](const Hdr& h) -> uint64_t {
        const uint32_t m = h.e0 - h.s0;
        if (m == 0u || !h.ready) return ~0ull;
        if (h.stream) return u64of(rdl(h.olo, 0u), rdl(h.ohi, 0u));
        const uint64_t Ol = u64of(h.olo, h.ohi);
        const uint64_t On = u64of(shfl(h.olo, lane + 1u), shfl(h.ohi, lane + 1u));
        const uint64_t ne = ballot(lane < m && On > Ol && ((h.f31 >> (lane & 31u)) & 1u));
        if (!ne) return ~0ull;
        const uint32_t k = (uint32_t)__builtin_ctzll(ne);
        return u64of(rdl(h.olo, k), rdl(h.ohi, k)) & ~3ull;
    };

    /* deferred code stores (vmcnt retires in issue order: issued after the next
     * chunk's gather, before its DMA) */
    uint64_t dc_at = ~0ull;
    uint32_t dc_code = 0, dc_pos = 0;
    auto flush = [&]() {
        if (dc_at != ~0ull) {
            const uint64_t j = dc_at + p0;
            if (dc_pos == 0xFu) {
                *reinterpret_cast<uint32_t*>(a.codes + j) = dc_code;
            } else if (dc_pos) {
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s)
                    if ((dc_pos >> s) & 1u) a.codes[j + s] = (uint8_t)(dc_code >> (8u * s));
            }
            dc_at = ~0ull;
        }
    };

    Hdr H, N;
    {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(ctr, 2u);
        t = rdl(t, 0u);
        range_of(t, H.s0, H.e0);
        range_of(t + 1u, N.s0, N.e0);
    }
    if (H.s0 >= H.e0) return;
    uint32_t tq = 0; /* lane 0: slot of the batch after N (atomic in flight) */
    if (lane == 0) tq = atomicAdd(ctr, 1u);
    hdr1(H);
    dma_states(H);
    hdr1(N);
    hdr2(H);

    for (;;) { /* batches: H current, N next */
        const uint32_t m = H.e0 - H.s0;
        const bool S = H.stream;
        bool fresh = true; /* the batch's first chunk step */
        if (a.hint && lane < SBQ) hs[lane] = AGNES_NOHINT;
        bool smf = SM;     /* the shadows are not yet set up from the staged States */
        uint32_t si = 0;
        for (;;) { /* streams of the batch: one (stream batch) or one per instance */
            uint64_t slo, shi;
            uint32_t sk = 0;
            if (S) {
                if (si) break;
                si = 1;
                slo = u64of(rdl(H.olo, 0u), rdl(H.ohi, 0u));
                shi = u64of(rdl(H.olo, m), rdl(H.ohi, m));
            } else {
                const uint64_t Ol = u64of(H.olo, H.ohi);
                const uint64_t On = u64of(shfl(H.olo, lane + 1u), shfl(H.ohi, lane + 1u));
                const uint64_t ne = ballot(lane >= si && lane < m && On > Ol);
                if (!ne) break;
                sk = (uint32_t)__builtin_ctzll(ne);
                si = sk + 1u;
                if (!((H.f31 >> sk) & 1u)) { /* sums may reach 2^31: the i64 LIST kernel */
                    if (lane == 0) a.list[atomicAdd(a.list_count, 1u)] = H.s0 + sk;
                    continue;
                }
                slo = u64of(rdl(H.olo, sk), rdl(H.ohi, sk));
                shi = u64of(rdl(H.olo, sk + 1u), rdl(H.ohi, sk + 1u));
            }
            const uint64_t c0 = slo & ~3ull;
            for (uint64_t c = c0; c < shi; c += CHUNK) {
                /* ---- segments: the instances the chunk straddles ---- */
                uint32_t k0, D = 0, segk = 0, segL = 0;
                uint64_t BL = 0;
                bool cont0, lastc;
                if (S) {
                    const uint64_t Ol = u64of(H.olo, H.ohi);
                    const uint64_t On = u64of(shfl(H.olo, lane + 1u), shfl(H.ohi, lane + 1u));
                    k0 = 63u - (uint32_t)__builtin_clzll(ballot(lane < m && Ol <= c));
                    /* non-empty instances starting inside the chunk, in stream order */
                    uint64_t bk = ballot(lane > k0 && lane < m && Ol < c + CHUNK && Ol < On);
                    segk = lane == 0u ? k0 : 0u;
                    uint32_t kl = k0;
                    while (bk) {
                        const uint32_t k = (uint32_t)__builtin_ctzll(bk);
                        bk &= bk - 1ull;
                        ++D;
                        const uint32_t L = (rdl(H.olo, k) - (uint32_t)c) >> 2; /* its first lane */
                        BL |= 1ull << L;
                        segk = lane == D ? k : segk;
                        segL = lane == D ? L : segL;
                        kl = k;
                    }
                    cont0 = u64of(rdl(H.olo, k0), rdl(H.ohi, k0)) < c;
                    lastc = u64of(rdl(H.olo, kl + 1u), rdl(H.ohi, kl + 1u)) > c + CHUNK;
                } else {
                    k0 = sk;
                    cont0 = c != c0;
                    lastc = shi > c + CHUNK;
                }
                /* the lane's segment dl and instance */
                uint32_t dl = 0, kln = k0;
                if (D) {
                    dl = mbcnt64(BL) + (uint32_t)((BL >> lane) & 1ull);
                    kln = shfl(segk, dl);
                }
                const uint32_t ilane = H.s0 + kln;
                const uint32_t setl = D ? shfl(H.olo, HI + kln) : rdl(H.olo, HI + k0);
                const uint32_t sok = setl < ns;
                const uint32_t pbase = sok ? setl * nv : 0u;
                const uint32_t lo_r = slo > c ? (uint32_t)(slo - c) : 0u;
                const uint32_t hi_r = shi - c < CHUNK ? (uint32_t)(shi - c) : CHUNK;

                /* ---- K1: votes of the chunk + validation + weight gather ---- */
                uint32_t value[VPL], key[VPL], r4, t4, pos = 0, ok = 0;
                uint32_t w[VPL];
                dma_wait(); /* this chunk's DMA (and a new batch's States) have landed */
                {
                    uint32_t inst[VPL], val[VPL];
                    if (pf_at == c) { /* prefetched by LDS-DMA */
                        const uint4 ia = *reinterpret_cast<const uint4*>(pfb + PF_INST + 16u * lane);
                        const uint4 va = *reinterpret_cast<const uint4*>(pfb + PF_VALUE + 16u * lane);
                        const uint4 da = *reinterpret_cast<const uint4*>(pfb + PF_VAL + 16u * lane);
                        inst[0] = ia.x; inst[1] = ia.y; inst[2] = ia.z; inst[3] = ia.w;
                        value[0] = va.x; value[1] = va.y; value[2] = va.z; value[3] = va.w;
                        val[0] = da.x; val[1] = da.y; val[2] = da.z; val[3] = da.w;
                        r4 = *reinterpret_cast<const uint32_t*>(pfb + PF_ROUND + 4u * lane);
                        t4 = *reinterpret_cast<const uint32_t*>(pfb + PF_TYPE + 4u * lane);
                    } else if (c + CHUNK <= NV) {
                        const uint64_t j = c + p0;
                        const uint4 ia = *reinterpret_cast<const uint4*>(a.vb.instance + j);
                        const uint4 va = *reinterpret_cast<const uint4*>(a.vb.value + j);
                        const uint4 da = *reinterpret_cast<const uint4*>(a.vb.validator + j);
                        inst[0] = ia.x; inst[1] = ia.y; inst[2] = ia.z; inst[3] = ia.w;
                        value[0] = va.x; value[1] = va.y; value[2] = va.z; value[3] = va.w;
                        val[0] = da.x; val[1] = da.y; val[2] = da.z; val[3] = da.w;
                        r4 = *reinterpret_cast<const uint32_t*>(a.vb.round + j);
                        t4 = *reinterpret_cast<const uint32_t*>(a.vb.type + j);
                    } else { /* the batch's last chunk */
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
                    /* the vote belongs to the stream, names its instance, round < R, type
                     * in {0, 1}, validator in the set (the boundary's checks) */
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s) {
                        const uint32_t r = byte_of(r4, s), t = byte_of(t4, s);
                        const uint32_t in = (uint32_t)(p0 + s >= lo_r) & (uint32_t)(p0 + s < hi_r);
                        const uint32_t o = in & (uint32_t)(inst[s] == ilane) & (uint32_t)(r < R) &
                                           (uint32_t)(t <= 1u) & (uint32_t)(val[s] < nv) & sok;
                        pos |= in << s;
                        ok |= o << s;
                        key[s] = o ? r * 2u + t : 0xFFFFFFFFu;
                        /* K1: w = power[set][validator] (consensus_executor.rs:62-63 ->
                         * validators.rs:7) */
                        const uint32_t idx = pbase + (o ? val[s] : 0u);
                        w[s] = PC ? reinterpret_cast<const uint32_t*>(agnes_smem)[idx] : a.power32[idx];
                    }
                }
                bad += __builtin_popcount(pos & ~ok);
                /* a gather from HBM retires before the DMA below is issued: a wait on it
                 * behind the DMA would wait for the DMA too (in-order vmcnt) */
                if (!PC) asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));
                if (fresh && !N.ready && N.s0 < N.e0) hdr2(N);
                fresh = false;
                /* the previous chunk's codes, then the next chunk by LDS-DMA */
                flush();
                {
                    uint64_t nc = ~0ull;
                    if (c + CHUNK < shi) {
                        nc = c + CHUNK;
                    } else if (!S) { /* the batch's next u32 instance */
                        const uint64_t Ol = u64of(H.olo, H.ohi);
                        const uint64_t On = u64of(shfl(H.olo, lane + 1u), shfl(H.ohi, lane + 1u));
                        const uint64_t ne = ballot(lane >= si && lane < m && On > Ol && ((H.f31 >> (lane & 31u)) & 1u));
                        if (ne) {
                            const uint32_t k = (uint32_t)__builtin_ctzll(ne);
                            nc = u64of(rdl(H.olo, k), rdl(H.ohi, k)) & ~3ull;
                        }
                    }
                    if (nc == ~0ull && N.s0 < N.e0) nc = first_chunk(N);
                    if (nc != ~0ull && nc + CHUNK <= NV) {
                        __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): this chunk's LDS reads are done */
                        const uint64_t jn = nc + p0;
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
                if (a.dbg & 1u) { /* development knob (AGNES_DEBUG_SKIP=1): memory traffic only */
                    dc_code = (value[0] ^ key[1] ^ w[2] ^ w[3] ^ r4) & 0x07070707u;
                    dc_pos = pos;
                    dc_at = c;
                    continue;
                }

                /* per-vote code: INVALID, else the tally event filled below */
                uint32_t code[VPL], nil = 0;
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s) {
                    code[s] = ((ok >> s) & 1u) ? 0u : AGNES_CODE_INVALID;
                    nil |= (uint32_t)(value[s] == AGNES_NIL) << s;
                }
                /* carried executors: read row A (segment 0, when it continues from the
                 * previous chunk), write row B (the segment running into the next chunk) */
                uint32_t* const A = crow + cpar * cw;
                uint32_t* const B = crow + (cpar ^ 1u) * cw;
                if (lastc) {
                    const bool keep = D == 0u && cont0;
                    for (uint32_t k = lane; k < 4u * R; k += 64u) B[k] = keep ? A[k] : 0u;
                    __builtin_amdgcn_wave_barrier();
                }
                const uint32_t q2s = D ? shfl(H.q2, HI + segk) : rdl(H.q2, HI + k0);
                const uint32_t qd = D ? shfl(q2s, dl) : q2s; /* the q2 of the lane's own segment */

                /* K2+K3 per (round, type) bucket present: one stream-order scan of its value
                 * and nil weights over the chunk (VoteCount::add_vote, round_votes.rs:48-56)
                 * and, per vote, is_quorum with precedence Value > Nil > Any > Init
                 * (:31-33, :58-66) and to_event (vote_executor.rs:26-36) */
                uint32_t rem = ok;
                for (;;) {
                    const uint64_t lm = ballot(rem != 0u);
                    if (!lm) break;
                    const uint32_t kl = (uint32_t)__builtin_ctzll(lm);
                    const uint32_t ks = (uint32_t)__builtin_ctz(rdl(rem, kl));
                    const uint32_t K = rdl(sel4(key, ks), kl);
                    uint32_t av[VPL], an[VPL], inb = 0;
#pragma unroll
                    for (uint32_t s = 0; s < VPL; ++s) {
                        const bool in = key[s] == K;
                        const bool isnil = (nil >> s) & 1u;
                        inb |= (uint32_t)in << s;
                        av[s] = (in && !isnil) ? w[s] : 0u;
                        an[s] = (in && isnil) ? w[s] : 0u;
                    }
                    rem &= ~inb;
                    av[1] += av[0]; av[2] += av[1]; av[3] += av[2];
                    an[1] += an[0]; an[2] += an[1]; an[3] += an[2];
                    const uint32_t iv = scan(av[3]), in_ = scan(an[3]);
                    const uint32_t exv = iv - av[3], exn = in_ - an[3];
                    const uint32_t cv = cont0 ? A[K] : 0u, cn = cont0 ? A[2u * R + K] : 0u;
                    /* segmented sum > q2  <=>  lane-local prefix > q2 + base - carry - exclusive prefix */
                    int32_t tv, tn, ta;
                    uint32_t bvl = 0, bnl = 0;
                    if (D == 0u) {
                        tv = (int32_t)(q2s - cv - exv);
                        tn = (int32_t)(q2s - cn - exn);
                    } else {
                        /* the lane before segment d's first; the shuffles run in every lane
                         * (a lane outside a ds_bpermute's exec mask reads as 0 to the others) */
                        const uint32_t src = segL - 1u;
                        const uint32_t bva = shfl(iv, src), bna = shfl(in_, src);
                        const uint32_t bv = lane == 0u ? 0u : bva;
                        const uint32_t bn = lane == 0u ? 0u : bna;
                        const uint32_t Tv = q2s + bv - (lane == 0u ? cv : 0u);
                        const uint32_t Tn = q2s + bn - (lane == 0u ? cn : 0u);
                        tv = (int32_t)(shfl(Tv, dl) - exv);
                        tn = (int32_t)(shfl(Tn, dl) - exn);
                        bvl = rdl(bv, D);
                        bnl = rdl(bn, D);
                    }
                    /* value + nil > q2: the two thresholds' sum less one q2 (mod 2^32) */
                    ta = (int32_t)((uint32_t)tv + (uint32_t)tn - qd);
                    if (K & 1u) { /* precommits: Value -> PrecommitValue, Nil -> None, Any -> PrecommitAny */
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s) {
                            const bool qv = (int32_t)av[s] > tv, qn = (int32_t)an[s] > tn,
                                       qa = (int32_t)(av[s] + an[s]) > ta;
                            const uint32_t ev = qv ? AGNES_CODE_PRECOMMIT_VALUE
                                              : (qn ? AGNES_CODE_NONE : (qa ? AGNES_CODE_PRECOMMIT_ANY : AGNES_CODE_NONE));
                            code[s] = ((inb >> s) & 1u) ? ev : code[s];
                        }
                    } else { /* prevotes: PolkaValue / PolkaNil / PolkaAny */
#pragma unroll
                        for (uint32_t s = 0; s < VPL; ++s) {
                            const bool qv = (int32_t)av[s] > tv, qn = (int32_t)an[s] > tn,
                                       qa = (int32_t)(av[s] + an[s]) > ta;
                            const uint32_t ev = qv ? AGNES_CODE_POLKA_VALUE
                                              : (qn ? AGNES_CODE_POLKA_NIL : (qa ? AGNES_CODE_POLKA_ANY : AGNES_CODE_NONE));
                            code[s] = ((inb >> s) & 1u) ? ev : code[s];
                        }
                    }
                    if (lastc && lane == 63u) { /* the last segment's weights so far */
                        B[K] += iv - bvl;
                        B[2u * R + K] += in_ - bnl;
                    }
                    __builtin_amdgcn_wave_barrier();
                }
                if (lastc) cpar ^= 1u;

                /* ---- K4: State::apply(v.round, event), stream order (consensus_executor.rs:64-68)
                 * Without RoundSkip the vote-driven steps form the monoid {id, Prevote ->
                 * Precommit, -> Commit} (state_machine.rs:196-211): in a segment every
                 * vote is decided by two positions, the first PrecommitValue (commit, any
                 * round: :211) and P1, the first PolkaNil / PolkaValue at eqr before it
                 * while in Prevote (:197-198).  Messages: TimeoutPrevote for PolkaAny at
                 * eqr before P1 in Prevote (:196), TimeoutPrecommit for PrecommitAny at eqr
                 * before the commit (:208), the step messages at P1 and the commit.  The
                 * State takes locked at P1 (a PolkaValue), valid = the last PolkaValue at
                 * eqr in Prevote / Precommit before the commit (:198, :202; its value is
                 * the last non-nil one among them, round_votes.rs:50-54) and the decision.
                 * Segments start at lane boundaries, so all of it is lane-parallel: byte
                 * masks per lane, "earlier in my segment" from two ballots, the results
                 * into the instance's LDS shadow (rare: a nil vote's label, label_at). */
                /* the split route's first-event hint: the earliest vote of each instance
                 * whose code carries an event (1..5); apply_codes starts its walk there */
                if (!SM && a.hint) {
                    uint32_t fs = VPL;
#pragma unroll
                    for (int s2 = (int)VPL - 1; s2 >= 0; --s2) {
                        const uint32_t ev = code[s2] & 7u;
                        if (ev != 0u && ev <= AGNES_CODE_PRECOMMIT_VALUE) fs = (uint32_t)s2;
                    }
                    const uint32_t ilo = D ? shfl(H.olo, kln) : rdl(H.olo, k0); /* low 32 bits of its start */
                    if (fs < VPL) atomicMin(hs + kln, (uint32_t)c + p0 + fs - ilo);
                }
                uint32_t smmsg = 0;
                if (SM) {
                    if (smf) { /* the batch's staged States have landed (dma_wait above) */
                        if (lane < m) {
                            const uint32_t* const sp = reinterpret_cast<const uint32_t*>(sb + 64u * lane);
                            const int64_t rnd = (int64_t)u64of(sp[2], sp[3]);
                            shw[8u * lane + SH_STEP] = sp[13] & 0xFFu;
                            shw[8u * lane + SH_EQ8] = (rnd >= 0 && rnd <= 255) ? (uint32_t)rnd : 0x100u;
                            shw[8u * lane + SH_FLAGS] = 0u;
                        }
                        smf = false;
                    }
                    /* the value of the Value event at chunk position f of a nil vote: the
                     * last value counted into its bucket before it (round_votes.rs:50-54),
                     * searched in the chunk's segment [plo, f), then in the instance's
                     * earlier chunks (newest first, one vote per lane: rare, few registers) */
                    auto label_at = [&](uint32_t f, uint32_t plo, uint64_t ibeg, uint32_t iid) -> uint32_t {
                        const uint32_t fl = f >> 2, fs = f & 3u;
                        const uint32_t K = rdl(sel4(key, fs), fl);
                        uint32_t cand = 0;
#pragma unroll
                        for (uint32_t s2 = 0; s2 < VPL; ++s2)
                            cand |= (uint32_t)(key[s2] == K && value[s2] != AGNES_NIL && p0 + s2 < f && p0 + s2 >= plo) << s2;
                        const uint64_t cl = ballot(cand != 0u);
                        if (cl) {
                            const uint32_t hl = 63u - (uint32_t)__builtin_clzll(cl);
                            const uint32_t hs = 31u - (uint32_t)__builtin_clz(rdl(cand, hl));
                            return rdl(sel4(value, hs), hl);
                        }
                        for (uint64_t pcz = c; pcz > (ibeg & ~3ull);) {
                            pcz -= CHUNK;
                            uint32_t hit = 0, hv = 0;
#pragma unroll 1
                            for (int s2 = (int)VPL - 1; s2 >= 0; --s2) {
                                const uint64_t j = pcz + p0 + (uint32_t)s2;
                                if (!hit && j >= ibeg && j < c) {
                                    const uint8_t *br = a.vb.round, *bt = a.vb.type;
                                    const uint32_t *bx = a.vb.validator, *bv = a.vb.value, *bi = a.vb.instance;
                                    asm volatile("" : "+s"(br), "+s"(bt), "+s"(bx), "+s"(bv), "+s"(bi));
                                    const uint32_t vr = br[j], vt = bt[j], vx = bx[j], vv = bv[j];
                                    if (bi[j] == iid && vr < R && vt <= 1u && vx < nv && vr * 2u + vt == K &&
                                        vv != AGNES_NIL) {
                                        hit = 1;
                                        hv = vv;
                                    }
                                }
                            }
                            const uint64_t hl = ballot(hit != 0u);
                            if (hl) return rdl(hv, 63u - (uint32_t)__builtin_clzll(hl));
                        }
                        return 0u; /* VoteCount::new's label (round_votes.rs:36-45) */
                    };
                    uint32_t* const sh = shw + 8u * kln;
                    const uint32_t step = sh[SH_STEP], eq8 = sh[SH_EQ8], vset = sh[SH_FLAGS] & F_VALID;
                    const uint32_t c4 = code[0] | (code[1] << 8) | (code[2] << 16) | (code[3] << 24);
                    const uint32_t e4 = c4 & 0x07070707u;
                    const uint32_t live0 = step != AGNES_STEP_COMMIT ? bytes_of(pos) : 0u; /* :205 */
                    const uint32_t eqm = eq8 < 0x100u ? zero_bytes(r4 ^ (eq8 * 0x01010101u)) & live0 : 0u;
                    const uint32_t cvb = zero_bytes(e4 ^ 0x05050505u) & live0;
                    const uint32_t pvb = zero_bytes(e4 ^ 0x03030303u) & eqm;
                    const uint32_t pnb = zero_bytes(e4 ^ 0x02020202u) & eqm;
                    const uint32_t pab = zero_bytes(e4 ^ 0x01010101u) & eqm;
                    const uint32_t cab = zero_bytes(e4 ^ 0x04040404u) & eqm;
                    const bool prevote = step == AGNES_STEP_PREVOTE;
                    const uint32_t p1b = prevote ? (pvb | pnb) : 0u;
                    /* my segment: [first lane ss, next start ns) */
                    const uint64_t SSm = BL | 1ull;
                    const uint64_t upto = lane == 63u ? ~0ull : ((2ull << lane) - 1ull);
                    const uint32_t ss = 63u - (uint32_t)__builtin_clzll(SSm & upto);
                    const uint64_t nsm = SSm & ~upto;
                    const uint64_t before = ((1ull << lane) - 1ull) & ~((1ull << ss) - 1ull);
                    const uint64_t after = (nsm ? ((nsm & (0ull - nsm)) - 1ull) : ~0ull) & ~upto;
                    const uint64_t MCV = ballot(cvb != 0u), MP1 = ballot(p1b != 0u);
                    const bool cv_before = (MCV & before) != 0ull, p1_before = (MP1 & before) != 0ull;
                    const uint32_t cs = cvb ? ((uint32_t)__builtin_ctz(cvb) >> 3) : 4u; /* my first commit slot */
                    const uint32_t alive = cv_before ? 0u : below_bytes(cs);
                    const uint32_t p1m = (!p1_before && !cv_before) ? (p1b & below_bytes(cs)) : 0u;
                    const uint32_t ps = p1m ? ((uint32_t)__builtin_ctz(p1m) >> 3) : 4u; /* my P1 slot */
                    const uint32_t tpr = (prevote && !p1_before) ? below_bytes(ps) : 0u;
                    smmsg = (pab & alive & tpr & (AGNES_VMSG_TIMEOUT_PREVOTE * 0x10101010u)) |
                            (cab & alive & (AGNES_VMSG_TIMEOUT_PRECOMMIT * 0x10101010u));
                    const bool p1_pv = p1m && ((pvb >> (8u * ps)) & 1u);
                    if (p1m) smmsg |= (p1_pv ? AGNES_VMSG_PRECOMMIT_VALUE : AGNES_VMSG_PRECOMMIT_NIL) << (8u * ps + 4u);
                    const bool commit = !cv_before && cvb != 0u;
                    if (commit) smmsg |= AGNES_VMSG_DECISION << (8u * cs + 4u);
                    /* valid: the PolkaValues at eqr in Prevote (after P1) / Precommit, alive */
                    const uint32_t vcand = (prevote || step == AGNES_STEP_PRECOMMIT) ? (pvb & alive) : 0u;
                    uint32_t nilb = 0;
#pragma unroll
                    for (uint32_t s2 = 0; s2 < VPL; ++s2) nilb |= (uint32_t)(value[s2] == AGNES_NIL) << s2;
                    const uint32_t vnn = vcand & ~bytes_of(nilb);
                    const uint64_t MV = ballot(vcand != 0u), MVN = ballot(vnn != 0u);
                    const uint64_t seg = before | after | (1ull << lane);
                    /* the shadow (one lane per segment and kind: no two lanes write one word) */
                    const bool p1_nil = p1_pv && value[ps & 3u] == AGNES_NIL;
                    if (p1m) {
                        atomicMax(sh + SH_STEP, (uint32_t)AGNES_STEP_PRECOMMIT);
                        atomicOr(sh + SH_FLAGS, p1_pv ? (F_STEP | F_LOCK) : F_STEP);
                        if (p1_pv && !p1_nil) sh[SH_LOCK] = value[ps & 3u];
                    }
                    const bool dec_nil = commit && value[cs & 3u] == AGNES_NIL;
                    if (commit) {
                        atomicMax(sh + SH_STEP, (uint32_t)AGNES_STEP_COMMIT);
                        atomicOr(sh + SH_FLAGS, F_STEP | F_DEC);
                        sh[SH_DECR] = byte_of(r4, cs & 3u);
                        if (!dec_nil) sh[SH_DEC] = value[cs & 3u];
                    }
                    if (vnn && !(MVN & after)) { /* the segment's last non-nil candidate */
                        sh[SH_VALID] = value[(31u - (uint32_t)__builtin_clz(vnn)) >> 3];
                        atomicOr(sh + SH_FLAGS, F_VALID);
                    }
                    /* only nil candidates in the segment and valid not yet set in this batch:
                     * the label of the first one (round_votes.rs:50-54) */
                    const bool fp_nil = vcand && !(MV & before) && !(MVN & seg) && !vset;
                    /* rare: labels of nil votes, by the bucket search */
                    uint64_t need = ballot(p1_nil || dec_nil || fp_nil);
                    while (need) {
                        const uint32_t L = (uint32_t)__builtin_ctzll(need);
                        need &= need - 1ull;
                        const uint32_t kk = rdl(kln, L), ssl = rdl(ss, L);
                        const uint32_t plo = 4u * ssl > lo_r ? 4u * ssl : lo_r;
                        const uint64_t ibeg = S ? u64of(rdl(H.olo, kk), rdl(H.ohi, kk)) : slo;
                        const uint32_t iid = H.s0 + kk;
                        uint32_t* const shk = shw + 8u * kk;
                        if (rdl((uint32_t)p1_nil, L)) {
                            const uint32_t lab = label_at(4u * L + rdl(ps, L), plo, ibeg, iid);
                            if (lane == 0u) shk[SH_LOCK] = lab;
                        }
                        if (rdl((uint32_t)dec_nil, L)) {
                            const uint32_t lab = label_at(4u * L + rdl(cs, L), plo, ibeg, iid);
                            if (lane == 0u) shk[SH_DEC] = lab;
                        }
                        if (rdl((uint32_t)fp_nil, L)) {
                            const uint32_t fs = (uint32_t)__builtin_ctz(rdl(vcand, L)) >> 3;
                            const uint32_t lab = label_at(4u * L + fs, plo, ibeg, iid);
                            if (lane == 0u) {
                                shk[SH_VALID] = lab;
                                atomicOr(shk + SH_FLAGS, F_VALID);
                            }
                        }
                    }
                }

                /* codes (deferred): one 4-B store when all 4 votes belong to the stream */
                dc_code = code[0] | (code[1] << 8) | (code[2] << 16) | (code[3] << 24) | smmsg;
                dc_pos = pos;
                dc_at = c;
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (a.hint && lane < m) a.hint[H.s0 + lane] = hs[lane];
        /* batch end: the shadows into the staged States, States back, then the next batch */
        if (SM && !smf && lane < m) {
            const uint32_t* const sh = shw + 8u * lane;
            const uint32_t f = sh[SH_FLAGS];
            if (f) {
                uint32_t* const sp = reinterpret_cast<uint32_t*>(sb + 64u * lane);
                uint32_t fl = (sp[13] & ~0xFFu) | sh[SH_STEP];
                if (f & F_LOCK) { sp[4] = sp[2]; sp[5] = sp[3]; sp[10] = sh[SH_LOCK]; fl |= 1u << 8; }
                if (f & F_VALID) { sp[6] = sp[2]; sp[7] = sp[3]; sp[11] = sh[SH_VALID]; fl |= 1u << 16; }
                if (f & F_DEC) { sp[8] = sh[SH_DECR]; sp[9] = 0u; sp[12] = sh[SH_DEC]; fl |= 1u << 24; }
                sp[13] = fl;
            }
        }
        store_states(H);
        if (N.s0 >= N.e0) break;
        if (!N.ready) hdr2(N);
        H = N;
        dma_states(H);
        range_of(rdl(tq, 0u), N.s0, N.e0); /* the batch after, grabbed one batch ago */
        if (lane == 0) tq = atomicAdd(ctr, 1u);
        hdr1(N);
    }
    flush();
    const uint32_t nb = rdl(scan(bad), 63u);
    if (lane == 0 && nb) atomicAdd(a.n_invalid, (unsigned long long)nb);
}

} // namespace stream
} // namespace agnes

/* ------------------------------------------------------------------ */
/* launcher                                                            */

template <bool SM>
static hipError_t launch_stream_k(const agnes_tally_args* a, int num_cus, hipStream_t st) {
    const uint32_t n = a->vb.n_instances;
    if (n == 0) return hipSuccess;
    using agnes::stream::tally_stream;
    const void* fns[2] = {reinterpret_cast<const void*>(&tally_stream<SM, false>),
                          reinterpret_cast<const void*>(&tally_stream<SM, true>)};
    const uint32_t lpw = agnes::stream::lds_bytes(SM, a->max_rounds);
    const uint64_t wave_lds = (uint64_t)lpw * AGNES_WAVES_PER_BLOCK;
    const uint64_t pcb = agnes::align16(4ull * a->n_sets * a->n_vals);
    /* blocks per CU from the occupancy query; the LDS power table only where it
     * costs no occupancy.  Cached per LDS shape. */
    struct Occ { uint64_t wave_lds, pcb; int per_cu; bool pc; };
    static thread_local Occ occ[8];
    static thread_local unsigned occ_next = 0;
    Occ* o = nullptr;
    for (auto& c : occ)
        if (c.per_cu && c.wave_lds == wave_lds && c.pcb == pcb) o = &c;
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
        *o = Occ{wave_lds, pcb, k0 > 0 ? k0 : 1, false};
        if (k1 > 0 && k1 >= k0) {
            o->per_cu = k1;
            o->pc = true;
        }
        if (const char* d = std::getenv("AGNES_BLOCKS_PER_CU")) { /* development knob */
            const int v = std::atoi(d);
            if (v > 0 && v < o->per_cu) o->per_cu = v;
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
    if (o->pc)
        hipLaunchKernelGGL((tally_stream<SM, true>), dim3((uint32_t)blocks), dim3(256), (size_t)lds, st, b, lpw);
    else
        hipLaunchKernelGGL((tally_stream<SM, false>), dim3((uint32_t)blocks), dim3(256), (size_t)lds, st, b, lpw);
    return hipGetLastError();
}

hipError_t agnes_launch_tally_stream(const agnes_tally_args* a, int num_cus, hipStream_t st) {
    const bool sm = (a->flags & AGNES_FLAG_STATE_MACHINE) != 0 && a->states != nullptr;
    return sm ? launch_stream_k<true>(a, num_cus, st) : launch_stream_k<false>(a, num_cus, st);
}
