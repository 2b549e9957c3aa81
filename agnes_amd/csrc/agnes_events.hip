/*
 * agnes_events.hip — the event stream of a coded batch (include/agnes.h
 * agnes_event_offsets / agnes_events): every Some(Event) the votes produced,
 * stream-compacted, with its payload.
 *
 * ConsensusExecutor::apply_vote (consensus_executor.rs:61-69) hands each vote to
 * its (round, type) VoteExecutor, whose apply returns Option<Event>
 * (vote_executor.rs:20-36); the tally left that as the vote's code (bits 0..2,
 * plus bit 3 for the RoundSkip extension's event, applied first).  PolkaValue and
 * PrecommitValue carry the Value in their VoteCount's single value slot after the
 * vote (round_votes.rs:50-54, 58-59): the last non-nil value among the votes the
 * tally added to that executor (every code but INVALID / REJECTED), Value{} (0)
 * before any.
 *
 * Two passes and a scan.  The count pass walks the codes (1 B per vote), one
 * instance per lane in 64-B windows; the exclusive scan of the counts is
 * agnes_edges.hip's.  The emit pass (event_emit_stream) walks a batch of EB
 * consecutive instances as one vote stream per wave, 256 votes per pass over code,
 * round, type and value (7 B per vote), the next pass loaded while the current one
 * is processed; it writes the 24-B records through an LDS staging area as
 * coalesced 8-B stores.  The value slot after a vote: its own value when non-nil,
 * else the last non-nil value of its (instance, round, type) in the pass, else the
 * carried slot in LDS ([EB][keys] per wave).  When the pass's (instance, round)
 * runs do not go back (every config the bench runs), one max-scan per vote type
 * finds that last value for all keys at once; otherwise one ballot pass per key
 * present.  Measured (C2, 200M votes, 67.8M records): 0.85 ms, against 1.01 ms for
 * the one-wave-per-instance walk (event_emit_wave, kept for keys > 64).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "agnes_device.h"
#include "agnes_internal.h"

namespace agnes {
namespace events {

struct EvArgs {
    agnes_vote_batch vb;
    const uint8_t* codes;
    uint64_t* offs; /* n_instances + 1 */
    agnes_vote_event* out;
    uint32_t keys;  /* 2 * max_rounds */
    /* (SEG emit) the segmented records: seg[mult * offsets[i] + k], k < counts[i] */
    uint4* seg;
    uint64_t* counts;
    uint32_t mult;
    /* the dense writers: out holds cap records; a record whose position is past cap, or
     * past its instance's (or batch's) end offset, is dropped and counted in *ovf
     * (agnes_records_overflow) -- offsets that disagree with the codes, or an undersized
     * out, never write outside out */
    uint64_t cap;
    unsigned long long* ovf;
};

/* a dense record at position d, bounded by lim (min of cap and the segment's end) */
__device__ __forceinline__ bool in_cap(uint64_t d, uint64_t lim, uint32_t& drop) {
    const bool ok = d < lim;
    drop += ok ? 0u : 1u;
    return ok;
}
__device__ __forceinline__ void flush_drops(const unsigned long long* ovf, uint32_t drop) {
    if (drop) atomicAdd(const_cast<unsigned long long*>(ovf), (unsigned long long)drop);
}

/* W consecutive bytes of a u8 column from w (W = 4: one dword; W >= 16: 16-B loads
 * of one line in flight together); past n_votes: zeros */
template <uint32_t W>
__device__ __forceinline__ void load_bytes(const uint8_t* col, uint64_t w, uint64_t NV, uint32_t (&v)[W / 4u]) {
    if (w + W <= NV) {
        if constexpr (W >= 16u) {
#pragma unroll
            for (uint32_t k = 0; k < W / 16u; ++k) {
                const uint4 q = *reinterpret_cast<const uint4*>(col + w + 16u * k);
                v[4u * k] = q.x;
                v[4u * k + 1u] = q.y;
                v[4u * k + 2u] = q.z;
                v[4u * k + 3u] = q.w;
            }
        } else {
            v[0] = *reinterpret_cast<const uint32_t*>(col + w);
        }
    } else {
#pragma unroll
        for (uint32_t d = 0; d < W / 4u; ++d) v[d] = 0u;
        for (uint32_t b = 0; b < W && w + b < NV; ++b) v[b >> 2] |= (uint32_t)col[w + b] << (8u * (b & 3u));
    }
}

/* W consecutive u32 values from w (16-B loads when the column allows) */
template <uint32_t W, bool A16>
__device__ __forceinline__ void load_words(const uint32_t* col, uint64_t w, uint64_t NV, uint32_t (&v)[W]) {
    if (A16 && w + W <= NV) {
#pragma unroll
        for (uint32_t k = 0; k < W / 4u; ++k) {
            const uint4 q = *reinterpret_cast<const uint4*>(col + w + 4u * k);
            v[4u * k] = q.x;
            v[4u * k + 1u] = q.y;
            v[4u * k + 2u] = q.z;
            v[4u * k + 3u] = q.w;
        }
    } else {
#pragma unroll
        for (uint32_t b = 0; b < W; ++b) v[b] = w + b < NV ? col[w + b] : AGNES_NIL;
    }
}

/* event kind of a code's bits 0..2 (vote_executor.rs:26-36) */
__device__ __forceinline__ uint32_t kind_of(uint32_t ev) {
    /* 1 PolkaAny, 2 PolkaNil, 3 PolkaValue, 4 PrecommitAny, 5 PrecommitValue */
    return ev - 1u + AGNES_EV_POLKA_ANY;
}

__device__ __forceinline__ void put(agnes_vote_event* o, uint64_t j, uint32_t i, uint32_t value, uint32_t round,
                                    uint32_t kind, uint32_t msg) {
    uint2* const q = reinterpret_cast<uint2*>(o);
    q[0] = make_uint2((uint32_t)j, (uint32_t)(j >> 32));
    q[1] = make_uint2(i, value);
    q[2] = make_uint2(round | (kind << 8) | (msg << 16), 0u);
}

/* the number of records of instance i: one per vote whose code is Some(Event), plus
 * one per RoundSkip bit, over the votes the tally added (W-byte windows of codes) */
template <uint32_t W>
__device__ __forceinline__ uint64_t count_records(const EvArgs& a, uint32_t i) {
    const uint64_t NV = a.vb.n_votes;
    uint64_t lo = a.vb.offsets[i], hi = a.vb.offsets[i + 1u];
    lo = lo < NV ? lo : NV;
    hi = hi < NV ? hi : NV;
    uint64_t cnt = 0;
    for (uint64_t w = lo & ~(uint64_t)(W - 1u); w < hi; w += W) {
        uint32_t c[W / 4u];
        load_bytes<W>(a.codes, w, NV, c);
#pragma unroll
        for (uint32_t b = 0; b < W; ++b) {
            const uint64_t j = w + b;
            const uint32_t cb = (c[b >> 2] >> (8u * (b & 3u))) & 0xFFu, ev = cb & AGNES_CODE_EVENT_MASK;
            if (j < lo || j >= hi || ev == AGNES_CODE_INVALID || ev == AGNES_CODE_REJECTED) continue;
            cnt += ((cb >> 3) & 1u) + (ev != AGNES_CODE_NONE ? 1u : 0u);
        }
    }
    return cnt;
}

/* the counts of the instances a tally's flow kernel handed to its walk list (the
 * flow kernel counted every other one itself): a grid-stride loop over the list */
template <uint32_t W>
__global__ __launch_bounds__(256) void event_count_list(EvArgs a, const uint32_t* walk, const uint32_t* walk_n) {
    const uint32_t L = *(volatile const uint32_t*)walk_n;
    for (uint32_t k = blockIdx.x * 256u + threadIdx.x; k < L; k += gridDim.x * 256u) {
        const uint32_t i = walk[k];
        a.offs[i + 1u] = count_records<W>(a, i);
    }
}

template <bool EMIT, uint32_t W, bool A16>
__global__ __launch_bounds__(64) void event_walk(EvArgs a) {
    uint32_t* const lab = reinterpret_cast<uint32_t*>(agnes_smem);
    const uint32_t lane = threadIdx.x;
    const uint32_t i = blockIdx.x * 64u + lane;
    if (i >= a.vb.n_instances) return;
    if (!EMIT) {
        a.offs[i + 1u] = count_records<W>(a, i);
        return;
    }
    for (uint32_t k = 0; k < a.keys; ++k) lab[k * 64u + lane] = 0u; /* VoteCount::new: Value{} */
    const uint64_t NV = a.vb.n_votes;
    uint64_t lo = a.vb.offsets[i], hi = a.vb.offsets[i + 1u];
    lo = lo < NV ? lo : NV;
    hi = hi < NV ? hi : NV;
    const uint64_t base = EMIT ? a.offs[i] : 0u;
    const uint64_t lim = EMIT ? min(a.offs[i + 1u], a.cap) : 0u;
    uint32_t drop = 0;
    uint64_t cnt = 0;
    for (uint64_t w = lo & ~(uint64_t)(W - 1u); w < hi; w += W) {
        uint32_t c[W / 4u];
        load_bytes<W>(a.codes, w, NV, c);
        uint32_t r[W / 4u], t[W / 4u], v[EMIT ? W : 1u];
        if (EMIT) {
            load_bytes<W>(a.vb.round, w, NV, r);
            load_bytes<W>(a.vb.type, w, NV, t);
            load_words<EMIT ? W : 1u, A16>(a.vb.value, w, NV, v);
        }
#pragma unroll
        for (uint32_t b = 0; b < W; ++b) {
            const uint64_t j = w + b;
            const uint32_t sh8 = 8u * (b & 3u);
            const uint32_t cb = (c[b >> 2] >> sh8) & 0xFFu, ev = cb & AGNES_CODE_EVENT_MASK;
            /* outside the instance, or a vote the tally did not add */
            if (j < lo || j >= hi || ev == AGNES_CODE_INVALID || ev == AGNES_CODE_REJECTED) continue;
            const uint32_t skip = (cb >> 3) & 1u, has = ev != AGNES_CODE_NONE ? 1u : 0u;
            const uint32_t rb = (r[b >> 2] >> sh8) & 0xFFu, tb = (t[b >> 2] >> sh8) & 0xFFu;
            const uint32_t key = rb * 2u + tb;
            if (tb > 1u || key >= a.keys) continue; /* (never for a code the tally wrote) */
            uint32_t* const p = lab + key * 64u + lane;
            if (v[b] != AGNES_NIL) *p = v[b]; /* the value slot, last writer wins */
            const uint32_t msg = cb >> AGNES_CODE_MSG_SHIFT;
            if (skip && in_cap(base + cnt, lim, drop)) put(a.out + base + cnt, j, i, AGNES_NIL, rb, AGNES_EV_ROUND_SKIP, msg);
            cnt += skip;
            if (has) {
                const bool val = ev == AGNES_CODE_POLKA_VALUE || ev == AGNES_CODE_PRECOMMIT_VALUE;
                if (in_cap(base + cnt, lim, drop)) put(a.out + base + cnt, j, i, val ? *p : AGNES_NIL, rb, kind_of(ev), msg);
                ++cnt;
            }
        }
    }
    flush_drops(a.ovf, drop);
}

/* ---- the segmented records (agnes_tally_records) ------------------------------------
 * Instance i's records go to seg[mult * offsets[i] + k] (mult 2 with RoundSkip: a vote
 * gives up to two records), k < counts[i], as 16-B agnes_seg_event.  The flow route
 * writes them from the tally kernel itself; these are the other routes' (one lane per
 * instance, the event_walk order) and the flow route's walk-list instances (LIST). */
__device__ __forceinline__ void put_seg(uint4* o, uint64_t j, uint32_t value, uint32_t round, uint32_t kind,
                                        uint32_t msg) {
    *o = make_uint4((uint32_t)j, (uint32_t)(j >> 32), value, round | (kind << 8) | (msg << 16));
}

template <bool LIST, uint32_t W, bool A16>
__global__ __launch_bounds__(64) void seg_walk(EvArgs a, const uint32_t* list, const uint32_t* list_n, uint32_t mult,
                                               uint4* seg, uint64_t* counts) {
    uint32_t* const lab = reinterpret_cast<uint32_t*>(agnes_smem);
    const uint32_t lane = threadIdx.x;
    uint32_t i;
    if (LIST) {
        const uint32_t k = blockIdx.x * 64u + lane;
        if (k >= *(volatile const uint32_t*)list_n) return;
        i = list[k];
    } else {
        i = blockIdx.x * 64u + lane;
        if (i >= a.vb.n_instances) return;
    }
    for (uint32_t k = 0; k < a.keys; ++k) lab[k * 64u + lane] = 0u; /* VoteCount::new: Value{} */
    const uint64_t NV = a.vb.n_votes;
    uint64_t lo = a.vb.offsets[i], hi = a.vb.offsets[i + 1u];
    lo = lo < NV ? lo : NV;
    hi = hi < NV ? hi : NV;
    uint4* const out = seg + (uint64_t)mult * a.vb.offsets[i];
    uint64_t cnt = 0;
    /* W-vote windows of every column (event_walk's order and rules) */
    for (uint64_t w = lo & ~(uint64_t)(W - 1u); w < hi; w += W) {
        uint32_t c[W / 4u], r[W / 4u], t[W / 4u], v[W];
        load_bytes<W>(a.codes, w, NV, c);
        load_bytes<W>(a.vb.round, w, NV, r);
        load_bytes<W>(a.vb.type, w, NV, t);
        load_words<W, A16>(a.vb.value, w, NV, v);
#pragma unroll
        for (uint32_t b = 0; b < W; ++b) {
            const uint64_t j = w + b;
            const uint32_t sh8 = 8u * (b & 3u);
            const uint32_t cb = (c[b >> 2] >> sh8) & 0xFFu, ev = cb & AGNES_CODE_EVENT_MASK;
            if (j < lo || j >= hi || ev == AGNES_CODE_INVALID || ev == AGNES_CODE_REJECTED) continue; /* not added */
            const uint32_t rb = (r[b >> 2] >> sh8) & 0xFFu, tb = (t[b >> 2] >> sh8) & 0xFFu, key = rb * 2u + tb;
            if (tb > 1u || key >= a.keys) continue; /* (never for a code the tally wrote) */
            uint32_t* const p = lab + key * 64u + lane;
            if (v[b] != AGNES_NIL) *p = v[b]; /* the value slot, last writer wins (round_votes.rs:50-54) */
            const uint32_t msg = cb >> AGNES_CODE_MSG_SHIFT;
            if ((cb >> 3) & 1u) put_seg(out + cnt++, j, AGNES_NIL, rb, AGNES_EV_ROUND_SKIP, msg);
            if (ev != AGNES_CODE_NONE) {
                const bool val = ev == AGNES_CODE_POLKA_VALUE || ev == AGNES_CODE_PRECOMMIT_VALUE;
                put_seg(out + cnt++, j, val ? *p : AGNES_NIL, rb, kind_of(ev), msg);
            }
        }
    }
    counts[i] = cnt;
}

/* the dense stream from the segmented one, adding the instance id (agnes_vote_event):
 * wave w writes the dense records of instances 32w .. 32w + 31 -- one contiguous range,
 * offs[32w] .. offs[32w + 32] -- 64 at a time, lane l the record at position p: its
 * instance by a 5-step binary search over the wave's offsets (one per lane, relative
 * to the range's start), then one 16-B read of that instance's segment.  Every lane
 * has a record in every step but the last (one instance per step left lanes idle) */
__global__ __launch_bounds__(256) void seg_compact(agnes_vote_batch vb, uint32_t mult, const uint4* seg,
                                                   const uint64_t* offs, agnes_vote_event* out, uint64_t cap,
                                                   unsigned long long* ovf) {
    const uint32_t lane = threadIdx.x & 63u, w = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t n = vb.n_instances, i0 = 32u * w;
    if (i0 >= n) return; /* wave-uniform */
    const uint32_t m = n - i0 < 32u ? n - i0 : 32u;
    uint2* const stage = reinterpret_cast<uint2*>(agnes_smem) + (threadIdx.x >> 6) * 192u; /* 1.5 KB per wave */
    /* the wave's range, bounded by out's capacity (offsets scanned from counts that are
     * not the segments', or an undersized out: the records past cap are dropped, counted) */
    const uint64_t base = offs[i0], end = offs[i0 + m];
    const uint64_t total = end > base ? end - base : 0u;
    const uint64_t keep = base >= cap ? 0u : (total < cap - base ? total : cap - base);
    if (lane == 0u && keep < total) atomicAdd(ovf, (unsigned long long)(total - keep));
    if (total > 0xFFFFFF00ull) { /* positions past u32 (4e9 records in 32 instances): per instance */
        for (uint32_t i = i0; i < i0 + m; ++i) {
            const uint64_t o = offs[i], oe = offs[i + 1u];
            if (o >= base + keep) break;
            const uint64_t cnt = (oe < base + keep ? oe : base + keep) > o ? (oe < base + keep ? oe : base + keep) - o : 0u;
            const uint4* const src = seg + (uint64_t)mult * vb.offsets[i];
            for (uint64_t k = lane; k < cnt; k += 64u) {
                const uint4 r = src[k];
                uint2* const q = reinterpret_cast<uint2*>(out + o + k);
                q[0] = make_uint2(r.x, r.y);
                q[1] = make_uint2(i, r.z);
                q[2] = make_uint2(r.w, 0u);
            }
        }
        return;
    }
    /* lane k < m: instance i0 + k's first dense position (relative) and its segment */
    const uint32_t rk = lane < m ? (uint32_t)(offs[i0 + lane] - base) : 0xFFFFFFFFu;
    const uint64_t sk = lane < m ? (uint64_t)mult * vb.offsets[i0 + lane] : 0ull;
    for (uint64_t p0 = 0; p0 < keep; p0 += 64u) {
        const uint32_t p = (uint32_t)p0 + lane;
        uint32_t k = 0; /* the last instance starting at or before p */
#pragma unroll
        for (uint32_t step = 16u; step; step >>= 1) {
            const uint32_t t = k + step;
            const uint32_t o = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(t << 2), (int)rk);
            k = o <= p ? t : k; /* lanes >= m hold 0xFFFFFFFF: never taken */
        }
        const uint32_t rkk = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)rk);
        const uint32_t slo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)(uint32_t)sk);
        const uint32_t shi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)(uint32_t)(sk >> 32));
        /* the step's 64 records staged in LDS as 24-B records, then out as three
         * contiguous 512-B runs of 8-B words (the lanes' own 24-B records would be
         * three stores strided by 24 B) */
        const uint32_t nrec = keep - p0 < 64u ? (uint32_t)(keep - p0) : 64u;
        if (lane < nrec) {
            const uint4 r = seg[(((uint64_t)shi << 32) | slo) + (p - rkk)];
            stage[3u * lane] = make_uint2(r.x, r.y);
            stage[3u * lane + 1u] = make_uint2(i0 + k, r.z);
            stage[3u * lane + 2u] = make_uint2(r.w, 0u);
        }
        __builtin_amdgcn_wave_barrier();
        uint2* const q = reinterpret_cast<uint2*>(out + base + p0);
#pragma unroll
        for (uint32_t j = 0; j < 3u; ++j) {
            const uint32_t x = 64u * j + lane;
            if (x < 3u * nrec) q[x] = stage[x];
        }
        __builtin_amdgcn_wave_barrier();
    }
}

/* The emit pass, one WAVE per instance (columns aligned: codes / round / type 4 B,
 * value 16 B): the instance in 256-vote passes, lane l holding votes w + 4l ..
 * w + 4l + 3 (coalesced 4-B / 16-B loads).  Per pass: each vote's record count
 * (skip + has), one wave scan for the record slots; per (round, type) key present,
 * the value slot after each vote (round_votes.rs:50-54: the last non-nil value the
 * key's bucket took, at or before the vote) from the lane's own earlier votes, else
 * the last earlier lane holding one (ballot + bpermute), else the slot carried from
 * the pass before (LDS); then the records, consecutive lanes' records adjacent. */
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false); /* row_shr:1 */
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false); /* row_shr:2 */
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false); /* row_shr:4 */
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false); /* row_shr:8 */
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false); /* row_bcast:15 */
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false); /* row_bcast:31 */
    return x;
}

/* one pass's columns of a lane: votes j0 .. j0 + 3 (zeros / NIL past n_votes) */
struct Pass {
    uint32_t c4, r4, t4, v[4];
};
__device__ __forceinline__ void load_pass(const EvArgs& a, uint64_t j0, uint64_t NV, Pass& p) {
    p.c4 = p.r4 = p.t4 = 0u;
    p.v[0] = p.v[1] = p.v[2] = p.v[3] = AGNES_NIL;
    if (j0 + 4u <= NV) {
        p.c4 = *reinterpret_cast<const uint32_t*>(a.codes + j0);
        p.r4 = *reinterpret_cast<const uint32_t*>(a.vb.round + j0);
        p.t4 = *reinterpret_cast<const uint32_t*>(a.vb.type + j0);
        const uint4 q = *reinterpret_cast<const uint4*>(a.vb.value + j0);
        p.v[0] = q.x;
        p.v[1] = q.y;
        p.v[2] = q.z;
        p.v[3] = q.w;
    } else {
#pragma unroll
        for (uint32_t s = 0; s < 4u; ++s)
            if (j0 + s < NV) {
                p.c4 |= (uint32_t)a.codes[j0 + s] << (8u * s);
                p.r4 |= (uint32_t)a.vb.round[j0 + s] << (8u * s);
                p.t4 |= (uint32_t)a.vb.type[j0 + s] << (8u * s);
                p.v[s] = a.vb.value[j0 + s];
            }
    }
}

/* waves over the instances (i = wave, wave + W, ...; the launcher gives every
 * instance its own wave, which measured faster than a resident persistent grid:
 * 1.03 vs 1.31 ms on C2), each instance in 256-vote passes; the next pass is loaded
 * before the current one is processed, so its latency hides behind the compute and
 * the record stores */
__global__ __launch_bounds__(256) void event_emit_wave(EvArgs a) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t W = gridDim.x * 4u;
    uint32_t i = blockIdx.x * 4u + wave;
    const uint32_t n = a.vb.n_instances;
    if (i >= n) return; /* wave-uniform */
    uint32_t* const lab = reinterpret_cast<uint32_t*>(agnes_smem) + wave * a.keys;
    const uint64_t NV = a.vb.n_votes;
    auto bounds = [&](uint32_t k, uint64_t& lo, uint64_t& hi) {
        lo = a.vb.offsets[k];
        hi = a.vb.offsets[k + 1u];
        lo = lo < NV ? lo : NV;
        hi = hi < NV ? hi : NV;
    };
    uint64_t lo, hi;
    bounds(i, lo, hi);
    uint64_t w = lo & ~3ull;
    Pass cur;
    load_pass(a, w + 4u * lane, NV, cur);
    uint64_t cnt = a.offs[i];
    uint64_t lim = min(a.offs[i + 1u], a.cap); /* the instance's records end there */
    uint32_t drop = 0;
    bool fresh = true;
    for (;;) {
        if (fresh) { /* VoteCount::new for every key: Value{} */
            for (uint32_t k = lane; k < a.keys; k += 64u) lab[k] = 0u;
            __builtin_amdgcn_wave_barrier();
            fresh = false;
        }
        /* the next pass: this instance's, or the first of the wave's next instance */
        uint32_t ni = i;
        uint64_t nw = w + 256u, nlo = lo, nhi = hi, ncnt = 0, nlim = 0;
        if (nw >= hi) {
            ni = i + W;
            if (ni < n) {
                bounds(ni, nlo, nhi);
                nw = nlo & ~3ull;
                ncnt = a.offs[ni];
                nlim = min(a.offs[ni + 1u], a.cap);
            }
        }
        Pass nxt;
        if (ni < n) load_pass(a, nw + 4u * lane, NV, nxt);
        if (w < hi) {
            const uint64_t j0 = w + 4u * lane;
            /* per vote: key (0xFFFFFFFF: no record, no value write), record count */
            uint32_t key[4], n_rec = 0, recs = 0; /* recs: 2 bits per vote (skip, has) */
#pragma unroll
            for (uint32_t s = 0; s < 4u; ++s) {
                const uint64_t j = j0 + s;
                const uint32_t cb = (cur.c4 >> (8u * s)) & 0xFFu, ev = cb & AGNES_CODE_EVENT_MASK;
                const uint32_t rb = (cur.r4 >> (8u * s)) & 0xFFu, tb = (cur.t4 >> (8u * s)) & 0xFFu;
                const uint32_t k = rb * 2u + tb;
                const bool in = j >= lo && j < hi && ev != AGNES_CODE_INVALID && ev != AGNES_CODE_REJECTED &&
                                tb <= 1u && k < a.keys;
                key[s] = in ? k : 0xFFFFFFFFu;
                const uint32_t skip = in ? (cb >> 3) & 1u : 0u, has = (in && ev != AGNES_CODE_NONE) ? 1u : 0u;
                recs |= (skip | (has << 1)) << (2u * s);
                n_rec += skip + has;
            }
            const uint32_t incl = wave_scan_incl(n_rec);
            const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
            /* the value slot after each vote, per key present */
            uint32_t slot[4] = {0u, 0u, 0u, 0u};
            uint32_t pend = (key[0] != 0xFFFFFFFFu ? 1u : 0u) | (key[1] != 0xFFFFFFFFu ? 2u : 0u) |
                            (key[2] != 0xFFFFFFFFu ? 4u : 0u) | (key[3] != 0xFFFFFFFFu ? 8u : 0u);
            for (;;) {
                const uint64_t lm = __builtin_amdgcn_ballot_w64(pend != 0u);
                if (!lm) break;
                const uint32_t kl = (uint32_t)__builtin_ctzll(lm);
                const uint32_t ks = (uint32_t)__builtin_ctz(__builtin_amdgcn_readlane(pend, kl));
                const uint32_t kv = ks == 0u ? key[0] : (ks == 1u ? key[1] : (ks == 2u ? key[2] : key[3]));
                const uint32_t K = __builtin_amdgcn_readlane(kv, kl);
                uint32_t inb = 0, last = 0, hasv = 0;
#pragma unroll
                for (uint32_t s = 0; s < 4u; ++s) {
                    const bool m = key[s] == K;
                    inb |= m ? 1u << s : 0u;
                    const bool nv = m && cur.v[s] != AGNES_NIL;
                    last = nv ? cur.v[s] : last;
                    hasv |= nv ? 1u : 0u;
                }
                pend &= ~inb;
                const uint64_t M = __builtin_amdgcn_ballot_w64(hasv != 0u);
                const uint64_t before = M & ((1ull << lane) - 1ull);
                const uint32_t src = before ? 63u - (uint32_t)__builtin_clzll(before) : 0u;
                const uint32_t from_lane = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)last);
                uint32_t run = before ? from_lane : lab[K];
#pragma unroll
                for (uint32_t s = 0; s < 4u; ++s) {
                    if (key[s] == K) {
                        if (cur.v[s] != AGNES_NIL) run = cur.v[s];
                        slot[s] = run;
                    }
                }
                if (M) { /* the slot after the pass: the last lane holding a non-nil value of K */
                    const uint32_t hl = 63u - (uint32_t)__builtin_clzll(M);
                    const uint32_t nl = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(hl << 2), (int)last);
                    __builtin_amdgcn_wave_barrier();
                    if (lane == 0u) lab[K] = nl;
                }
                __builtin_amdgcn_wave_barrier();
            }
            /* the records, in stream order */
            uint64_t o = cnt + (incl - n_rec);
#pragma unroll
            for (uint32_t s = 0; s < 4u; ++s) {
                const uint32_t two = (recs >> (2u * s)) & 3u;
                if (two) {
                    const uint32_t cb = (cur.c4 >> (8u * s)) & 0xFFu, ev = cb & AGNES_CODE_EVENT_MASK;
                    const uint32_t rb = (cur.r4 >> (8u * s)) & 0xFFu, msg = cb >> AGNES_CODE_MSG_SHIFT;
                    const uint64_t j = j0 + s;
                    if ((two & 1u) && in_cap(o, lim, drop)) put(a.out + o, j, i, AGNES_NIL, rb, AGNES_EV_ROUND_SKIP, msg);
                    o += two & 1u;
                    if (two & 2u) {
                        const bool val = ev == AGNES_CODE_POLKA_VALUE || ev == AGNES_CODE_PRECOMMIT_VALUE;
                        if (in_cap(o, lim, drop)) put(a.out + o, j, i, val ? slot[s] : AGNES_NIL, rb, kind_of(ev), msg);
                        ++o;
                    }
                }
            }
            cnt += total;
        }
        if (ni >= n) break;
        if (ni != i) { /* the wave's next instance */
            i = ni;
            lo = nlo;
            hi = nhi;
            cnt = ncnt;
            lim = nlim;
            fresh = true;
        }
        w = nw;
        cur = nxt;
    }
    flush_drops(a.ovf, drop);
}

/* ---- the batch-stream emit (aligned columns): a wave walks a batch of up to EB
 * consecutive instances as ONE vote stream, so a short instance (C2: 200 votes) no
 * longer leaves most of a pass idle; the next pass (this batch's, or the first of
 * the wave's next batch, whose offsets were loaded one batch ahead) is loaded while
 * the current one is processed ---------------------------------------------------- */
constexpr uint32_t EB = 32u; /* instances per batch (offsets in lanes 0..EB) */
#ifndef EV_STAGE
#define EV_STAGE 256u /* records a pass stages in LDS (6 KB per wave) */
#endif
#ifndef EV_PREFETCH
#define EV_PREFETCH 1
#endif

/* a batch's offsets in lanes 0..m (clamped to n_votes): the loads, then the
 * wave-uniform bounds once they are needed */
struct EvRaw {
    uint32_t olo, ohi;
};
struct EvBatch {
    uint32_t s0, m, olo, ohi;
    uint64_t O0, Om;
};
__device__ __forceinline__ EvRaw ev_load(const EvArgs& a, uint32_t b, uint32_t lane) {
    const uint32_t n = a.vb.n_instances, s0 = b * EB, m = n - s0 < EB ? n - s0 : EB;
    const uint64_t NV = a.vb.n_votes;
    uint64_t o = 0;
    if (lane <= m) {
        o = a.vb.offsets[s0 + lane];
        o = o < NV ? o : NV;
    }
    return EvRaw{(uint32_t)o, (uint32_t)(o >> 32)};
}
__device__ __forceinline__ EvBatch ev_batch(const EvArgs& a, uint32_t b, EvRaw r) {
    EvBatch B;
    const uint32_t n = a.vb.n_instances;
    B.s0 = b * EB;
    B.m = n - B.s0 < EB ? n - B.s0 : EB;
    B.olo = r.olo;
    B.ohi = r.ohi;
    B.O0 = ((uint64_t)__builtin_amdgcn_readlane(B.ohi, 0) << 32) | (uint32_t)__builtin_amdgcn_readlane(B.olo, 0);
    B.Om = ((uint64_t)__builtin_amdgcn_readlane(B.ohi, B.m) << 32) | (uint32_t)__builtin_amdgcn_readlane(B.olo, B.m);
    return B;
}

/* inclusive max-scan over the wave (row_shr 1,2,4,8, row_bcast 15, 31) */
__device__ __forceinline__ uint32_t wave_max_incl(uint32_t x) {
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false));
    return x;
}
/* the value of lane - 1 (0 in lane 0) */
__device__ __forceinline__ uint32_t from_prev(uint32_t x, uint32_t lane) {
    const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - 1u) << 2), (int)x);
    return lane ? y : 0u;
}

/* V votes per lane (a pass is 64 V votes): byte columns as V/4 dwords, values as V u32 */
template <uint32_t V>
struct PassV {
    uint32_t c4[V / 4u], r4[V / 4u], t4[V / 4u], v[V];
};
template <uint32_t V>
__device__ __forceinline__ void load_pass_v(const EvArgs& a, uint64_t j0, uint64_t NV, PassV<V>& p) {
#pragma unroll
    for (uint32_t q = 0; q < V / 4u; ++q) p.c4[q] = p.r4[q] = p.t4[q] = 0u;
#pragma unroll
    for (uint32_t s = 0; s < V; ++s) p.v[s] = AGNES_NIL;
    if (j0 + V <= NV) {
        if constexpr (V == 8u) { /* j0 is a multiple of 8: 8-B byte-column loads, 32-B value loads */
            const uint2 c = *reinterpret_cast<const uint2*>(a.codes + j0);
            const uint2 r = *reinterpret_cast<const uint2*>(a.vb.round + j0);
            const uint2 t = *reinterpret_cast<const uint2*>(a.vb.type + j0);
            p.c4[0] = c.x; p.c4[1] = c.y;
            p.r4[0] = r.x; p.r4[1] = r.y;
            p.t4[0] = t.x; p.t4[1] = t.y;
        } else {
#pragma unroll
            for (uint32_t q = 0; q < V / 4u; ++q) {
                p.c4[q] = *reinterpret_cast<const uint32_t*>(a.codes + j0 + 4u * q);
                p.r4[q] = *reinterpret_cast<const uint32_t*>(a.vb.round + j0 + 4u * q);
                p.t4[q] = *reinterpret_cast<const uint32_t*>(a.vb.type + j0 + 4u * q);
            }
        }
#pragma unroll
        for (uint32_t q = 0; q < V / 4u; ++q) {
            const uint4 x = *reinterpret_cast<const uint4*>(a.vb.value + j0 + 4u * q);
            p.v[4u * q] = x.x;
            p.v[4u * q + 1u] = x.y;
            p.v[4u * q + 2u] = x.z;
            p.v[4u * q + 3u] = x.w;
        }
    } else {
#pragma unroll
        for (uint32_t s = 0; s < V; ++s)
            if (j0 + s < NV) {
                p.c4[s >> 2] |= (uint32_t)a.codes[j0 + s] << (8u * (s & 3u));
                p.r4[s >> 2] |= (uint32_t)a.vb.round[j0 + s] << (8u * (s & 3u));
                p.t4[s >> 2] |= (uint32_t)a.vb.type[j0 + s] << (8u * (s & 3u));
                p.v[s] = a.vb.value[j0 + s];
            }
    }
}

/* SEG (agnes_tally_records on the routes whose tally does not write the records): the
 * same pass, each record to its instance's segment instead of the dense stream, with no
 * count pass before it.  Positions are batch-relative: the pass where instance k's first
 * vote lies gives its first record's position fpos[k] (the records of the pass before
 * that vote: the lane's exclusive scan and its masks, read from the lane holding it), so
 * a record at batch-relative position d goes to seg + d + (mult * offsets[i] - fpos[k])
 * (per batch instance in LDS, where the staging area was), and at the batch's end
 * counts[i] = fpos[k + 1] - fpos[k] (the batch's total for its last instance) */
template <uint32_t V, uint32_t WPE, bool SEG = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void event_emit_stream(EvArgs a) {
    constexpr uint32_t P = 64u * V; /* votes per pass */
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t n = a.vb.n_instances, NB = (n + EB - 1u) / EB, BS = gridDim.x * 4u;
    const uint64_t NV = a.vb.n_votes;
    const uint32_t keys = a.keys, R2 = keys >> 1;
    /* per wave: the value slots [EB][keys], then the record staging area */
    uint32_t* const lab = reinterpret_cast<uint32_t*>(agnes_smem) + wave * (EB * keys + 6u * EV_STAGE);
    uint32_t* const stage = lab + EB * keys;
    uint64_t* const dl = reinterpret_cast<uint64_t*>(stage); /* (SEG) [EB] */
    uint32_t* const fpos = stage + 2u * EB;                  /* (SEG) [EB] */
    uint32_t b = blockIdx.x * 4u + wave;
    if (b >= NB) return; /* wave-uniform */
    EvBatch B = ev_batch(a, b, ev_load(a, b, lane));
    /* (SEG) the batch's first instance starts at position 0 */
    auto seg_batch = [&](const EvBatch& X) {
        if (SEG && lane == 0u) {
            fpos[0] = 0u;
            dl[0] = (uint64_t)a.mult * (((uint64_t)X.ohi << 32) | X.olo);
        }
    };
    /* (SEG) the batch's counts from its instances' first positions and its total */
    auto seg_counts = [&](const EvBatch& X, uint32_t total) {
        if constexpr (SEG) {
            __builtin_amdgcn_wave_barrier();
            const uint64_t ol = ((uint64_t)X.ohi << 32) | X.olo;
            /* an instance starting at the batch's end (no vote left) starts at the total */
            const uint32_t st = lane == 0u ? 0u : (ol >= X.Om ? total : fpos[lane < EB ? lane : 0u]);
            const uint32_t nx = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane + 1u) << 2), (int)st);
            if (lane < X.m) a.counts[X.s0 + lane] = (uint64_t)((lane + 1u < X.m ? nx : total) - st);
        }
    };
    seg_batch(B);
    uint32_t nb = b + BS;
    EvRaw NR = nb < NB ? ev_load(a, nb, lane) : EvRaw{0u, 0u};
    uint64_t ncnt = (!SEG && nb < NB) ? a.offs[nb * EB] : 0u;
    uint64_t cnt = SEG ? 0u : a.offs[B.s0]; /* the batch's first record (SEG: batch-relative) */
    /* (dense) the batch's records end at offs[its end], and out holds cap of them */
    uint64_t lim = SEG ? 0u : min(a.offs[B.s0 + B.m], a.cap);
    uint64_t nlim = (!SEG && nb < NB) ? min(a.offs[min(nb * EB + EB, n)], a.cap) : 0u;
    uint32_t drop = 0;
    uint64_t c = B.O0 & ~(uint64_t)(V - 1u);
    PassV<V> cur;
    load_pass_v<V>(a, c + V * lane, NV, cur);
    for (uint32_t k = lane; k < EB * keys; k += 64u) lab[k] = 0u; /* VoteCount::new: Value{} */
    __builtin_amdgcn_wave_barrier();
    auto byte_at = [](const uint32_t (&w)[V / 4u], uint32_t s) -> uint32_t { return (w[s >> 2] >> (8u * (s & 3u))) & 0xFFu; };
    for (;;) {
        uint64_t nc = c + P;
        const bool sw = nc >= B.Om, last = sw && nb >= NB;
        EvBatch NBt = B;
        if (sw && !last) {
            NBt = ev_batch(a, nb, NR);
            nc = NBt.O0 & ~(uint64_t)(V - 1u);
        }
        PassV<V> nxt;
        if (!last) load_pass_v<V>(a, nc + V * lane, NV, nxt);
        if (c < B.Om) {
            const uint64_t ol = ((uint64_t)B.ohi << 32) | B.olo;
            /* the pass's positions of the batch's votes, [lo, hi) (wave-uniform) */
            const uint32_t lo = B.O0 > c ? (uint32_t)(B.O0 - c) : 0u;
            const uint32_t hi = B.Om - c < P ? (uint32_t)(B.Om - c) : P;
            const uint32_t p0 = V * lane;
            /* per vote: batch instance (the count of the batch's later instances starting at
             * or before it: ballots over the offsets' lanes) */
            uint32_t kk[V];
            {
                /* instances 1..m-1 starting inside (c, c + P): few; every vote counts them */
                const uint64_t st = __builtin_amdgcn_ballot_w64(lane >= 1u && lane < B.m && ol > c && ol < c + P);
                const uint64_t pre = __builtin_amdgcn_ballot_w64(lane >= 1u && lane < B.m && ol <= c);
                const uint32_t k0 = (uint32_t)__builtin_popcountll(pre);
#pragma unroll
                for (uint32_t s = 0; s < V; ++s) kk[s] = k0;
                uint64_t rest = st;
                while (rest) {
                    const uint32_t k = (uint32_t)__builtin_ctzll(rest);
                    rest &= rest - 1ull;
                    const uint32_t ks = __builtin_amdgcn_readlane(B.olo, k) - (uint32_t)c; /* in (0, P) */
#pragma unroll
                    for (uint32_t s = 0; s < V; ++s) kk[s] += (p0 + s >= ks) ? 1u : 0u;
                }
            }
            /* the votes' masks, bit s = vote s: tallied (a batch vote, code not INVALID /
             * REJECTED, type <= 1, round < max_rounds), with an event, with the RoundSkip bit */
            uint32_t inm = 0, hasm = 0, skm = 0;
            {
                const int l0 = min(max((int)lo - (int)p0, 0), (int)V), h0 = min(max((int)hi - (int)p0, 0), (int)V);
                const uint32_t inr = ((1u << h0) - 1u) & ~((1u << l0) - 1u);
                auto nib = [](uint32_t x) { return ((x * 0x01020408u) >> 24) & 0xFu; };
#pragma unroll
                for (uint32_t q = 0; q < V / 4u; ++q) {
                    const uint32_t e4 = cur.c4[q] & 0x07070707u;
                    const uint32_t okev = ~((e4 + 0x02020202u) >> 3) & 0x01010101u;
                    const uint32_t tx = cur.t4[q] & 0xFEFEFEFEu;
                    const uint32_t okt = ~((((tx & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | tx) >> 7) & 0x01010101u;
                    const uint32_t okr = (~(((cur.r4[q] | 0x80808080u) - R2 * 0x01010101u) | cur.r4[q]) >> 7) & 0x01010101u;
                    const uint32_t in4 = nib(okev & okt & okr) << (4u * q);
                    inm |= in4;
                    hasm |= in4 & (nib((e4 | (e4 >> 1) | (e4 >> 2)) & 0x01010101u) << (4u * q));
                    skm |= in4 & (nib((cur.c4[q] >> 3) & 0x01010101u) << (4u * q));
                }
                inm &= inr;
                hasm &= inr;
                skm &= inr;
            }
            const uint32_t n_rec = (uint32_t)__builtin_popcount(hasm) + (uint32_t)__builtin_popcount(skm);
            uint32_t key[V], rid[V];
            /* the run check: (instance, round) non-decreasing over the pass's tallied votes */
            uint32_t rmax = 0u, bad = 0u, rfirst = 0xFFFFFFFFu;
            uint32_t lv[2] = {0u, 0u}, lr[2] = {0u, 0u}, fr[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
#pragma unroll
            for (uint32_t s = 0; s < V; ++s) {
                const uint32_t rb = byte_at(cur.r4, s), tb = byte_at(cur.t4, s) & 1u;
                const bool in = (inm >> s) & 1u;
                key[s] = in ? kk[s] * keys + rb * 2u + tb : 0xFFFFFFFFu;
                /* run id + 1 (0: not tallied) */
                rid[s] = in ? kk[s] * R2 + rb + 1u : 0u;
                bad |= (in && rid[s] < rmax) ? 1u : 0u;
                rmax = max(rmax, rid[s]);
                rfirst = (in && rfirst == 0xFFFFFFFFu) ? rid[s] : rfirst;
                const bool nn = in && cur.v[s] != AGNES_NIL;
                /* per type: the lane's last non-nil vote (value, run) and its first's run */
                lv[0] = (nn && !tb) ? cur.v[s] : lv[0];
                lv[1] = (nn && tb) ? cur.v[s] : lv[1];
                lr[0] = (nn && !tb) ? rid[s] : lr[0];
                lr[1] = (nn && tb) ? rid[s] : lr[1];
                fr[0] = (nn && !tb && fr[0] == 0xFFFFFFFFu) ? rid[s] : fr[0];
                fr[1] = (nn && tb && fr[1] == 0xFFFFFFFFu) ? rid[s] : fr[1];
            }
            const uint32_t incl = wave_scan_incl(n_rec);
            if constexpr (SEG) {
                /* the first positions of the batch's instances starting in this pass */
                uint64_t rest = __builtin_amdgcn_ballot_w64(lane >= 1u && lane < B.m && ol >= c && ol < c + P);
                const uint32_t ex = incl - n_rec;
                while (rest) {
                    const uint32_t k = (uint32_t)__builtin_ctzll(rest);
                    rest &= rest - 1ull;
                    const uint32_t ks = (uint32_t)__builtin_amdgcn_readlane(B.olo, k) - (uint32_t)c; /* [0, P) */
                    const uint32_t L = ks / V, below = (1u << (ks % V)) - 1u;
                    const uint32_t pos = (uint32_t)cnt + (uint32_t)__builtin_amdgcn_readlane(ex, L) +
                                         (uint32_t)__builtin_popcount((uint32_t)__builtin_amdgcn_readlane(hasm, L) & below) +
                                         (uint32_t)__builtin_popcount((uint32_t)__builtin_amdgcn_readlane(skm, L) & below);
                    const uint64_t okk = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(B.ohi, k) << 32) |
                                         (uint32_t)__builtin_amdgcn_readlane(B.olo, k);
                    if (lane == 0u) {
                        fpos[k] = pos;
                        dl[k] = (uint64_t)a.mult * okk - pos;
                    }
                }
                __builtin_amdgcn_wave_barrier();
            }
            uint32_t slot[V];
#pragma unroll
            for (uint32_t s = 0; s < V; ++s) slot[s] = 0u;
            /* runs: one scan per type instead of a pass per key */
            const uint32_t pmax = from_prev(wave_max_incl(rmax), lane);
            bad |= (rfirst != 0xFFFFFFFFu && rfirst < pmax) ? 1u : 0u;
            if (!__builtin_amdgcn_ballot_w64(bad != 0u)) {
                /* per type: the last earlier lane holding a non-nil vote, (run << 6 | lane) */
                uint32_t cr[2], cv[2], tail_nx[2];
#pragma unroll
                for (uint32_t t = 0; t < 2u; ++t) {
                    const uint32_t Pm = lr[t] ? (lr[t] << 6) | lane : 0u;
                    const uint32_t E = from_prev(wave_max_incl(Pm), lane);
                    cr[t] = E >> 6;
                    cv[t] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((E & 63u) << 2), (int)lv[t]);
                    /* the next lane holding a non-nil vote of type t: its first run (a tail test) */
                    const uint64_t M = __builtin_amdgcn_ballot_w64(lr[t] != 0u) & ~((2ull << lane) - 1ull);
                    const uint32_t nl = M ? (uint32_t)__builtin_ctzll(M) : lane;
                    const uint32_t f = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(nl << 2), (int)fr[t]);
                    tail_nx[t] = M ? f : 0u;
                }
                /* per vote, in order: its own value, the run's last in this pass, or the carry */
                uint32_t wr = 0u; /* votes that are the last non-nil of their (run, type) in the pass */
#pragma unroll
                for (uint32_t s = 0; s < V; ++s) {
                    if (rid[s]) {
                        const uint32_t tb = byte_at(cur.t4, s) & 1u;
                        const uint32_t r_t = tb ? cr[1] : cr[0], v_t = tb ? cv[1] : cv[0];
                        if (cur.v[s] != AGNES_NIL) {
                            slot[s] = cur.v[s];
                            if (tb) { cr[1] = rid[s]; cv[1] = cur.v[s]; } else { cr[0] = rid[s]; cv[0] = cur.v[s]; }
                            wr |= 1u << s;
                        } else {
                            slot[s] = r_t == rid[s] ? v_t : lab[key[s]];
                        }
                    }
                }
                /* a non-nil vote is its (run, type)'s last in the pass unless a later one of the
                 * lane, or the next lane's first of that type, has the same run: scanning the
                 * lane's votes backwards, the next non-nil vote of each type */
                {
                    uint32_t nx[2] = {tail_nx[0], tail_nx[1]};
#pragma unroll
                    for (int s = (int)V - 1; s >= 0; --s) {
                        if ((wr >> s) & 1u) {
                            const uint32_t tb = byte_at(cur.t4, (uint32_t)s) & 1u;
                            const uint32_t nxr = tb ? nx[1] : nx[0];
                            if (nxr == rid[s]) wr &= ~(1u << s);
                            if (tb) nx[1] = rid[s]; else nx[0] = rid[s];
                        }
                    }
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (uint32_t s = 0; s < V; ++s)
                    if ((wr >> s) & 1u) lab[key[s]] = cur.v[s];
                __builtin_amdgcn_wave_barrier();
            } else {
                /* rounds revisited inside the pass: one pass per (instance, round, type) present
                 * (round_votes.rs:50-54: the last non-nil value its bucket took) */
                uint32_t pend = 0;
#pragma unroll
                for (uint32_t s = 0; s < V; ++s) pend |= (key[s] != 0xFFFFFFFFu ? 1u : 0u) << s;
                for (;;) {
                    const uint64_t lm = __builtin_amdgcn_ballot_w64(pend != 0u);
                    if (!lm) break;
                    const uint32_t kl = (uint32_t)__builtin_ctzll(lm);
                    const uint32_t ks = (uint32_t)__builtin_ctz(__builtin_amdgcn_readlane(pend, kl));
                    uint32_t kv = key[0];
#pragma unroll
                    for (uint32_t s = 1; s < V; ++s) kv = ks == s ? key[s] : kv;
                    const uint32_t K = __builtin_amdgcn_readlane(kv, kl);
                    uint32_t inb = 0, lastv = 0, hasv = 0;
#pragma unroll
                    for (uint32_t s = 0; s < V; ++s) {
                        const bool mm = key[s] == K;
                        inb |= mm ? 1u << s : 0u;
                        const bool nv = mm && cur.v[s] != AGNES_NIL;
                        lastv = nv ? cur.v[s] : lastv;
                        hasv |= nv ? 1u : 0u;
                    }
                    pend &= ~inb;
                    const uint64_t M = __builtin_amdgcn_ballot_w64(hasv != 0u);
                    const uint64_t bef = M & ((1ull << lane) - 1ull);
                    const uint32_t src = bef ? 63u - (uint32_t)__builtin_clzll(bef) : 0u;
                    const uint32_t from_lane = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)lastv);
                    uint32_t run = bef ? from_lane : lab[K];
#pragma unroll
                    for (uint32_t s = 0; s < V; ++s) {
                        if (key[s] == K) {
                            if (cur.v[s] != AGNES_NIL) run = cur.v[s];
                            slot[s] = run;
                        }
                    }
                    if (M) {
                        const uint32_t hl = 63u - (uint32_t)__builtin_clzll(M);
                        const uint32_t nl = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(hl << 2), (int)lastv);
                        __builtin_amdgcn_wave_barrier();
                        if (lane == 0u) lab[K] = nl;
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
            /* the records in stream order: through the staging area and out as coalesced 8-B
             * stores (a record is 3 of them), or straight out when the pass has more than
             * the area holds */
            const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
            /* (dense) the pass's records that fit below lim; the rest dropped and counted */
            const uint32_t fit = SEG ? total : (cnt >= lim ? 0u : (lim - cnt < total ? (uint32_t)(lim - cnt) : total));
            if (!SEG && fit < total && lane == 0u) drop += total - fit;
            const bool staged = !SEG && total <= EV_STAGE;
            auto emit = [&](agnes_vote_event* dst) {
                uint32_t o = incl - n_rec;
#pragma unroll
                for (uint32_t s = 0; s < V; ++s) {
                    const uint32_t two = ((skm >> s) & 1u) | (((hasm >> s) & 1u) << 1);
                    if (two) {
                        const uint32_t cb = byte_at(cur.c4, s), ev = cb & AGNES_CODE_EVENT_MASK;
                        const uint32_t rb = byte_at(cur.r4, s), msg = cb >> AGNES_CODE_MSG_SHIFT;
                        const uint64_t j = c + p0 + s;
                        const uint32_t inst = B.s0 + kk[s];
                        if ((two & 1u) && o < fit) put(dst + o, j, inst, AGNES_NIL, rb, AGNES_EV_ROUND_SKIP, msg);
                        o += two & 1u;
                        if (two & 2u) {
                            const bool val = ev == AGNES_CODE_POLKA_VALUE || ev == AGNES_CODE_PRECOMMIT_VALUE;
                            if (o < fit) put(dst + o, j, inst, val ? slot[s] : AGNES_NIL, rb, kind_of(ev), msg);
                            ++o;
                        }
                    }
                }
            };
            if constexpr (SEG) {
                uint32_t o = incl - n_rec;
#pragma unroll
                for (uint32_t s = 0; s < V; ++s) {
                    const uint32_t two = ((skm >> s) & 1u) | (((hasm >> s) & 1u) << 1);
                    if (two) {
                        const uint32_t cb = byte_at(cur.c4, s), ev = cb & AGNES_CODE_EVENT_MASK;
                        const uint32_t rb = byte_at(cur.r4, s), msg = cb >> AGNES_CODE_MSG_SHIFT;
                        const uint64_t j = c + p0 + s;
                        uint4* const d = a.seg + (cnt + o + dl[kk[s]]);
                        if (two & 1u) put_seg(d, j, AGNES_NIL, rb, AGNES_EV_ROUND_SKIP, msg);
                        if (two & 2u) {
                            const bool val = ev == AGNES_CODE_POLKA_VALUE || ev == AGNES_CODE_PRECOMMIT_VALUE;
                            put_seg(d + (two & 1u), j, val ? slot[s] : AGNES_NIL, rb, kind_of(ev), msg);
                        }
                        o += (two & 1u) + (two >> 1);
                    }
                }
            } else if (staged) /* (two instantiations: LDS stores here, global ones below) */
                emit(reinterpret_cast<agnes_vote_event*>(stage));
            else
                emit(a.out + cnt);
            if (staged) {
                __builtin_amdgcn_wave_barrier();
                uint2* const out8 = reinterpret_cast<uint2*>(a.out + cnt);
                for (uint32_t w8 = lane; w8 < 3u * fit; w8 += 64u) out8[w8] = reinterpret_cast<const uint2*>(stage)[w8];
                __builtin_amdgcn_wave_barrier();
            }
            cnt += total;
        }
        if (sw) seg_counts(B, (uint32_t)cnt);
        if (last) break;
        if (sw) { /* the wave's next batch */
            b = nb;
            B = NBt;
            cnt = ncnt;
            lim = nlim;
            nb = b + BS;
            if (nb < NB) {
                NR = ev_load(a, nb, lane);
                ncnt = SEG ? 0u : a.offs[nb * EB];
                nlim = SEG ? 0u : min(a.offs[min(nb * EB + EB, n)], a.cap);
            }
            __builtin_amdgcn_wave_barrier();
            for (uint32_t k = lane; k < EB * keys; k += 64u) lab[k] = 0u;
            seg_batch(B);
            __builtin_amdgcn_wave_barrier();
        }
        c = nc;
        cur = nxt;
    }
    if (!SEG) flush_drops(a.ovf, drop); /* (lane 0 counted the wave's) */
}

} // namespace events
} // namespace agnes

/* ------------------------------------------------------------------ */

hipError_t agnes_launch_event_count_list(const agnes_vote_batch* vb, const uint8_t* codes, const uint32_t* walk,
                                         const uint32_t* walk_n, uint64_t* offs, int num_cus, hipStream_t st) {
    using namespace agnes::events;
    const uint32_t n = vb->n_instances;
    if (n == 0) return hipSuccess;
    EvArgs a{*vb, codes, offs, nullptr, 0u};
    /* the list is usually empty: a small grid (a block of 256 lanes per CU) that
     * strides over it */
    uint32_t blocks = (n + 255u) / 256u;
    const uint32_t cap = (uint32_t)(num_cus > 0 ? num_cus : 256);
    if (blocks > cap) blocks = cap;
    AgnesKt kt("event_count_list", st);
    if ((reinterpret_cast<uintptr_t>(codes) & 15u) == 0u)
        hipLaunchKernelGGL((event_count_list<64u>), dim3(blocks), dim3(256), 0, st, a, walk, walk_n);
    else
        hipLaunchKernelGGL((event_count_list<4u>), dim3(blocks), dim3(256), 0, st, a, walk, walk_n);
    return hipGetLastError();
}

hipError_t agnes_launch_events(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds,
                               uint64_t* offs, agnes_vote_event* out, uint64_t* scratch, hipStream_t st, uint64_t cap,
                               unsigned long long* ovf) {
    using namespace agnes::events;
    const uint32_t n = vb->n_instances;
    EvArgs a{*vb, codes, offs, out, 2u * max_rounds, nullptr, nullptr, 0u, cap, ovf};
    const dim3 grid((n + 63u) / 64u), blk(64);
    if (!out) { /* pass 1: counts (codes only), then the scan */
        hipError_t e = hipMemsetAsync(offs, 0, sizeof(uint64_t), st);
        if (e != hipSuccess || n == 0) return e;
        {
            AgnesKt kt("event_count", st);
            if ((reinterpret_cast<uintptr_t>(codes) & 15u) == 0u) /* 64-B windows when aligned */
                hipLaunchKernelGGL((event_walk<false, 64u, true>), grid, blk, 0, st, a);
            else
                hipLaunchKernelGGL((event_walk<false, 4u, false>), grid, blk, 0, st, a);
        }
        AgnesKt kt("event_scan", st);
        return agnes_launch_offsets_scan(offs, n, scratch, st);
    }
    if (n == 0) return hipSuccess;
    const size_t lds = (size_t)a.keys * 64u * sizeof(uint32_t);
    const bool a16 = ((reinterpret_cast<uintptr_t>(codes) | reinterpret_cast<uintptr_t>(vb->round) |
                       reinterpret_cast<uintptr_t>(vb->type) | reinterpret_cast<uintptr_t>(vb->value)) & 15u) == 0u;
    AgnesKt kt("event_emit", st);
    if (a16 && a.keys <= 64u) {
        /* batches of EB instances as one stream per wave; a resident grid (the blocks a
         * CU holds x 256 CUs), so each wave walks several batches and prefetches across them */
        const uint32_t NB = (n + EB - 1u) / EB;
        const size_t lds_s = (size_t)4u * (EB * a.keys + 6u * EV_STAGE) * sizeof(uint32_t);
/* 4 votes per lane (256-vote passes).  8 (512-vote passes, 4 waves per SIMD)
         * measured: C2 0.80 vs 0.78 ms, C3 2.94 vs 3.02, C4 1.90 vs ~1.4 (its next-round
         * votes send more passes to the per-key path, and a wider pass holds more keys) */
        const void* fn = reinterpret_cast<const void*>(&event_emit_stream<4u, 5u>);
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds_s) != hipSuccess || per_cu < 1)
            per_cu = 1;
        const uint32_t cap = EV_PREFETCH ? 256u * (uint32_t)per_cu : 0xFFFFFFFFu;
        const uint32_t sblocks = (NB + 3u) / 4u < cap ? (NB + 3u) / 4u : cap;
        hipLaunchKernelGGL((event_emit_stream<4u, 5u>), dim3(sblocks), dim3(256), lds_s, st, a);
    } else if (a16) {
        /* one wave per instance, coalesced; the next pass of a long instance is loaded
         * while the current one is processed */
        const size_t lds_w = (size_t)4u * a.keys * sizeof(uint32_t);
        const uint32_t blocks = (n + 3u) / 4u;
        hipLaunchKernelGGL(event_emit_wave, dim3(blocks), dim3(256), lds_w, st, a);
    } else
        hipLaunchKernelGGL((event_walk<true, 4u, false>), grid, blk, lds, st, a);
    return hipGetLastError();
}

bool agnes_seg_emit_ok(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds) {
    return ((reinterpret_cast<uintptr_t>(codes) | reinterpret_cast<uintptr_t>(vb->round) |
             reinterpret_cast<uintptr_t>(vb->type) | reinterpret_cast<uintptr_t>(vb->value)) & 15u) == 0u &&
           2u * max_rounds <= 64u;
}

hipError_t agnes_launch_seg_emit(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds, uint32_t mult,
                                 uint64_t* counts, void* seg, hipStream_t st) {
    using namespace agnes::events;
    const uint32_t n = vb->n_instances;
    if (n == 0) return hipSuccess;
    if (!agnes_seg_emit_ok(vb, codes, max_rounds)) return hipErrorInvalidValue;
    static_assert(6u * EV_STAGE >= 3u * EB, "the (SEG) per-instance deltas and positions fit the staging area");
    EvArgs a{*vb, codes, nullptr, nullptr, 2u * max_rounds, reinterpret_cast<uint4*>(seg), counts, mult};
    const uint32_t NB = (n + EB - 1u) / EB;
    const size_t lds_s = (size_t)4u * (EB * a.keys + 6u * EV_STAGE) * sizeof(uint32_t);
    const void* fn = reinterpret_cast<const void*>(&event_emit_stream<4u, 5u, true>);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, lds_s) != hipSuccess || per_cu < 1) per_cu = 1;
    const uint32_t cap = EV_PREFETCH ? 256u * (uint32_t)per_cu : 0xFFFFFFFFu;
    const uint32_t sblocks = (NB + 3u) / 4u < cap ? (NB + 3u) / 4u : cap;
    AgnesKt kt("seg_emit", st);
    hipLaunchKernelGGL((event_emit_stream<4u, 5u, true>), dim3(sblocks), dim3(256), lds_s, st, a);
    return hipGetLastError();
}

hipError_t agnes_launch_seg_walk(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds, uint32_t mult,
                                 const uint32_t* list, const uint32_t* list_n, uint64_t* counts, void* seg,
                                 hipStream_t st) {
    using namespace agnes::events;
    const uint32_t n = vb->n_instances;
    if (n == 0) return hipSuccess;
    EvArgs a{*vb, codes, nullptr, nullptr, 2u * max_rounds};
    const size_t lds = (size_t)a.keys * 64u * sizeof(uint32_t);
    /* 16-vote windows when the u8 columns are 16-B aligned, else 4-vote ones; the value
     * column is 16-B aligned (agnes_tally_records' requirement) */
    const bool w16 = ((reinterpret_cast<uintptr_t>(codes) | reinterpret_cast<uintptr_t>(vb->round) |
                       reinterpret_cast<uintptr_t>(vb->type)) & 15u) == 0u;
    const bool a16 = (reinterpret_cast<uintptr_t>(vb->value) & 15u) == 0u;
    const dim3 grid((n + 63u) / 64u), blk(64);
    uint4* const sg = reinterpret_cast<uint4*>(seg);
    AgnesKt kt("seg_walk", st);
#define AGNES_SEG_WALK(L, W_, A_) hipLaunchKernelGGL((seg_walk<L, W_, A_>), grid, blk, lds, st, a, list, list_n, mult, sg, counts)
    if (list) {
        if (w16 && a16) AGNES_SEG_WALK(true, 16u, true); else if (a16) AGNES_SEG_WALK(true, 4u, true); else AGNES_SEG_WALK(true, 4u, false);
    } else {
        if (w16 && a16) AGNES_SEG_WALK(false, 16u, true); else if (a16) AGNES_SEG_WALK(false, 4u, true); else AGNES_SEG_WALK(false, 4u, false);
    }
#undef AGNES_SEG_WALK
    return hipGetLastError();
}

hipError_t agnes_launch_seg_compact(const agnes_vote_batch* vb, uint32_t mult, const void* seg, const uint64_t* offs,
                                    agnes_vote_event* out, hipStream_t st, uint64_t cap, unsigned long long* ovf) {
    const uint32_t n = vb->n_instances;
    if (n == 0) return hipSuccess;
    const uint32_t waves = (n + 31u) / 32u, blocks = (waves + 3u) / 4u;
    AgnesKt kt("seg_compact", st);
    hipLaunchKernelGGL(agnes::events::seg_compact, dim3(blocks), dim3(256), 4u * 192u * sizeof(uint2), st, *vb, mult,
                       reinterpret_cast<const uint4*>(seg), offs, out, cap, ovf);
    return hipGetLastError();
}
