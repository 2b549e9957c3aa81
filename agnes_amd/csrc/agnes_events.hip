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
 * Two walks, one instance per lane (as the edge summary): a count pass over the
 * codes (1 B per vote), the exclusive scan of the counts (agnes_edges.hip), and an
 * emit pass that follows each executor's value slot in LDS ([key][lane], a wave's
 * 64 lookups on 64 banks) over codes, round, type and value (7 B per vote) and
 * writes 24-B records at the scanned offsets.  HBM bound.
 */
#include <hip/hip_runtime.h>

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
};

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

template <bool EMIT, uint32_t W, bool A16>
__global__ __launch_bounds__(64) void event_walk(EvArgs a) {
    uint32_t* const lab = reinterpret_cast<uint32_t*>(agnes_smem);
    const uint32_t lane = threadIdx.x;
    const uint32_t i = blockIdx.x * 64u + lane;
    if (i >= a.vb.n_instances) return;
    if (EMIT)
        for (uint32_t k = 0; k < a.keys; ++k) lab[k * 64u + lane] = 0u; /* VoteCount::new: Value{} */
    const uint64_t NV = a.vb.n_votes;
    uint64_t lo = a.vb.offsets[i], hi = a.vb.offsets[i + 1u];
    lo = lo < NV ? lo : NV;
    hi = hi < NV ? hi : NV;
    const uint64_t base = EMIT ? a.offs[i] : 0u;
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
            if (!EMIT) {
                cnt += skip + has;
                continue;
            }
            const uint32_t rb = (r[b >> 2] >> sh8) & 0xFFu, tb = (t[b >> 2] >> sh8) & 0xFFu;
            const uint32_t key = rb * 2u + tb;
            if (tb > 1u || key >= a.keys) continue; /* (never for a code the tally wrote) */
            uint32_t* const p = lab + key * 64u + lane;
            if (v[b] != AGNES_NIL) *p = v[b]; /* the value slot, last writer wins */
            const uint32_t msg = cb >> AGNES_CODE_MSG_SHIFT;
            if (skip) put(a.out + base + cnt++, j, i, AGNES_NIL, rb, AGNES_EV_ROUND_SKIP, msg);
            if (has) {
                const bool val = ev == AGNES_CODE_POLKA_VALUE || ev == AGNES_CODE_PRECOMMIT_VALUE;
                put(a.out + base + cnt++, j, i, val ? *p : AGNES_NIL, rb, kind_of(ev), msg);
            }
        }
    }
    if (!EMIT) a.offs[i + 1u] = cnt;
}

} // namespace events
} // namespace agnes

/* ------------------------------------------------------------------ */

hipError_t agnes_launch_events(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds,
                               uint64_t* offs, agnes_vote_event* out, uint64_t* scratch, hipStream_t st) {
    using namespace agnes::events;
    const uint32_t n = vb->n_instances;
    EvArgs a{*vb, codes, offs, out, 2u * max_rounds};
    const dim3 grid((n + 63u) / 64u), blk(64);
    if (!out) { /* pass 1: counts (codes only, 64-B windows when aligned), then the scan */
        hipError_t e = hipMemsetAsync(offs, 0, sizeof(uint64_t), st);
        if (e != hipSuccess || n == 0) return e;
        {
            AgnesKt kt("event_count", st);
            if ((reinterpret_cast<uintptr_t>(codes) & 15u) == 0u)
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
    if (a16) hipLaunchKernelGGL((event_walk<true, 16u, true>), grid, blk, lds, st, a);
    else hipLaunchKernelGGL((event_walk<true, 4u, false>), grid, blk, lds, st, a);
    return hipGetLastError();
}
