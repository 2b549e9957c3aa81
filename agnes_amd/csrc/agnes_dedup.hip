/*
 * agnes_dedup.hip — DEDUP mode for ONE instance split over segments and ranks
 * (C5, SURVEY.md §8(e): "DEDUP mode adds an all-reduce(min) of first_index").
 *
 * DEDUP keeps the first vote of each (round, type, validator) and rejects the
 * rest (include/agnes.h AGNES_MODE_DEDUP; the checker's orc_tally).  When one
 * instance's stream is cut into slices, a vote's slice cannot tell whether an
 * earlier slice saw its key, so the split path finds the first vote of every key
 * up front:
 *   1. agnes_dedup_first — every valid vote j of the slice atomically lowers
 *      first[key] to base + j (its index in the whole stream);
 *   2. the caller all-reduces `first` with MIN over the ranks (agnes_amd/dist.py);
 *   3. agnes_dedup_mask — a copy of the type column in which every valid vote that
 *      is not its key's first carries AGNES_TYPE_MASKED: the carried tally (REFERENCE
 *      semantics) then skips it like an invalid vote, so it neither adds weight nor
 *      writes a label (round_votes.rs:48-56 is never reached for it);
 *   4. agnes_dedup_reject — after the tally, the masked votes' codes INVALID ->
 *      REJECTED.
 * Validity is the tally's: instance id == the instance, round < max_rounds,
 * type <= 1, set < n_sets, validator < n_vals.  All HBM-streaming, one vote per
 * lane, coalesced; first[] is 8 B per (round, type, validator) key.
 */
#include <hip/hip_runtime.h>

#include <cstdint>

#include "agnes_device.h"
#include "agnes_internal.h"

namespace agnes {
namespace dedup {

struct DedupArgs {
    const uint32_t* instance;
    const uint8_t* round;
    const uint8_t* type;
    const uint32_t* validator;
    uint64_t n_votes;
    uint64_t base;
    uint32_t inst_id;
    uint32_t max_rounds;
    uint32_t n_vals;
    uint32_t set_ok;
};

__device__ __forceinline__ bool valid_key(const DedupArgs& a, uint64_t j, uint64_t& key) {
    const uint32_t r = a.round[j], t = a.type[j], x = a.validator[j];
    const bool ok = a.set_ok && a.instance[j] == a.inst_id && r < a.max_rounds && t <= 1u && x < a.n_vals;
    key = ((uint64_t)r * 2u + t) * a.n_vals + x;
    return ok;
}

/* 0xFF in byte s for bit s of ok (ok < 16) */
__device__ __forceinline__ uint32_t ok_bytes(uint32_t ok) {
    const uint32_t b = (ok * 0x00204081u) & 0x01010101u;
    return (b << 8) - b;
}

/* V4: four consecutive votes per thread (instance / validator 16-B, round / type 4-B
 * aligned columns): the keys of votes j .. j+3 (j a multiple of 4), bit s of the
 * returned mask = vote j+s is valid; tb: their type bytes */
template <bool V4>
__device__ __forceinline__ uint32_t valid_keys4(const DedupArgs& a, uint64_t j, uint64_t (&key)[4], uint32_t& tb) {
    uint32_t ok = 0;
    tb = 0;
    if (V4 && j + 4u <= a.n_votes) {
        const uint4 in = *reinterpret_cast<const uint4*>(a.instance + j);
        const uint4 vx = *reinterpret_cast<const uint4*>(a.validator + j);
        const uint32_t r4 = *reinterpret_cast<const uint32_t*>(a.round + j);
        const uint32_t t4 = *reinterpret_cast<const uint32_t*>(a.type + j);
        tb = t4;
        const uint32_t ins[4] = {in.x, in.y, in.z, in.w}, xs[4] = {vx.x, vx.y, vx.z, vx.w};
#pragma unroll
        for (uint32_t s = 0; s < 4u; ++s) {
            const uint32_t r = (r4 >> (8u * s)) & 0xFFu, t = (t4 >> (8u * s)) & 0xFFu, x = xs[s];
            key[s] = ((uint64_t)r * 2u + t) * a.n_vals + x;
            ok |= (a.set_ok && ins[s] == a.inst_id && r < a.max_rounds && t <= 1u && x < a.n_vals) ? 1u << s : 0u;
        }
    } else {
#pragma unroll
        for (uint32_t s = 0; s < 4u; ++s) {
            key[s] = 0;
            if (j + s < a.n_votes) {
                if (valid_key(a, j + s, key[s])) ok |= 1u << s;
                tb |= (uint32_t)a.type[j + s] << (8u * s);
            }
        }
    }
    return ok;
}

__global__ __launch_bounds__(256) void first_kernel(DedupArgs a, unsigned long long* first) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a.n_votes; j += stride) {
        uint64_t key;
        if (valid_key(a, j, key)) atomicMin(first + key, (unsigned long long)(a.base + j));
    }
}

template <bool V4>
__global__ __launch_bounds__(256) void mask_kernel(DedupArgs a, const unsigned long long* first, uint8_t* type_out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    if (V4) { /* four votes per thread; the keys' first-index gathers issued together */
        for (uint64_t j = 4u * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x); j < a.n_votes; j += 4u * stride) {
            uint64_t key[4];
            uint32_t tb;
            const uint32_t ok = valid_keys4<true>(a, j, key, tb);
            unsigned long long f[4];
#pragma unroll
            for (uint32_t s = 0; s < 4u; ++s) f[s] = ((ok >> s) & 1u) ? first[key[s]] : 0ull;
            uint32_t o = 0;
#pragma unroll
            for (uint32_t s = 0; s < 4u; ++s) {
                const uint32_t t = j + s < a.n_votes ? a.type[j + s] : 0u;
                const uint32_t b = ((ok >> s) & 1u) ? (f[s] == a.base + j + s ? t : AGNES_TYPE_MASKED) : 0xFFu;
                o |= b << (8u * s);
            }
            if (j + 4u <= a.n_votes) *reinterpret_cast<uint32_t*>(type_out + j) = o;
            else
                for (uint32_t s = 0; s < 4u && j + s < a.n_votes; ++s) type_out[j + s] = (uint8_t)(o >> (8u * s));
        }
        return;
    }
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a.n_votes; j += stride) {
        uint64_t key;
        const uint32_t t = a.type[j];
        uint32_t o;
        /* a vote failing the DEDUP checks is INVALID in the one-stream DEDUP tally
         * (oracle orc_tally: DEDUP needs its validator); 0xFF makes the carried
         * REFERENCE tally reject it too, whatever column it reads (a weight column
         * does not look at the validator) */
        if (valid_key(a, j, key)) o = first[key] == a.base + j ? t : AGNES_TYPE_MASKED;
        else o = 0xFFu;
        type_out[j] = (uint8_t)o;
    }
}

__global__ __launch_bounds__(256) void fill_kernel(uint64_t* first, uint64_t n) { /* INT64_MAX: no vote yet */
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) first[k] = 0x7FFFFFFFFFFFFFFFull;
}

__global__ __launch_bounds__(256) void reject_kernel(const uint8_t* type_masked, uint64_t n, uint8_t* codes) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride)
        if (type_masked[j] == AGNES_TYPE_MASKED) codes[j] = AGNES_CODE_REJECTED;
}

/* ---- the first-index table without global atomics (round 4) ----
 * One device-scope atomicMin per vote on a random line of a 16 MB table runs at
 * the memory side's atomic rate (C5d: 2.4M atomics, 0.094 ms).  Instead the valid
 * votes are counting-sorted by key bucket (KB consecutive keys, one block's LDS
 * table each) and every bucket's minimum is taken with LDS atomics:
 *   count    block g of G (BV votes each): an LDS histogram over the buckets,
 *            written to cnt[b * G + g];
 *   prefix   block b: its row of cnt as an exclusive scan (the offset of each
 *            block's votes inside the bucket) and the row's total;
 *   scatter  block g: the bucket starts (an exclusive scan of the row totals in
 *            LDS; block 0 writes them out), the block's valid votes sorted by
 *            bucket in LDS, then written as {key % KB, j} (8 B) runs per bucket;
 *   min      block b: an LDS table of KB u32 indices, atomicMin per entry, then
 *            first[key] = min(first[key], base + index) for its keys (coalesced).
 * About 10 + 10 + 8 + 8 B per vote plus the table's read and write. */
#ifndef AGNES_DEDUP_KB
#define AGNES_DEDUP_KB 8192
#endif
constexpr uint32_t KB = AGNES_DEDUP_KB; /* keys per bucket (32 KB of LDS indices) */
constexpr uint32_t MAX_NB = 1024u; /* buckets (LDS histograms)               */
#ifndef AGNES_DEDUP_BV
#define AGNES_DEDUP_BV 4096
#endif
constexpr uint32_t BV = AGNES_DEDUP_BV; /* votes per count / scatter block */
static_assert((KB & (KB - 1u)) == 0u && KB * 4u <= 64u * 1024u, "AGNES_DEDUP_KB: a power of two, its LDS table <= 64 KiB");
static_assert(BV % 4u == 0u && BV * 8u <= 64u * 1024u, "AGNES_DEDUP_BV: a multiple of 4, its LDS stage <= 64 KiB");

/* exclusive scan of x[0..n) in LDS, n <= 1024, by a 256-thread block; the total into x[n] */
__device__ void lds_scan_1024(uint32_t* x, uint32_t n) {
    __shared__ uint32_t wsum[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint32_t v[4], s = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
        const uint32_t i = 4u * t + k;
        v[k] = i < n ? x[i] : 0u;
        s += v[k];
    }
    const uint32_t incl = scan(s);
    if (lane == 63u) wsum[w] = incl;
    __syncthreads();
    uint32_t before = incl - s, total = 0;
    for (uint32_t q = 0; q < 4u; ++q) {
        before += q < w ? wsum[q] : 0u;
        total += wsum[q];
    }
#pragma unroll
    for (uint32_t k = 0; k < 4u; ++k) {
        const uint32_t i = 4u * t + k;
        if (i < n) x[i] = before;
        before += v[k];
    }
    if (t == 0u) x[n] = total;
    __syncthreads();
}

template <bool V4>
__global__ __launch_bounds__(256) void bucket_count(DedupArgs a, uint32_t nb, uint32_t G, uint32_t* cnt) {
    __shared__ uint32_t hist[MAX_NB];
    const uint32_t g = blockIdx.x;
    for (uint32_t b = threadIdx.x; b < nb; b += 256u) hist[b] = 0u;
    __syncthreads();
    const uint64_t j0 = (uint64_t)g * BV, j1 = j0 + BV < a.n_votes ? j0 + BV : a.n_votes;
    for (uint64_t j = j0 + 4u * threadIdx.x; j < j1; j += 1024u) {
        uint64_t key[4];
        uint32_t tb;
        const uint32_t ok = valid_keys4<V4>(a, j, key, tb);
#pragma unroll
        for (uint32_t s = 0; s < 4u; ++s)
            if ((ok >> s) & 1u) atomicAdd(&hist[(uint32_t)(key[s] / KB)], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += 256u) cnt[(uint64_t)b * G + g] = hist[b];
}

/* row b of cnt -> its exclusive scan in place, the row total into rowtot[b] */
__global__ __launch_bounds__(256) void bucket_prefix(uint32_t G, uint32_t* cnt, uint32_t* rowtot) {
    __shared__ uint32_t wsum[4];
    uint32_t* const row = cnt + (uint64_t)blockIdx.x * G;
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < G; c0 += 256u) {
        const uint32_t i = c0 + t;
        const uint32_t v = i < G ? row[i] : 0u;
        const uint32_t incl = scan(v);
        if (lane == 63u) wsum[w] = incl;
        __syncthreads();
        uint32_t before = incl - v, total = 0;
        for (uint32_t q = 0; q < 4u; ++q) {
            before += q < w ? wsum[q] : 0u;
            total += wsum[q];
        }
        if (i < G) row[i] = carry + before;
        carry += total;
        __syncthreads();
    }
    if (t == 0u) rowtot[blockIdx.x] = carry;
}

/* The block's valid votes are first sorted by bucket in LDS (a local counting sort:
 * the block's per-bucket counts are its column of cnt), then written out in that
 * order, so each bucket's run of the block (~BV / nb pairs) leaves as consecutive
 * 8-B stores instead of one random line per vote.  MASK (agnes_dedup_first_mask):
 * also the mask's defaults, the vote's own type for a valid vote (the min pass
 * writes AGNES_TYPE_MASKED over the ones that are not their key's first) and 0xFF for
 * an invalid one. */
template <bool V4, bool MASK>
__global__ __launch_bounds__(256) void bucket_scatter(DedupArgs a, uint32_t nb, uint32_t G, const uint32_t* cnt,
                                                      const uint32_t* rowtot, uint32_t* bstart, uint2* pairs,
                                                      uint8_t* type_out) {
    __shared__ uint32_t cur[MAX_NB + 1u]; /* the block's first global slot per bucket */
    __shared__ uint32_t lst[MAX_NB + 1u]; /* the block's local start per bucket       */
    __shared__ uint32_t lcur[MAX_NB];     /* local slot cursors                       */
    __shared__ uint2 stage[BV];
    __shared__ uint16_t sbk[BV];
    const uint32_t g = blockIdx.x;
    for (uint32_t b = threadIdx.x; b < nb; b += 256u) cur[b] = rowtot[b];
    __syncthreads();
    lds_scan_1024(cur, nb); /* cur[b] = the bucket's start */
    if (g == 0u)
        for (uint32_t b = threadIdx.x; b <= nb; b += 256u) bstart[b] = cur[b];
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += 256u) {
        const uint32_t o = cnt[(uint64_t)b * G + g]; /* the block's offset inside the bucket */
        const uint32_t o1 = g + 1u < G ? cnt[(uint64_t)b * G + g + 1u] : rowtot[b];
        cur[b] += o;
        lst[b] = o1 - o; /* the block's count, scanned below */
    }
    __syncthreads();
    lds_scan_1024(lst, nb);
    for (uint32_t b = threadIdx.x; b < nb; b += 256u) lcur[b] = lst[b];
    __syncthreads();
    const uint64_t j0 = (uint64_t)g * BV, j1 = j0 + BV < a.n_votes ? j0 + BV : a.n_votes;
    for (uint64_t j = j0 + 4u * threadIdx.x; j < j1; j += 1024u) {
        uint64_t key[4];
        uint32_t tb;
        const uint32_t ok = valid_keys4<V4>(a, j, key, tb);
#pragma unroll
        for (uint32_t s = 0; s < 4u; ++s) {
            if ((ok >> s) & 1u) {
                const uint32_t bk = (uint32_t)(key[s] / KB);
                const uint32_t p = atomicAdd(&lcur[bk], 1u);
                stage[p] = make_uint2((uint32_t)(key[s] % KB), (uint32_t)(j + s));
                sbk[p] = (uint16_t)bk;
            }
        }
        if (MASK) {
            const uint32_t m = ok_bytes(ok);
            const uint32_t o = (tb & m) | ~m;
            if (V4 && j + 4u <= a.n_votes) *reinterpret_cast<uint32_t*>(type_out + j) = o;
            else
                for (uint32_t s = 0; s < 4u && j + s < j1; ++s) type_out[j + s] = (uint8_t)(o >> (8u * s));
        }
    }
    __syncthreads();
    const uint32_t tot = lst[nb];
    for (uint32_t i = threadIdx.x; i < tot; i += 256u) {
        const uint32_t bk = sbk[i];
        pairs[cur[bk] + (i - lst[bk])] = stage[i];
    }
}

constexpr uint32_t MT = 1024u; /* threads of a min block (one block per CU) */
template <bool MASK>
__global__ __launch_bounds__(MT) void bucket_min(uint64_t n_keys, const uint32_t* bstart, const uint2* pairs,
                                                 uint64_t base, unsigned long long* first, uint8_t* type_out) {
    __shared__ uint32_t tab[KB];
    const uint32_t b = blockIdx.x;
    for (uint32_t k = threadIdx.x; k < KB; k += MT) tab[k] = 0xFFFFFFFFu;
    __syncthreads();
    const uint32_t e0 = bstart[b], e1 = bstart[b + 1u];
    for (uint32_t e = e0 + threadIdx.x; e < e1; e += MT) {
        const uint2 q = pairs[e];
        atomicMin(&tab[q.x], q.y);
    }
    __syncthreads();
    const uint64_t k0 = (uint64_t)b * KB;
    for (uint32_t k = threadIdx.x; k < KB && k0 + k < n_keys; k += MT) {
        const uint32_t x = tab[k];
        if (MASK) { /* agnes_dedup_first_mask: the table written whole (no caller fill, no read) */
            first[k0 + k] = x != 0xFFFFFFFFu ? base + x : 0x7FFFFFFFFFFFFFFFull;
        } else if (x != 0xFFFFFFFFu) { /* agnes_dedup_first: lowered */
            const unsigned long long v = base + x, old = first[k0 + k];
            if (v < old) first[k0 + k] = v;
        }
    }
    if (MASK) { /* AGNES_TYPE_MASKED over the scatter's type for a vote that is not its key's first */
        __syncthreads();
        for (uint32_t e = e0 + threadIdx.x; e < e1; e += MT) {
            const uint2 q = pairs[e];
            if (tab[q.x] != q.y) type_out[q.y] = (uint8_t)AGNES_TYPE_MASKED;
        }
    }
}

} // namespace dedup
} // namespace agnes

/* ------------------------------------------------------------------ */

/* the columns allow four votes per thread (16-B / 4-B vector loads) */
static bool dedup_v4(const agnes_vote_batch* vb) {
    return ((reinterpret_cast<uintptr_t>(vb->instance) | reinterpret_cast<uintptr_t>(vb->validator)) & 15u) == 0u &&
           ((reinterpret_cast<uintptr_t>(vb->round) | reinterpret_cast<uintptr_t>(vb->type)) & 3u) == 0u;
}

static dim3 dedup_grid(uint64_t n) {
    uint64_t b = (n + 255u) / 256u;
    if (b > 8192u) b = 8192u;
    return dim3((uint32_t)(b ? b : 1u));
}

hipError_t agnes_launch_dedup(const agnes_vote_batch* vb, uint32_t inst_id, uint32_t max_rounds,
                              uint32_t n_vals, bool set_ok, uint64_t base, uint64_t* first,
                              uint8_t* type_out, hipStream_t st) {
    using namespace agnes::dedup;
    if (vb->n_votes == 0) return hipSuccess;
    const DedupArgs a{vb->instance, vb->round, vb->type, vb->validator, vb->n_votes,
                      base, inst_id, max_rounds, n_vals, set_ok ? 1u : 0u};
    unsigned long long* f = reinterpret_cast<unsigned long long*>(first);
    if (!type_out) {
        AgnesKt kt("dedup_first", st);
        hipLaunchKernelGGL(first_kernel, dedup_grid(vb->n_votes), dim3(256), 0, st, a, f);
    } else {
        AgnesKt kt("dedup_mask", st);
        const bool v4 = dedup_v4(vb) && (reinterpret_cast<uintptr_t>(type_out) & 3u) == 0u;
        if (v4) hipLaunchKernelGGL(mask_kernel<true>, dedup_grid((vb->n_votes + 3u) / 4u), dim3(256), 0, st, a, f, type_out);
        else hipLaunchKernelGGL(mask_kernel<false>, dedup_grid(vb->n_votes), dim3(256), 0, st, a, f, type_out);
    }
    return hipGetLastError();
}

bool agnes_dedup_bucketed(uint64_t n_votes, uint32_t max_rounds, uint32_t n_vals) {
    using namespace agnes::dedup;
    const uint64_t n_keys = 2ull * max_rounds * n_vals;
    return n_votes < (1ull << 32) && (n_keys + KB - 1u) / KB <= MAX_NB;
}

static uint32_t dedup_blocks(uint64_t n_votes) {
    return (uint32_t)((n_votes + agnes::dedup::BV - 1u) / agnes::dedup::BV);
}

uint64_t agnes_dedup_scratch_bytes(uint64_t n_votes, uint32_t max_rounds, uint32_t n_vals) {
    using namespace agnes::dedup;
    const uint64_t nb = (2ull * max_rounds * n_vals + KB - 1u) / KB, G = dedup_blocks(n_votes);
    return agnes::align16(4u * nb * G) + 2u * agnes::align16(4u * (nb + 1u)) + 8u * n_votes;
}

hipError_t agnes_launch_dedup_first_bucketed(const agnes_vote_batch* vb, uint32_t inst_id, uint32_t max_rounds,
                                             uint32_t n_vals, bool set_ok, uint64_t base, uint64_t* first,
                                             uint8_t* type_out, void* scratch, hipStream_t st) {
    using namespace agnes::dedup;
    if (vb->n_votes == 0) return hipSuccess;
    const DedupArgs a{vb->instance, vb->round, vb->type, vb->validator, vb->n_votes,
                      base, inst_id, max_rounds, n_vals, set_ok ? 1u : 0u};
    const uint64_t n_keys = 2ull * max_rounds * n_vals;
    const uint32_t nb = (uint32_t)((n_keys + KB - 1u) / KB), G = dedup_blocks(vb->n_votes);
    unsigned char* const sp = reinterpret_cast<unsigned char*>(scratch);
    const uint64_t o1 = agnes::align16(4ull * nb * G), o2 = o1 + agnes::align16(4ull * (nb + 1u)),
                   o3 = o2 + agnes::align16(4ull * (nb + 1u));
    uint32_t* const cnt = reinterpret_cast<uint32_t*>(sp);
    uint32_t* const rowtot = reinterpret_cast<uint32_t*>(sp + o1);
    uint32_t* const bstart = reinterpret_cast<uint32_t*>(sp + o2);
    uint2* const pairs = reinterpret_cast<uint2*>(sp + o3);
    const bool v4 = dedup_v4(vb) && (reinterpret_cast<uintptr_t>(type_out) & 3u) == 0u;
    unsigned long long* const f = reinterpret_cast<unsigned long long*>(first);
    AgnesKt kt(type_out ? "dedup_first_mask" : "dedup_first", st);
    if (v4) hipLaunchKernelGGL(bucket_count<true>, dim3(G), dim3(256), 0, st, a, nb, G, cnt);
    else hipLaunchKernelGGL(bucket_count<false>, dim3(G), dim3(256), 0, st, a, nb, G, cnt);
    hipLaunchKernelGGL(bucket_prefix, dim3(nb), dim3(256), 0, st, G, cnt, rowtot);
    if (type_out) {
        if (v4) hipLaunchKernelGGL((bucket_scatter<true, true>), dim3(G), dim3(256), 0, st, a, nb, G, cnt, rowtot, bstart, pairs, type_out);
        else hipLaunchKernelGGL((bucket_scatter<false, true>), dim3(G), dim3(256), 0, st, a, nb, G, cnt, rowtot, bstart, pairs, type_out);
        hipLaunchKernelGGL(bucket_min<true>, dim3(nb), dim3(MT), 0, st, n_keys, bstart, pairs, base, f, type_out);
    } else {
        if (v4) hipLaunchKernelGGL((bucket_scatter<true, false>), dim3(G), dim3(256), 0, st, a, nb, G, cnt, rowtot, bstart, pairs, type_out);
        else hipLaunchKernelGGL((bucket_scatter<false, false>), dim3(G), dim3(256), 0, st, a, nb, G, cnt, rowtot, bstart, pairs, type_out);
        hipLaunchKernelGGL(bucket_min<false>, dim3(nb), dim3(MT), 0, st, n_keys, bstart, pairs, base, f, type_out);
    }
    return hipGetLastError();
}

hipError_t agnes_launch_dedup_fill(uint64_t* first, uint64_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(agnes::dedup::fill_kernel, dedup_grid(n), dim3(256), 0, st, first, n);
    return hipGetLastError();
}

hipError_t agnes_launch_dedup_reject(const uint8_t* type_masked, uint64_t n, uint8_t* codes, hipStream_t st) {
    if (n == 0) return hipSuccess;
    AgnesKt kt("dedup_reject", st);
    hipLaunchKernelGGL(agnes::dedup::reject_kernel, dedup_grid(n), dim3(256), 0, st, type_masked, n, codes);
    return hipGetLastError();
}
