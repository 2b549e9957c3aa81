/*
 * agnes_edges.hip — edge-triggered summary of a coded batch (SURVEY.md §8(f) 1;
 * include/agnes.h agnes_edge_offsets / agnes_edges).
 *
 * VoteExecutor::apply (vote_executor.rs:20-36) is level-triggered: after a
 * threshold holds, every later vote of the executor repeats the event, and
 * State::apply repeats its Timeout messages the same way (state_machine.rs:196,
 * 208).  The summary keeps, per instance, the votes that change their (round,
 * type) executor's level (code bits 0..3) or carry a message (bits 4..7) other
 * than the executor's last one.  The (round, type) executors of an instance are the HeightVotes the
 * reference leaves as a stub (consensus_executor.rs:5; vote_executor.rs:9,14).
 *
 * Two walks of the codes, one instance per lane (like apply_codes): a count pass
 * that writes each instance's edge count, an exclusive scan of the counts (three
 * small kernels), and an emit pass that writes 16-B records at the scanned
 * offsets — ordered by instance then vote, deterministic.  Each lane keeps one
 * byte per executor (level | last message << 4) in LDS, [slot][lane] (slot = key /
 * 4, key = round * 2 + type), so a wave's 64 lookups hit 64 banks.  Each lane reads 64-B
 * windows of each column (four 16-B loads of one line in flight together).  HBM
 * bound: 3 B per vote read per pass (code, round, type) + 16 B per edge written.
 */
#include <hip/hip_runtime.h>

#include <cstdint>

#include "agnes_device.h"
#include "agnes_internal.h"

namespace agnes {
namespace edges {

struct EdgeArgs {
    agnes_vote_batch vb;
    const uint8_t* codes;
    uint64_t* offs;   /* n_instances + 1 */
    agnes_edge* out;
    uint32_t keys;    /* 2 * max_rounds */
    uint32_t nslots;  /* ceil(keys / 4) byte words per lane */
    /* (the dense emit) out holds cap records; an edge past cap or past its instance's end
     * offset is dropped and counted in *ovf (agnes_records_overflow) */
    uint64_t cap;
    unsigned long long* ovf;
};

template <uint32_t W>
__device__ __forceinline__ void load_win(const uint8_t* col, uint64_t w, uint64_t NV, uint32_t (&v)[W / 4u]) {
    if (w + W <= NV) {
        if constexpr (W >= 16u) { /* W/16 16-B loads of one line, in flight together */
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
    } else { /* the batch's last window: its real bytes only */
#pragma unroll
        for (uint32_t d = 0; d < W / 4u; ++d) v[d] = 0u;
        for (uint32_t b = 0; b < W && w + b < NV; ++b) v[b >> 2] |= (uint32_t)col[w + b] << (8u * (b & 3u));
    }
}

/* REG: up to 8 executors (keys < 8, max_rounds <= 4): their bytes live in one u64
 * register (byte key), not in LDS — the read-modify-write of a vote's executor byte
 * is then a 64-bit shift and xor, not an LDS round trip the next vote of the same
 * executor waits on */
template <bool EMIT, uint32_t W, bool REG>
__device__ __forceinline__ uint64_t walk_one(const EdgeArgs& a, uint32_t i, uint32_t lane, uint64_t base,
                                             uint64_t lim = ~0ull) {
    uint32_t* const tab = reinterpret_cast<uint32_t*>(agnes_smem);
    uint64_t st = 0; /* (REG) VoteCount::new: level 0 */
    if (!REG)
        for (uint32_t s = 0; s < a.nslots; ++s) tab[s * 64u + lane] = 0u; /* VoteCount::new: level 0 */
    const uint64_t NV = a.vb.n_votes;
    uint64_t lo = a.vb.offsets[i], hi = a.vb.offsets[i + 1u];
    lo = lo < NV ? lo : NV;
    hi = hi < NV ? hi : NV;
    uint64_t cnt = 0;
    for (uint64_t w = lo & ~(uint64_t)(W - 1u); w < hi; w += W) {
        uint32_t c[W / 4u], r[W / 4u], t[W / 4u];
        load_win<W>(a.codes, w, NV, c);
        load_win<W>(a.vb.round, w, NV, r);
        load_win<W>(a.vb.type, w, NV, t);
#pragma unroll
        for (uint32_t b = 0; b < W; ++b) {
            const uint64_t j = w + b;
            const uint32_t sh8 = 8u * (b & 3u);
            const uint32_t cb = (c[b >> 2] >> sh8) & 0xFFu, rb = (r[b >> 2] >> sh8) & 0xFFu,
                           tb = (t[b >> 2] >> sh8) & 0xFFu;
            const uint32_t ev = cb & AGNES_CODE_EVENT_MASK;
            const uint32_t key = rb * 2u + tb;
            /* outside the instance, INVALID / REJECTED (never counted), or no executor */
            if (j < lo || j >= hi || ev == AGNES_CODE_INVALID || ev == AGNES_CODE_REJECTED || tb > 1u ||
                key >= a.keys)
                continue;
            /* the executor's byte: level (bits 0..3) | last message (bits 4..7) */
            uint32_t* const p = tab + (key >> 2) * 64u + lane;
            const uint32_t x = REG ? 0u : *p, sh = REG ? 8u * key : 8u * (key & 3u);
            const uint32_t old = REG ? (uint32_t)(st >> sh) & 0xFFu : (x >> sh) & 0xFFu;
            const uint32_t msg = cb >> AGNES_CODE_MSG_SHIFT;
            const uint32_t nb = (cb & 0xFu) | (msg ? msg << AGNES_CODE_MSG_SHIFT : old & 0xF0u);
            if (nb != old) {
                if (EMIT && base + cnt < lim) {
                    const uint32_t tail = rb | (tb << 8) | (cb << 16) | (old << 24);
                    *reinterpret_cast<uint4*>(a.out + base + cnt) =
                        make_uint4((uint32_t)j, (uint32_t)(j >> 32), i, tail);
                }
                ++cnt;
                if (REG) st ^= (uint64_t)(old ^ nb) << sh;
                else *p = x ^ ((old ^ nb) << sh);
            }
        }
    }
    return cnt;
}

template <bool EMIT, uint32_t W, bool REG>
__global__ __launch_bounds__(64) void edge_walk(EdgeArgs a) {
    const uint32_t lane = threadIdx.x;
    const uint32_t i = blockIdx.x * 64u + lane;
    if (i >= a.vb.n_instances) return;
    if (EMIT) { /* (the count that did not fit below lim: dropped) */
        const uint64_t o = a.offs[i], lim = min(a.offs[i + 1u], a.cap);
        const uint64_t cnt = walk_one<true, W, REG>(a, i, lane, o, lim);
        const uint64_t kept = o >= lim ? 0u : (cnt < lim - o ? cnt : lim - o);
        if (kept < cnt) atomicAdd(a.ovf, (unsigned long long)(cnt - kept));
    } else {
        a.offs[i + 1u] = walk_one<false, W, REG>(a, i, lane, 0u);
    }
}

/* the segmented edges (agnes_tally_edges) of every instance, or of the ones on a list
 * (the flow route's walk list): instance i's at out[offsets[i] + k], k < counts[i]
 * (a vote is at most one edge), one lane per instance, the same windowed walk */
template <bool LIST, uint32_t W, bool REG>
__global__ __launch_bounds__(64) void edge_seg_walk(EdgeArgs a, const uint32_t* list, const uint32_t* list_n,
                                                    uint64_t* counts) {
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
    counts[i] = walk_one<true, W, REG>(a, i, lane, a.vb.offsets[i]);
}

/* the dense summary from the segmented one: wave w writes the edges of instances
 * 32w .. 32w + 31 -- one contiguous range, offs[32w] .. offs[32w + 32] -- 64 at a time,
 * lane l the edge at position p: its instance by a 5-step binary search over the
 * wave's offsets (one per lane, relative to the range's start), then one 16-B read of
 * that instance's segment and one 16-B store (a few edges per instance: one instance
 * per step left most lanes idle) */
__global__ __launch_bounds__(256) void edge_compact(agnes_vote_batch vb, const agnes_edge* seg, const uint64_t* offs,
                                                    agnes_edge* out, uint64_t cap, unsigned long long* ovf) {
    const uint32_t lane = threadIdx.x & 63u, w = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t n = vb.n_instances, i0 = 32u * w;
    if (i0 >= n) return; /* wave-uniform */
    const uint32_t m = n - i0 < 32u ? n - i0 : 32u;
    /* the wave's range bounded by out's capacity (the edges past cap dropped, counted) */
    const uint64_t base = offs[i0], end = offs[i0 + m];
    const uint64_t tot = end > base ? end - base : 0u;
    const uint64_t total = base >= cap ? 0u : (tot < cap - base ? tot : cap - base);
    if (lane == 0u && total < tot) atomicAdd(ovf, (unsigned long long)(tot - total));
    if (total > 0xFFFFFF00ull) { /* positions past u32 (4e9 edges in 32 instances): per instance */
        for (uint32_t i = i0; i < i0 + m; ++i) {
            const uint64_t o = offs[i], oe = offs[i + 1u] < base + total ? offs[i + 1u] : base + total;
            if (o >= oe) continue;
            const uint64_t cnt = oe - o;
            const uint4* const s = reinterpret_cast<const uint4*>(seg + vb.offsets[i]);
            for (uint64_t k = lane; k < cnt; k += 64u) reinterpret_cast<uint4*>(out + o)[k] = s[k];
        }
        return;
    }
    const uint32_t rk = lane < m ? (uint32_t)(offs[i0 + lane] - base) : 0xFFFFFFFFu;
    const uint64_t sk = lane < m ? vb.offsets[i0 + lane] : 0ull;
    const uint4* const src = reinterpret_cast<const uint4*>(seg);
    uint4* const dst = reinterpret_cast<uint4*>(out + base);
    for (uint64_t p0 = 0; p0 < total; p0 += 64u) {
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
        if ((uint64_t)p < total) dst[p] = src[(((uint64_t)shi << 32) | slo) + (p - rkk)];
    }
}

/* window of the aligned path: 64 B per column (four 16-B loads of one 128-B line
 * issued together, so the line is fetched once although the wave's 64 lanes read
 * 64 different lines) */
#ifndef AGNES_EDGE_W
#define AGNES_EDGE_W 64
#endif
constexpr uint32_t EW = AGNES_EDGE_W;

/* ---- exclusive offsets: inclusive scan of offs[1..n] in place, three kernels ---- */
constexpr uint32_t SCAN_T = 256u, SCAN_PER = 4u, SCAN_BLK = SCAN_T * SCAN_PER;

/* inclusive scan of x[0..n) inside one 256-thread block; the block total returned */
__device__ uint64_t block_scan(uint64_t (&v)[SCAN_PER], uint64_t* wsum) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
#pragma unroll
    for (uint32_t k = 1; k < SCAN_PER; ++k) v[k] += v[k - 1u];
    const uint64_t incl = scan(v[SCAN_PER - 1u]); /* wave inclusive over the threads' sums */
    if (lane == 63u) wsum[wv] = incl;
    __syncthreads();
    uint64_t before = incl - v[SCAN_PER - 1u], total = 0;
    for (uint32_t q = 0; q < SCAN_T / 64u; ++q) {
        if (q < wv) before += wsum[q];
        total += wsum[q];
    }
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; ++k) v[k] += before;
    __syncthreads(); /* wsum reusable */
    return total;
}

__global__ __launch_bounds__(SCAN_T) void scan_blocks(uint64_t* x, uint64_t n, uint64_t* part) {
    __shared__ uint64_t wsum[SCAN_T / 64u];
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_BLK + threadIdx.x * SCAN_PER;
    uint64_t v[SCAN_PER];
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; ++k) v[k] = b0 + k < n ? x[b0 + k] : 0u;
    const uint64_t total = block_scan(v, wsum);
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; ++k)
        if (b0 + k < n) x[b0 + k] = v[k];
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

/* one block: exclusive scan of the block totals in place */
__global__ __launch_bounds__(SCAN_T) void scan_parts(uint64_t* part, uint64_t nb) {
    __shared__ uint64_t wsum[SCAN_T / 64u];
    uint64_t carry = 0;
    for (uint64_t c0 = 0; c0 < nb; c0 += SCAN_BLK) {
        const uint64_t b0 = c0 + threadIdx.x * SCAN_PER;
        uint64_t v[SCAN_PER], in[SCAN_PER];
#pragma unroll
        for (uint32_t k = 0; k < SCAN_PER; ++k) in[k] = v[k] = b0 + k < nb ? part[b0 + k] : 0u;
        const uint64_t total = block_scan(v, wsum);
#pragma unroll
        for (uint32_t k = 0; k < SCAN_PER; ++k)
            if (b0 + k < nb) part[b0 + k] = carry + v[k] - in[k];
        carry += total;
    }
}

__global__ __launch_bounds__(SCAN_T) void scan_add(uint64_t* x, uint64_t n, const uint64_t* part) {
    const uint64_t add = part[blockIdx.x];
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_BLK + threadIdx.x * SCAN_PER;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_PER; ++k)
        if (b0 + k < n) x[b0 + k] += add;
}

} // namespace edges
} // namespace agnes

/* ------------------------------------------------------------------ */

hipError_t agnes_launch_offsets_scan(uint64_t* offs, uint32_t n, uint64_t* scratch, hipStream_t st) {
    using namespace agnes::edges;
    const uint64_t nb = agnes_edges_scratch_words(n);
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(scan_blocks, dim3((uint32_t)nb), dim3(SCAN_T), 0, st, offs + 1, (uint64_t)n, scratch);
    if (nb > 1u) {
        hipLaunchKernelGGL(scan_parts, dim3(1), dim3(SCAN_T), 0, st, scratch, nb);
        hipLaunchKernelGGL(scan_add, dim3((uint32_t)nb), dim3(SCAN_T), 0, st, offs + 1, (uint64_t)n, scratch);
    }
    return hipGetLastError();
}

uint64_t agnes_edges_scratch_words(uint32_t n_instances) {
    return ((uint64_t)n_instances + agnes::edges::SCAN_BLK - 1u) / agnes::edges::SCAN_BLK;
}

hipError_t agnes_launch_edges(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds,
                              uint64_t* offs, agnes_edge* out, uint64_t* scratch, hipStream_t st, uint64_t cap,
                              unsigned long long* ovf) {
    using namespace agnes::edges;
    const uint32_t n = vb->n_instances;
    EdgeArgs a{*vb, codes, offs, out, 2u * max_rounds, (2u * max_rounds + 3u) / 4u, cap, ovf};
    /* 16-B windows when the three columns allow them */
    const bool w16 = ((reinterpret_cast<uintptr_t>(codes) | reinterpret_cast<uintptr_t>(vb->round) |
                       reinterpret_cast<uintptr_t>(vb->type)) & 15u) == 0u;
    const dim3 grid((n + 63u) / 64u), blk(64);
    const bool reg = a.keys <= 8u; /* every executor byte in one u64 register */
    const size_t lds = reg ? 0u : (size_t)a.nslots * 64u * sizeof(uint32_t);
    if (!out) { /* pass 1: counts, then the exclusive scan */
        hipError_t e = hipMemsetAsync(offs, 0, sizeof(uint64_t), st);
        if (e != hipSuccess || n == 0) return e;
        {
            AgnesKt kt("edge_count", st);
            if (reg) {
                if (w16) hipLaunchKernelGGL((edge_walk<false, EW, true>), grid, blk, lds, st, a);
                else hipLaunchKernelGGL((edge_walk<false, 4u, true>), grid, blk, lds, st, a);
            } else {
                if (w16) hipLaunchKernelGGL((edge_walk<false, EW, false>), grid, blk, lds, st, a);
                else hipLaunchKernelGGL((edge_walk<false, 4u, false>), grid, blk, lds, st, a);
            }
        }
        AgnesKt kt("edge_scan", st);
        return agnes_launch_offsets_scan(offs, n, scratch, st);
    }
    if (n == 0) return hipSuccess;
    AgnesKt kt("edge_emit", st);
    if (reg) {
        if (w16) hipLaunchKernelGGL((edge_walk<true, EW, true>), grid, blk, lds, st, a);
        else hipLaunchKernelGGL((edge_walk<true, 4u, true>), grid, blk, lds, st, a);
    } else {
        if (w16) hipLaunchKernelGGL((edge_walk<true, EW, false>), grid, blk, lds, st, a);
        else hipLaunchKernelGGL((edge_walk<true, 4u, false>), grid, blk, lds, st, a);
    }
    return hipGetLastError();
}

hipError_t agnes_launch_edge_seg_walk(const agnes_vote_batch* vb, const uint8_t* codes, uint32_t max_rounds,
                                      const uint32_t* list, const uint32_t* list_n, uint64_t* counts, agnes_edge* seg,
                                      hipStream_t st) {
    using namespace agnes::edges;
    const uint32_t n = vb->n_instances;
    if (n == 0) return hipSuccess;
    EdgeArgs a{*vb, codes, nullptr, seg, 2u * max_rounds, (2u * max_rounds + 3u) / 4u};
    const bool w16 = ((reinterpret_cast<uintptr_t>(codes) | reinterpret_cast<uintptr_t>(vb->round) |
                       reinterpret_cast<uintptr_t>(vb->type)) & 15u) == 0u;
    const bool reg = a.keys <= 8u;
    const size_t lds = reg ? 0u : (size_t)a.nslots * 64u * sizeof(uint32_t);
    const dim3 grid((n + 63u) / 64u), blk(64);
    AgnesKt kt("edge_seg_walk", st);
#define AGNES_EDGE_SEG(L, W_, R_) hipLaunchKernelGGL((edge_seg_walk<L, W_, R_>), grid, blk, lds, st, a, list, list_n, counts)
    if (list) {
        if (reg) { if (w16) AGNES_EDGE_SEG(true, EW, true); else AGNES_EDGE_SEG(true, 4u, true); }
        else { if (w16) AGNES_EDGE_SEG(true, EW, false); else AGNES_EDGE_SEG(true, 4u, false); }
    } else {
        if (reg) { if (w16) AGNES_EDGE_SEG(false, EW, true); else AGNES_EDGE_SEG(false, 4u, true); }
        else { if (w16) AGNES_EDGE_SEG(false, EW, false); else AGNES_EDGE_SEG(false, 4u, false); }
    }
#undef AGNES_EDGE_SEG
    return hipGetLastError();
}

hipError_t agnes_launch_edge_compact(const agnes_vote_batch* vb, const agnes_edge* seg, const uint64_t* offs,
                                     agnes_edge* out, hipStream_t st, uint64_t cap, unsigned long long* ovf) {
    const uint32_t n = vb->n_instances;
    if (n == 0) return hipSuccess;
    const uint32_t waves = (n + 31u) / 32u, blocks = (waves + 3u) / 4u;
    AgnesKt kt("edge_compact", st);
    hipLaunchKernelGGL(agnes::edges::edge_compact, dim3(blocks), dim3(256), 0, st, *vb, seg, offs, out, cap, ovf);
    return hipGetLastError();
}
