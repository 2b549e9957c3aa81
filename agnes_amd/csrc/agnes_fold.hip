/*
 * agnes_fold.hip — the fold of VoteCount partials (include/agnes.h
 * agnes_fold_counts) for one instance split into consecutive slices (C5,
 * agnes_amd/dist.py tally_one_instance): the slices' partial (round, type)
 * VoteCounts fold like consecutive add_vote calls (round_votes.rs:48-56): the
 * weights add (i64, wrapping as the reference's release build) and the value slot
 * is the later slice's when it wrote one (last writer wins, :50-54).
 *
 * One block per bucket k; each thread folds a run of consecutive slices, a block
 * scan of the runs gives every slice the fold of the slices before it, starting
 * from an optional carry-in; the slices are rewritten with that (the next pass's
 * carry-in) and the total written out.  Latency bound (S x K x 24 B): up to 8192
 * slices the runs stay in registers (fold_regs: one load batch per thread, wave
 * shuffles), beyond that the slices are read twice (fold_kernel).
 */
#include <hip/hip_runtime.h>

#include <cstdint>

#include "agnes_internal.h"

namespace agnes {
namespace fold {

constexpr uint32_t T = 256u;

struct Agg {
    uint64_t vw, nw; /* wrapping i64 sums, as u64 */
    uint32_t lab;    /* AGNES_NIL: no value written */
};

__device__ __forceinline__ Agg comb(const Agg& a, const Agg& b) {
    return Agg{a.vw + b.vw, a.nw + b.nw, b.lab != AGNES_NIL ? b.lab : a.lab};
}

__device__ __forceinline__ Agg load(const agnes_vote_count& c) {
    return Agg{(uint64_t)c.value_w, (uint64_t)c.nil_w, c.value};
}

__device__ __forceinline__ void store(agnes_vote_count& c, const Agg& a, bool nil_to_zero) {
    c.value_w = (int64_t)a.vw;
    c.nil_w = (int64_t)a.nw;
    c.value = (nil_to_zero && a.lab == AGNES_NIL) ? 0u : a.lab;
    c.reserved = 0u;
}

__global__ __launch_bounds__(T) void fold_kernel(agnes_vote_count* counts, uint32_t S, uint32_t K,
                                                 const agnes_vote_count* carry, agnes_vote_count* totals,
                                                 uint32_t flags) {
    __shared__ Agg part[T];
    const uint32_t k = blockIdx.x, t = threadIdx.x;
    const uint32_t per = (S + T - 1u) / T;
    const uint32_t s0 = t * per < S ? t * per : S, s1 = s0 + per < S ? s0 + per : S;
    if (flags & AGNES_FOLD_RESET) { /* VoteCount::new in every slice (no value written yet) */
        for (uint32_t s = s0; s < s1; ++s) store(counts[(uint64_t)s * K + k], Agg{0u, 0u, AGNES_NIL}, false);
        return;
    }
    Agg run{0u, 0u, AGNES_NIL};
    for (uint32_t s = s0; s < s1; ++s) run = comb(run, load(counts[(uint64_t)s * K + k]));
    part[t] = run;
    __syncthreads();
    /* inclusive scan of the runs (Hillis-Steele over T entries) */
    for (uint32_t d = 1; d < T; d <<= 1) {
        const Agg x = t >= d ? part[t - d] : Agg{0u, 0u, AGNES_NIL};
        __syncthreads();
        if (t >= d) part[t] = comb(x, part[t]);
        __syncthreads();
    }
    Agg base{0u, 0u, AGNES_NIL};
    if (carry) {
        base = load(carry[k]);
        if ((flags & AGNES_FOLD_CARRY_ZERO_NONE) && base.lab == 0u) base.lab = AGNES_NIL;
    }
    if (flags & AGNES_FOLD_APPLY) { /* each slice := carry-in + the slices before it */
        Agg pre = comb(base, t ? part[t - 1u] : Agg{0u, 0u, AGNES_NIL});
        for (uint32_t s = s0; s < s1; ++s) {
            agnes_vote_count& c = counts[(uint64_t)s * K + k];
            const Agg own = load(c);
            store(c, pre, (flags & AGNES_FOLD_ZERO_LABELS) != 0u);
            pre = comb(pre, own);
        }
    }
    if (totals && t == T - 1u) store(totals[k], comb(base, part[T - 1u]), (flags & AGNES_FOLD_TOTAL_ZERO_LABELS) != 0u);
}

/* The same fold with the slices in registers (S <= TR * PR, one block of TR threads
 * per bucket): every slice is loaded once, in one batch per thread, and the block
 * scan is wave shuffles plus one LDS step over the 16 waves. */
constexpr uint32_t TR = 1024u, PR = 8u;

__device__ __forceinline__ Agg shfl_up(const Agg& a, uint32_t d) {
    return Agg{(uint64_t)__shfl_up((unsigned long long)a.vw, d, 64), (uint64_t)__shfl_up((unsigned long long)a.nw, d, 64),
               (uint32_t)__shfl_up((unsigned int)a.lab, d, 64)};
}

__global__ __launch_bounds__(TR) void fold_regs(agnes_vote_count* counts, uint32_t S, uint32_t K,
                                                const agnes_vote_count* carry, agnes_vote_count* totals,
                                                uint32_t flags) {
    __shared__ Agg wpart[TR / 64u];
    const uint32_t k = blockIdx.x, t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const Agg id{0u, 0u, AGNES_NIL};
    const uint32_t per = (S + TR - 1u) / TR;
    const uint32_t s0 = t * per < S ? t * per : S, s1 = s0 + per < S ? s0 + per : S;
    Agg v[PR];
#pragma unroll
    for (uint32_t i = 0; i < PR; ++i) v[i] = s0 + i < s1 ? load(counts[(uint64_t)(s0 + i) * K + k]) : id;
    Agg run = id;
#pragma unroll
    for (uint32_t i = 0; i < PR; ++i) run = comb(run, v[i]);
    /* inclusive scan over the wave, then the waves before this one */
    Agg inc = run;
    for (uint32_t d = 1; d < 64u; d <<= 1) {
        const Agg o = shfl_up(inc, d);
        if (lane >= d) inc = comb(o, inc);
    }
    if (lane == 63u) wpart[wv] = inc;
    __syncthreads();
    Agg pre = id;
    if (carry) {
        pre = load(carry[k]);
        if ((flags & AGNES_FOLD_CARRY_ZERO_NONE) && pre.lab == 0u) pre.lab = AGNES_NIL;
    }
    for (uint32_t i = 0; i < wv; ++i) pre = comb(pre, wpart[i]);
    const Agg ex = shfl_up(inc, 1u);
    if (lane) pre = comb(pre, ex);
    if (flags & AGNES_FOLD_APPLY) { /* each slice := carry-in + the slices before it */
#pragma unroll
        for (uint32_t i = 0; i < PR; ++i) {
            if (s0 + i < s1) {
                store(counts[(uint64_t)(s0 + i) * K + k], pre, (flags & AGNES_FOLD_ZERO_LABELS) != 0u);
                pre = comb(pre, v[i]);
            }
        }
    } else {
        pre = comb(pre, run);
    }
    if (totals && t == TR - 1u) store(totals[k], pre, (flags & AGNES_FOLD_TOTAL_ZERO_LABELS) != 0u);
}

} // namespace fold
} // namespace agnes

hipError_t agnes_launch_fold(agnes_vote_count* counts, uint32_t n_slices, uint32_t keys,
                             const agnes_vote_count* carry, agnes_vote_count* totals, uint32_t flags,
                             hipStream_t st) {
    if (keys == 0) return hipSuccess;
    AgnesKt kt("fold", st);
    using namespace agnes::fold;
    if (!(flags & AGNES_FOLD_RESET) && (uint64_t)n_slices <= (uint64_t)TR * PR)
        hipLaunchKernelGGL(fold_regs, dim3(keys), dim3(TR), 0, st, counts, n_slices, keys, carry, totals, flags);
    else
        hipLaunchKernelGGL(fold_kernel, dim3(keys), dim3(T), 0, st, counts, n_slices, keys, carry, totals, flags);
    return hipGetLastError();
}
