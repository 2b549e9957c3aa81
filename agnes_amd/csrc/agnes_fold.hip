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
 * carry-in) and the total written out.  Latency bound (S x K x 24 B).
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

} // namespace fold
} // namespace agnes

hipError_t agnes_launch_fold(agnes_vote_count* counts, uint32_t n_slices, uint32_t keys,
                             const agnes_vote_count* carry, agnes_vote_count* totals, uint32_t flags,
                             hipStream_t st) {
    if (keys == 0) return hipSuccess;
    AgnesKt kt("fold", st);
    hipLaunchKernelGGL(agnes::fold::fold_kernel, dim3(keys), dim3(agnes::fold::T), 0, st, counts, n_slices, keys,
                       carry, totals, flags);
    return hipGetLastError();
}
