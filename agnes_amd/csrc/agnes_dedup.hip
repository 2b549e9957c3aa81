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

__global__ __launch_bounds__(256) void first_kernel(DedupArgs a, unsigned long long* first) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < a.n_votes; j += stride) {
        uint64_t key;
        if (valid_key(a, j, key)) atomicMin(first + key, (unsigned long long)(a.base + j));
    }
}

__global__ __launch_bounds__(256) void mask_kernel(DedupArgs a, const unsigned long long* first, uint8_t* type_out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
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

__global__ __launch_bounds__(256) void reject_kernel(const uint8_t* type_masked, uint64_t n, uint8_t* codes) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride)
        if (type_masked[j] == AGNES_TYPE_MASKED) codes[j] = AGNES_CODE_REJECTED;
}

} // namespace dedup
} // namespace agnes

/* ------------------------------------------------------------------ */

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
        hipLaunchKernelGGL(mask_kernel, dedup_grid(vb->n_votes), dim3(256), 0, st, a, f, type_out);
    }
    return hipGetLastError();
}

hipError_t agnes_launch_dedup_reject(const uint8_t* type_masked, uint64_t n, uint8_t* codes, hipStream_t st) {
    if (n == 0) return hipSuccess;
    AgnesKt kt("dedup_reject", st);
    hipLaunchKernelGGL(agnes::dedup::reject_kernel, dedup_grid(n), dim3(256), 0, st, type_masked, n, codes);
    return hipGetLastError();
}
