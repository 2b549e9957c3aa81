/*
 * agnes_partials.hip — pass A of the split-instance protocol as one reduction
 * (include/agnes.h agnes_tally_partials; C5, agnes_amd/dist.py tally_one_instance).
 *
 * Pass A only needs each segment's VoteCounts after its votes from
 * RoundVotes::new: add_vote (round_votes.rs:48-56) adds the vote's weight to the
 * (round, type) bucket's value or nil side and a non-nil vote writes the value
 * slot (the last writer wins).  No threshold, no per-vote code: a sum per side
 * and an arg-max of the position per key.  The carried tally (the i64 kernel with
 * its K1-K3 machinery, ~2 waves per SIMD) spent 34 us on C5's 2M votes, most of it
 * waiting on the power gathers; this kernel runs a block per segment at full
 * occupancy, so 8x as many gathers are in flight.  It also writes each vote's
 * weight (i64, 0 when the vote is not valid): pass B reads that column
 * (AGNES_FLAG_WEIGHTS_CACHED) instead of gathering the table a second time.
 *
 * Per block: the key table in LDS ([K] value weight, nil weight, label as
 * (position + 1) << 32 | value); per wave, 4 votes per lane (strided by the
 * block, coalesced), one ballot pass per key present with DPP sums, then LDS
 * atomics from one lane.  Validity is the tally's (agnes_kernels.hip prep_chunk):
 * instance id, round < max_rounds, type <= 1, set < n_sets, validator < n_vals.
 */
#include <hip/hip_runtime.h>

#include <cstdint>

#include "agnes_device.h"
#include "agnes_internal.h"

namespace agnes {
namespace partials {

constexpr uint32_t T = 256u;
constexpr uint32_t VPT = 4u; /* votes per thread per step */

struct PArgs {
    agnes_vote_batch vb;
    const int64_t* power;
    const uint32_t* power32; /* the same weights, for sets whose weights are < 2^31 */
    const agnes_set_info* sets;
    uint32_t n_sets, n_vals, keys, max_rounds;
    uint32_t one_inst, one_id;
    agnes_carry_rec* counts;
    int64_t* wout;
};

__global__ __launch_bounds__(T) void partials_kernel(PArgs a) {
    const uint32_t seg = blockIdx.x, tid = threadIdx.x, lane = tid & 63u;
    const uint32_t K = a.keys;
    unsigned long long* const vw = reinterpret_cast<unsigned long long*>(agnes_smem);
    unsigned long long* const nw = vw + K;
    unsigned long long* const lb = nw + K;
    for (uint32_t k = tid; k < K; k += T) vw[k] = nw[k] = lb[k] = 0ull;
    const agnes_vote_batch& vb = a.vb;
    const uint64_t NV = vb.n_votes;
    uint64_t beg = vb.offsets[seg], end = vb.offsets[seg + 1u];
    beg = beg < NV ? beg : NV;
    end = end < NV ? end : NV;
    end = end > beg ? end : beg;
    const uint32_t ns = a.n_sets, nv = a.n_vals;
    const uint32_t set = vb.instance_set ? vb.instance_set[seg] : (ns ? (a.one_inst ? a.one_id : seg) % ns : 0u);
    const bool set_ok = set < ns;
    const uint32_t iid = a.one_inst ? a.one_id : seg;
    const uint64_t pbase = (uint64_t)set * nv;
    /* weights below 2^31 (agnes_set_info.fast): gather the u32 table, half the lines */
    const bool w32 = set_ok && a.sets[set].fast;
    __syncthreads();

    for (uint64_t base = beg; base < end; base += (uint64_t)VPT * T) {
        uint32_t key[VPT], val[VPT], okm = 0u, nnm = 0u;
        uint64_t w[VPT];
#pragma unroll
        for (uint32_t s = 0; s < VPT; ++s) {
            const uint64_t j = base + (uint64_t)s * T + tid;
            const bool in = j < end;
            uint32_t inst = 0u, r = 0xFFu, t = 0xFFu, x = 0xFFFFFFFFu;
            val[s] = AGNES_NIL;
            if (in) {
                inst = vb.instance[j];
                r = vb.round[j];
                t = vb.type[j];
                val[s] = vb.value[j];
                x = vb.validator[j];
            }
            const bool ok = in && set_ok && inst == iid && r < a.max_rounds && t <= 1u && x < nv;
            w[s] = !ok ? 0ull : (w32 ? (uint64_t)a.power32[pbase + x] : (uint64_t)a.power[pbase + x]);
            if (a.wout && in) a.wout[j] = (int64_t)w[s];
            key[s] = r * 2u + t;
            okm |= (uint32_t)ok << s;
            nnm |= (uint32_t)(ok && val[s] != AGNES_NIL) << s;
        }
        /* one pass per key present in the wave's 256 votes */
        uint32_t pend = okm;
        for (;;) {
            const uint64_t lm = __builtin_amdgcn_ballot_w64(pend != 0u);
            if (!lm) break;
            const uint32_t kl = (uint32_t)__builtin_ctzll(lm);
            const uint32_t ks = (uint32_t)__builtin_ctz(__builtin_amdgcn_readlane(pend, kl));
            const uint32_t kv = ks == 0u ? key[0] : (ks == 1u ? key[1] : (ks == 2u ? key[2] : key[3]));
            const uint32_t Kc = __builtin_amdgcn_readlane(kv, kl);
            uint64_t sv = 0ull, sn = 0ull;
            uint32_t mm = 0u;
#pragma unroll
            for (uint32_t s = 0; s < VPT; ++s) {
                const bool m = ((pend >> s) & 1u) && key[s] == Kc;
                mm |= (uint32_t)m << s;
                const bool nn = (nnm >> s) & 1u;
                sv += (m && nn) ? w[s] : 0ull;
                sn += (m && !nn) ? w[s] : 0ull;
            }
            pend &= ~mm;
            sv = rdl(scan(sv), 63u);
            sn = rdl(scan(sn), 63u);
            /* the label: the latest non-nil vote of the key (positions order by (s, thread)) */
            unsigned long long lab = 0ull;
#pragma unroll
            for (int s = (int)VPT - 1; s >= 0; --s) {
                const uint64_t bl = __builtin_amdgcn_ballot_w64(((mm & nnm) >> s) & 1u);
                if (bl && !lab) {
                    const uint32_t hl = 63u - (uint32_t)__builtin_clzll(bl);
                    const uint64_t pos = base + (uint64_t)s * T + (tid - lane) + hl - beg;
                    lab = ((pos + 1ull) << 32) | __builtin_amdgcn_readlane(val[s], hl);
                }
            }
            if (lane == 0u) {
                if (sv) atomicAdd(vw + Kc, (unsigned long long)sv);
                if (sn) atomicAdd(nw + Kc, (unsigned long long)sn);
                if (lab) atomicMax(lb + Kc, lab);
            }
        }
    }
    __syncthreads();
    for (uint32_t k = tid; k < K; k += T) {
        agnes_carry_rec c;
        c.value_w = (int64_t)vw[k];
        c.nil_w = (int64_t)nw[k];
        c.value = lb[k] ? (uint32_t)lb[k] : AGNES_NIL;
        c.pad = 0u;
        a.counts[(uint64_t)seg * K + k] = c;
    }
}

} // namespace partials
} // namespace agnes

hipError_t agnes_launch_partials(const agnes_vote_batch* vb, const int64_t* power, const uint32_t* power32,
                                 const agnes_set_info* sets, uint32_t n_sets, uint32_t n_vals,
                                 uint32_t max_rounds, uint32_t one_inst, uint32_t one_id, agnes_carry_rec* counts,
                                 int64_t* weights, hipStream_t st) {
    using namespace agnes::partials;
    const uint32_t n = vb->n_instances;
    if (n == 0) return hipSuccess;
    PArgs a{*vb, power, power32, sets, n_sets, n_vals, 2u * max_rounds, max_rounds, one_inst, one_id, counts, weights};
    AgnesKt kt("partials", st);
    hipLaunchKernelGGL(partials_kernel, dim3(n), dim3(T), (size_t)3u * a.keys * sizeof(uint64_t), st, a);
    return hipGetLastError();
}
