/*
 * agnes_valset.hip — device-side validator-set build (SURVEY.md §8(f) 3;
 * include/agnes.h agnes_valset_build / agnes_valset_find).
 *
 * ValidatorSet (validators.rs:23-56, the intended behaviour: the file does not
 * compile) keeps its validators sorted by address (ValidatorSet::sort, :49-55:
 * sort_unstable_by address, then Vec::dedup), Validator::address is the public
 * key (:15-17), and VoteExecutor::new takes the set's total weight
 * (vote_executor.rs:13).  Here many sets are built at once from one flat list
 * (validator i: address addr[i], power power[i], set set_of[i]):
 *   1. sort indices by (set, address bytes, power, index) -- a bitonic network
 *      over the next power of two: the global stages one launch each, the stages
 *      inside a 2048-index tile in LDS.  (sort_unstable_by leaves equal
 *      addresses in any order; ordering them by power is one of those orders, and
 *      the index tiebreak makes the result deterministic.)
 *   2. Vec::dedup: drop an entry equal in (set, address, power) to the one before
 *      it (a derived PartialEq compares both fields); the first index is kept;
 *   3. compact (exclusive scan of the kept flags, agnes_edges.hip), per-set
 *      offsets by binary search, per-set wrapping totals (one block per set).
 * agnes_valset_find is the lookup ValidatorSet::update / remove start with: the
 * first validator of a set with a given address (binary search).
 * Not on the tally path (a set changes between heights, not per vote).
 */
#include <hip/hip_runtime.h>

#include <cstdint>

#include "agnes_internal.h"

namespace agnes {
namespace valset {

constexpr uint32_t T = 256u;
constexpr uint32_t TILE = 2048u; /* indices sorted in LDS by one block */
constexpr uint32_t PAD = 0xFFFFFFFFu;

struct Keys {
    const uint8_t* addr;
    const int64_t* power;
    const uint32_t* set_of;
    uint32_t addr_len;
    uint32_t n;
};

__device__ __forceinline__ uint32_t set_at(const Keys& k, uint32_t i) { return k.set_of ? k.set_of[i] : 0u; }

/* -1 / 0 / 1: the order of validators i and j by (set, address, power) */
__device__ int cmp3(const Keys& k, uint32_t i, uint32_t j) {
    const uint32_t si = set_at(k, i), sj = set_at(k, j);
    if (si != sj) return si < sj ? -1 : 1;
    const uint8_t* a = k.addr + (uint64_t)i * k.addr_len;
    const uint8_t* b = k.addr + (uint64_t)j * k.addr_len;
    for (uint32_t t = 0; t < k.addr_len; ++t)
        if (a[t] != b[t]) return a[t] < b[t] ? -1 : 1;
    const int64_t pi = k.power[i], pj = k.power[j];
    if (pi != pj) return pi < pj ? -1 : 1;
    return 0;
}

/* strict total order on indices, padding last */
__device__ __forceinline__ bool less(const Keys& k, uint32_t i, uint32_t j) {
    if (i == PAD || j == PAD) return i != PAD && j == PAD;
    const int c = cmp3(k, i, j);
    return c != 0 ? c < 0 : i < j;
}

__global__ __launch_bounds__(T) void init_kernel(uint32_t* idx, uint32_t N, uint32_t n) {
    for (uint32_t t = blockIdx.x * T + threadIdx.x; t < N; t += gridDim.x * T) idx[t] = t < n ? t : PAD;
}

/* one bitonic stage (block size kk, distance j) over the whole array */
__global__ __launch_bounds__(T) void step_kernel(Keys k, uint32_t* idx, uint32_t N, uint32_t kk, uint32_t j) {
    for (uint32_t t = blockIdx.x * T + threadIdx.x; t < N; t += gridDim.x * T) {
        const uint32_t p = t ^ j;
        if (p <= t) continue;
        const uint32_t a = idx[t], b = idx[p];
        const bool asc = (t & kk) == 0u;
        if (asc ? less(k, b, a) : less(k, a, b)) {
            idx[t] = b;
            idx[p] = a;
        }
    }
}

/* every stage with distance < TILE for block sizes kk0 .. (kk0 == 0: all sizes
 * up to TILE, the tiles' own sort), inside one tile */
__global__ __launch_bounds__(T) void tile_kernel(Keys k, uint32_t* idx, uint32_t N, uint32_t kk_fixed) {
    __shared__ uint32_t s[TILE];
    const uint32_t base = blockIdx.x * TILE;
    for (uint32_t t = threadIdx.x; t < TILE; t += T) s[t] = base + t < N ? idx[base + t] : PAD;
    __syncthreads();
    auto stage = [&](uint32_t kk, uint32_t j) {
        for (uint32_t t = threadIdx.x; t < TILE; t += T) {
            const uint32_t p = t ^ j;
            if (p > t) {
                const uint32_t a = s[t], b = s[p];
                const bool asc = ((base + t) & kk) == 0u;
                if (asc ? less(k, b, a) : less(k, a, b)) {
                    s[t] = b;
                    s[p] = a;
                }
            }
        }
        __syncthreads();
    };
    if (kk_fixed == 0u) {
        for (uint32_t kk = 2u; kk <= TILE; kk <<= 1)
            for (uint32_t j = kk >> 1; j > 0u; j >>= 1) stage(kk, j);
    } else {
        for (uint32_t j = TILE >> 1; j > 0u; j >>= 1) stage(kk_fixed, j);
    }
    for (uint32_t t = threadIdx.x; t < TILE; t += T)
        if (base + t < N) idx[base + t] = s[t];
}

/* kept flags into pos[1 + t] (Vec::dedup: equal to the entry before -> dropped;
 * a set id outside [0, n_sets) -> dropped) */
__global__ __launch_bounds__(T) void flag_kernel(Keys k, const uint32_t* idx, uint32_t N, uint32_t n_sets, uint64_t* pos) {
    for (uint32_t t = blockIdx.x * T + threadIdx.x; t < N; t += gridDim.x * T) {
        const uint32_t a = idx[t];
        bool keep = a != PAD && set_at(k, a) < n_sets;
        if (keep && t > 0u) {
            const uint32_t b = idx[t - 1u];
            keep = b == PAD || cmp3(k, b, a) != 0;
        }
        pos[1u + t] = keep ? 1u : 0u;
    }
}

__global__ __launch_bounds__(T) void scatter_kernel(Keys k, const uint32_t* idx, uint32_t N, const uint64_t* pos,
                                                    uint32_t* order, int64_t* power_out, uint32_t* set_out,
                                                    uint8_t* addr_out) {
    for (uint32_t t = blockIdx.x * T + threadIdx.x; t < N; t += gridDim.x * T) {
        if (pos[t + 1u] == pos[t]) continue; /* dropped */
        const uint64_t o = pos[t];
        const uint32_t a = idx[t];
        order[o] = a;
        power_out[o] = k.power[a];
        set_out[o] = set_at(k, a);
        if (addr_out)
            for (uint32_t b = 0; b < k.addr_len; ++b)
                addr_out[o * k.addr_len + b] = k.addr[(uint64_t)a * k.addr_len + b];
    }
}

__global__ __launch_bounds__(T) void offsets_kernel(const uint32_t* set_out, const uint64_t* pos, uint32_t N,
                                                    uint32_t n_sets, uint64_t* set_offsets) {
    const uint64_t m = pos[N];
    for (uint32_t s = blockIdx.x * T + threadIdx.x; s <= n_sets; s += gridDim.x * T) {
        uint64_t lo = 0, hi = m; /* first output with set >= s */
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (set_out[mid] < s) lo = mid + 1u;
            else hi = mid;
        }
        set_offsets[s] = s == n_sets ? m : lo;
    }
}

__global__ __launch_bounds__(T) void totals_kernel(const int64_t* power_out, const uint64_t* set_offsets, int64_t* totals) {
    __shared__ uint64_t part[T];
    const uint32_t s = blockIdx.x;
    uint64_t acc = 0; /* wrapping i64, as the reference's release build */
    for (uint64_t o = set_offsets[s] + threadIdx.x; o < set_offsets[s + 1u]; o += T) acc += (uint64_t)power_out[o];
    part[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t d = T / 2u; d > 0u; d >>= 1) {
        if (threadIdx.x < d) part[threadIdx.x] += part[threadIdx.x + d];
        __syncthreads();
    }
    if (threadIdx.x == 0) totals[s] = (int64_t)part[0];
}

__global__ __launch_bounds__(T) void find_kernel(const uint8_t* sorted_addr, uint32_t addr_len, const uint64_t* set_offsets,
                                                 uint32_t n_sets, const uint8_t* q_addr, const uint32_t* q_set,
                                                 uint64_t n_q, uint64_t* out) {
    for (uint64_t q = (uint64_t)blockIdx.x * T + threadIdx.x; q < n_q; q += (uint64_t)gridDim.x * T) {
        const uint32_t s = q_set ? q_set[q] : 0u;
        if (s >= n_sets) {
            out[q] = ~0ull;
            continue;
        }
        const uint8_t* key = q_addr + q * addr_len;
        auto cmp = [&](uint64_t o) -> int { /* sorted address o vs the query */
            const uint8_t* a = sorted_addr + o * addr_len;
            for (uint32_t t = 0; t < addr_len; ++t)
                if (a[t] != key[t]) return a[t] < key[t] ? -1 : 1;
            return 0;
        };
        uint64_t lo = set_offsets[s], hi = set_offsets[s + 1u];
        const uint64_t end = hi;
        while (lo < hi) { /* first address >= the query */
            const uint64_t mid = (lo + hi) >> 1;
            if (cmp(mid) < 0) lo = mid + 1u;
            else hi = mid;
        }
        out[q] = (lo < end && cmp(lo) == 0) ? lo : ~0ull;
    }
}

} // namespace valset
} // namespace agnes

static dim3 vs_grid(uint64_t n) {
    const uint64_t b = (n + agnes::valset::T - 1u) / agnes::valset::T;
    return dim3((uint32_t)(b == 0 ? 1u : (b < 4096u ? b : 4096u)));
}

hipError_t agnes_launch_valset_build(const uint8_t* addr, uint32_t addr_len, const int64_t* power, const uint32_t* set_of,
                                     uint32_t n, uint32_t n_sets, uint32_t* idx, uint32_t N, uint64_t* pos,
                                     uint64_t* scan_scratch, uint32_t* set_out, uint32_t* order, int64_t* power_out,
                                     uint8_t* addr_out, uint64_t* set_offsets, int64_t* totals, hipStream_t st) {
    using namespace agnes::valset;
    const Keys k{addr, power, set_of, addr_len, n};
    AgnesKt kt("valset_build", st);
    hipLaunchKernelGGL(init_kernel, vs_grid(N), dim3(T), 0, st, idx, N, n);
    /* bitonic sort of N = 2^m >= TILE indices: tiles in LDS, then per block size the
     * stages with distance >= TILE globally and the rest in LDS */
    hipLaunchKernelGGL(tile_kernel, dim3(N / TILE), dim3(T), 0, st, k, idx, N, 0u);
    for (uint32_t kk = TILE << 1; kk <= N; kk <<= 1) {
        for (uint32_t j = kk >> 1; j >= TILE; j >>= 1)
            hipLaunchKernelGGL(step_kernel, vs_grid(N), dim3(T), 0, st, k, idx, N, kk, j);
        hipLaunchKernelGGL(tile_kernel, dim3(N / TILE), dim3(T), 0, st, k, idx, N, kk);
    }
    hipError_t e = hipMemsetAsync(pos, 0, sizeof(uint64_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(flag_kernel, vs_grid(N), dim3(T), 0, st, k, idx, N, n_sets, pos);
    e = agnes_launch_offsets_scan(pos, N, scan_scratch, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(scatter_kernel, vs_grid(N), dim3(T), 0, st, k, idx, N, pos, order, power_out, set_out, addr_out);
    hipLaunchKernelGGL(offsets_kernel, vs_grid((uint64_t)n_sets + 1u), dim3(T), 0, st, set_out, pos, N, n_sets,
                       set_offsets);
    hipLaunchKernelGGL(totals_kernel, dim3(n_sets), dim3(T), 0, st, power_out, set_offsets, totals);
    return hipGetLastError();
}

hipError_t agnes_launch_valset_find(const uint8_t* sorted_addr, uint32_t addr_len, const uint64_t* set_offsets,
                                    uint32_t n_sets, const uint8_t* q_addr, const uint32_t* q_set, uint64_t n_q,
                                    uint64_t* out, hipStream_t st) {
    if (n_q == 0) return hipSuccess;
    AgnesKt kt("valset_find", st);
    hipLaunchKernelGGL(agnes::valset::find_kernel, vs_grid(n_q), dim3(agnes::valset::T), 0, st, sorted_addr, addr_len,
                       set_offsets, n_sets, q_addr, q_set, n_q, out);
    return hipGetLastError();
}
