/*
 * agnes_device.h — wave64 primitives shared by the tally kernels
 * (agnes_kernels.hip: general i64 kernel; agnes_fast.hip: u32 fast kernel).
 */
#ifndef AGNES_DEVICE_H
#define AGNES_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace agnes {

/* the kernels' dynamic LDS (block caches, then the per-wave executor areas) */
extern __shared__ __attribute__((aligned(16))) unsigned char agnes_smem[];

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t rdl(uint32_t x, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
}
__device__ __forceinline__ uint64_t rdl(uint64_t x, uint32_t l) {
    uint32_t lo = rdl((uint32_t)x, l), hi = rdl((uint32_t)(x >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
/* x with lane l replaced by the uniform v (v_writelane) */
template <uint32_t L>
__device__ __forceinline__ uint32_t wrl(uint32_t x, uint32_t v) {
    static_assert(L < 64, "lane");
    asm("v_writelane_b32 %0, %1, %2" : "+v"(x) : "s"(v), "n"(L));
    return x;
}
__device__ __forceinline__ uint32_t rfl(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
    return ((uint64_t)rfl((uint32_t)(x >> 32)) << 32) | rfl((uint32_t)x);
}
__device__ __forceinline__ uint64_t lanemask_le(uint32_t l) { return (2ull << l) - 1ull; }
__device__ __forceinline__ uint64_t lanemask_lt(uint32_t l) { return (1ull << l) - 1ull; }
/* x of lane `src` (ds_bpermute) */
__device__ __forceinline__ uint32_t shfl(uint32_t x, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)x);
}
__device__ __forceinline__ uint64_t shfl(uint64_t x, uint32_t src) {
    return ((uint64_t)shfl((uint32_t)(x >> 32), src) << 32) | shfl((uint32_t)x, src);
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xf, false);
}

/* wave64 inclusive scan: row_shr 1,2,4,8 inside 16-lane rows, then row_bcast15
 * (rows 1,3) and row_bcast31 (rows 2,3).  All 64 lanes must be active. */
__device__ __forceinline__ uint32_t scan(uint32_t x) {
    x += dpp<0x111, 0xf>(x);
    x += dpp<0x112, 0xf>(x);
    x += dpp<0x114, 0xf>(x);
    x += dpp<0x118, 0xf>(x);
    x += dpp<0x142, 0xa>(x);
    x += dpp<0x143, 0xc>(x);
    return x;
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp_step64(uint64_t x) {
    uint32_t lo = dpp<CTRL, ROW_MASK>((uint32_t)x);
    uint32_t hi = dpp<CTRL, ROW_MASK>((uint32_t)(x >> 32));
    return x + (((uint64_t)hi << 32) | lo);
}

/* u64 steps as two DPP-sourced adds (carry through VCC): the lane's own value plus
 * the source lane's, bound_ctrl zero for a source outside the row, rows outside
 * row_mask unchanged — 2 VALU per step instead of the compiler's moves + adds.
 * s_nop 1: the DPP read of a VGPR the previous VALU wrote needs 2 wait states. */
#define AGNES_DPP_ADD64(CTRL, RMASK)                                                                   \
    asm volatile("s_nop 1\n\t"                                                                         \
                 "v_add_co_u32_dpp %0, vcc, %0, %0 " CTRL " row_mask:" RMASK " bank_mask:0xf bound_ctrl:1\n\t" \
                 "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc " CTRL " row_mask:" RMASK " bank_mask:0xf bound_ctrl:1"   \
                 : "+v"(lo), "+v"(hi)                                                                  \
                 :                                                                                     \
                 : "vcc")
__device__ __forceinline__ uint64_t scan(uint64_t x) {
#ifdef AGNES_SCAN64_PLAIN
    x = dpp_step64<0x111, 0xf>(x);
    x = dpp_step64<0x112, 0xf>(x);
    x = dpp_step64<0x114, 0xf>(x);
    x = dpp_step64<0x118, 0xf>(x);
    x = dpp_step64<0x142, 0xa>(x);
    x = dpp_step64<0x143, 0xc>(x);
    return x;
#else
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    AGNES_DPP_ADD64("row_shr:1", "0xf");
    AGNES_DPP_ADD64("row_shr:2", "0xf");
    AGNES_DPP_ADD64("row_shr:4", "0xf");
    AGNES_DPP_ADD64("row_shr:8", "0xf");
    AGNES_DPP_ADD64("row_bcast:15", "0xa");
    AGNES_DPP_ADD64("row_bcast:31", "0xc");
    /* the compiler's hazard tracking does not look inside the asm: the wait states a
     * following DPP read of lo / hi would need */
    asm volatile("s_nop 1" ::: "memory");
    return ((uint64_t)hi << 32) | lo;
#endif
}

__host__ __device__ inline uint64_t align16(uint64_t x) { return (x + 15u) & ~15ull; }

__device__ inline void fill_u32(uint32_t* p, uint64_t n, uint32_t v, uint32_t lane) {
    const uint64_t n4 = n >> 2;
    uint4* q = reinterpret_cast<uint4*>(p);
    const uint4 vv = make_uint4(v, v, v, v);
    for (uint64_t k = lane; k < n4; k += 64) q[k] = vv;
    for (uint64_t k = (n4 << 2) + lane; k < n; k += 64) p[k] = v;
}

} // namespace agnes

#endif
