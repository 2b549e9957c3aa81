// Bandwidth probe for the round-2 sweep kernel's memory pipeline (development
// tool, not part of the engine).  Every variant moves the 14 B/vote SoA in and
// 1 B/vote out over contiguous per-wave vote ranges, like the tally kernels:
//   staged<U>   U chunks (256 votes) of loads into VGPRs, then their stores
//   ring<D>     a D-slot LDS-DMA ring per wave: D chunks in flight while one is read
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe3 tools/stream_probe3.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

struct Cols {
    const uint32_t* inst;
    const uint8_t* round;
    const uint8_t* type;
    const uint32_t* value;
    const uint32_t* val;
    uint8_t* out;
    uint64_t n;
};

extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

__device__ __forceinline__ void wave_range(uint64_t n, uint64_t& b, uint64_t& e) {
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    uint64_t per = (n + W - 1) / W;
    per = (per + 255) / 256 * 256;
    b = w * per;
    e = b + per < n ? b + per : n;
    if (b > n) b = n;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void glds16(const void* g, unsigned char* l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds_addr(l)) : "memory");
}
__device__ __forceinline__ void glds4(const void* g, unsigned char* l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds_addr(l)) : "memory");
}
__device__ __forceinline__ void glds16nt(const void* g, unsigned char* l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds_addr(l)) : "memory");
}
__device__ __forceinline__ void glds4nt(const void* g, unsigned char* l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds_addr(l)) : "memory");
}
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void vm_wait_n(uint32_t n) { /* n wave-uniform */
    switch (n) {
    case 0: vm_wait<0>(); break; case 1: vm_wait<1>(); break; case 2: vm_wait<2>(); break;
    case 3: vm_wait<3>(); break; case 4: vm_wait<4>(); break; case 5: vm_wait<5>(); break;
    case 6: vm_wait<6>(); break; case 7: vm_wait<7>(); break; case 8: vm_wait<8>(); break;
    case 9: vm_wait<9>(); break; case 10: vm_wait<10>(); break; case 11: vm_wait<11>(); break;
    case 12: vm_wait<12>(); break; case 13: vm_wait<13>(); break; default: vm_wait<0>(); break;
    }
}

/* a few VALU per vote so the loop is not pure copy: COMPUTE adds that many
 * dependent integer ops per lane per chunk */
template <int COMPUTE>
__device__ __forceinline__ uint32_t work(uint4 a, uint4 v, uint4 x, uint32_t r, uint32_t t) {
    uint32_t o = (a.x ^ v.y ^ x.z ^ a.w) + r + t;
#pragma unroll
    for (int k = 0; k < COMPUTE; ++k) o = o * 0x9E3779B1u + (o >> 7) + v.x;
    return o;
}

template <int U, int COMPUTE>
__global__ __launch_bounds__(256) void staged(Cols c) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t b, e;
    wave_range(c.n, b, e);
    for (uint64_t j0 = b; j0 + 256 * U <= e; j0 += 256 * U) {
        uint4 a[U], v[U], x[U];
        uint32_t r[U], t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = j0 + u * 256 + lane * 4;
            a[u] = *(const uint4*)(c.inst + j);
            v[u] = *(const uint4*)(c.value + j);
            x[u] = *(const uint4*)(c.val + j);
            r[u] = *(const uint32_t*)(c.round + j);
            t[u] = *(const uint32_t*)(c.type + j);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = j0 + u * 256 + lane * 4;
            *(uint32_t*)(c.out + j) = work<COMPUTE>(a[u], v[u], x[u], r[u], t[u]);
        }
    }
}

/* D-slot LDS-DMA ring per wave (3.5 KB per slot); the chunk D ahead is issued
 * right after the current one is read out of LDS */
constexpr uint32_t SLOT = 3584;
template <int D, int COMPUTE, bool NT = false, bool STRIDE = false>
__global__ __launch_bounds__(256) void ring(Cols c) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned char* const base = smem + wave * (D * SLOT);
    uint64_t b, e;
    wave_range(c.n, b, e);
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t wv = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    uint64_t nck = 0; /* STRIDE: chunks of this wave */
    if (STRIDE) {
        const uint64_t tot = c.n / 256;
        nck = tot > wv ? (tot - wv + W - 1) / W : 0;
        b = 0;
        e = nck * 256; /* virtual range: chunk index k -> address (wv + k W) 256 */
    }
    auto addr = [&](uint64_t j0) -> uint64_t { return STRIDE ? (wv + (j0 / 256) * W) * 256 : j0; };
    auto issue = [&](uint64_t j0v, uint32_t s) {
        const uint64_t j0 = addr(j0v);
        unsigned char* p = base + s * SLOT;
        const uint64_t j = j0 + lane * 4;
        if (NT) {
            glds16nt(c.inst + j, p);
            glds16nt(c.value + j, p + 1024);
            glds16nt(c.val + j, p + 2048);
            glds4nt(c.round + j, p + 3072);
            glds4nt(c.type + j, p + 3328);
        } else {
            glds16(c.inst + j, p);
            glds16(c.value + j, p + 1024);
            glds16(c.val + j, p + 2048);
            glds4(c.round + j, p + 3072);
            glds4(c.type + j, p + 3328);
        }
    };
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (b + (uint64_t)d * 256 + 256 <= e) issue(b + (uint64_t)d * 256, d);
    uint32_t s = 0;
    for (uint64_t j0 = b; j0 + 256 <= e; j0 += 256) {
        /* the oldest slot has landed when only the younger chunks' DMAs (5 each)
         * and the stores issued after it remain in flight */
        const uint64_t k = (j0 - b) / 256;
        const uint64_t left = (e - j0) / 256 - 1;
        const uint32_t ca = (uint32_t)(left < (uint64_t)(D - 1) ? left : (uint64_t)(D - 1));
        const uint32_t sa = (uint32_t)(k < (uint64_t)D ? k : (uint64_t)D);
        vm_wait_n(5 * ca + sa);
        unsigned char* p = base + s * SLOT;
        const uint4 a = *(const uint4*)(p + 16 * lane);
        const uint4 v = *(const uint4*)(p + 1024 + 16 * lane);
        const uint4 x = *(const uint4*)(p + 2048 + 16 * lane);
        const uint32_t r = *(const uint32_t*)(p + 3072 + 4 * lane);
        const uint32_t t = *(const uint32_t*)(p + 3328 + 4 * lane);
        __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0) */
        const uint64_t nj = j0 + (uint64_t)D * 256;
        if (nj + 256 <= e) issue(nj, s);
        s = s + 1 == D ? 0 : s + 1;
        *(uint32_t*)(c.out + addr(j0) + lane * 4) = work<COMPUTE>(a, v, x, r, t);
    }
}

/* staged<U> with chunk groups dealt round-robin over the waves (grid-stride):
 * the whole chip sweeps one window of consecutive chunks at a time */
template <int U, bool NT>
__global__ __launch_bounds__(256) void strided(Cols c) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    for (uint64_t j0 = w * 256 * U; j0 + 256 * U <= c.n; j0 += W * 256 * U) {
        uint4 a[U], v[U], x[U];
        uint32_t r[U], t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = j0 + u * 256 + lane * 4;
            if (NT) {
                a[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load((const __attribute__((ext_vector_type(4))) unsigned*)(c.inst + j)));
                v[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load((const __attribute__((ext_vector_type(4))) unsigned*)(c.value + j)));
                x[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load((const __attribute__((ext_vector_type(4))) unsigned*)(c.val + j)));
                r[u] = __builtin_nontemporal_load((const uint32_t*)(c.round + j));
                t[u] = __builtin_nontemporal_load((const uint32_t*)(c.type + j));
            } else {
                a[u] = *(const uint4*)(c.inst + j);
                v[u] = *(const uint4*)(c.value + j);
                x[u] = *(const uint4*)(c.val + j);
                r[u] = *(const uint32_t*)(c.round + j);
                t[u] = *(const uint32_t*)(c.type + j);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = j0 + u * 256 + lane * 4;
            *(uint32_t*)(c.out + j) = work<0>(a[u], v[u], x[u], r[u], t[u]);
        }
    }
}

/* float4 copy, grid-stride (the guide's 6.29 TB/s shape) */
__global__ __launch_bounds__(256) void copy4(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

/* read-only staged (14 B/vote, per-wave contiguous ranges) */
__global__ __launch_bounds__(256) void readonly(Cols c) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t b, e;
    wave_range(c.n, b, e);
    uint32_t s = 0;
    for (uint64_t j0 = b; j0 + 512 <= e; j0 += 512) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const uint64_t j = j0 + u * 256 + lane * 4;
            const uint4 a = *(const uint4*)(c.inst + j), v = *(const uint4*)(c.value + j), x = *(const uint4*)(c.val + j);
            s += a.x ^ v.y ^ x.z ^ *(const uint32_t*)(c.round + j) ^ *(const uint32_t*)(c.type + j);
        }
    }
    if (s == 0x12345678u) c.out[lane] = 1;
}

template <typename K, typename... A>
static float timeit(K k, int blocks, size_t lds, int reps, A... args) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    if (lds > 48 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, args...);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, 0, args...);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (hipGetLastError() != hipSuccess) return -1.f;
    return ms / reps;
}

int main() {
    const uint64_t n = 200000000ull;
    Cols c;
    CK(hipMalloc((void**)&c.inst, n * 4)); CK(hipMalloc((void**)&c.value, n * 4)); CK(hipMalloc((void**)&c.val, n * 4));
    CK(hipMalloc((void**)&c.round, n)); CK(hipMalloc((void**)&c.type, n)); CK(hipMalloc((void**)&c.out, n));
    CK(hipMemset((void*)c.inst, 1, n * 4)); CK(hipMemset((void*)c.value, 2, n * 4)); CK(hipMemset((void*)c.val, 3, n * 4));
    CK(hipMemset((void*)c.round, 4, n)); CK(hipMemset((void*)c.type, 5, n));
    c.n = n;
    const double bytes = 15.0 * n;
    auto rep = [&](const char* name, int bpc, float ms) {
        printf("%-22s blocks/CU %d  %.3f ms  %.0f GB/s\n", name, bpc, ms, bytes / ms / 1e6);
    };
    for (int bpc : {4, 8}) {
        const int blocks = 256 * bpc;
        printf("copy4 (32 B/elem)      blocks/CU %d  %.0f GB/s\n", bpc, 32.0 * (n / 4) / timeit(copy4, blocks, 0, 5, (const uint4*)c.inst, (uint4*)c.value, n / 4) / 1e6);
        printf("readonly (14 B/vote)   blocks/CU %d  %.0f GB/s\n", bpc, 14.0 * n / timeit(readonly, blocks, 0, 5, c) / 1e6);
        rep("strided1", bpc, timeit(strided<1, false>, blocks, 0, 5, c));
        rep("strided2", bpc, timeit(strided<2, false>, blocks, 0, 5, c));
        rep("strided4", bpc, timeit(strided<4, false>, blocks, 0, 5, c));
        rep("strided2 nt", bpc, timeit(strided<2, true>, blocks, 0, 5, c));
    }
    for (int bpc : {4, 6, 8}) {
        const int blocks = 256 * bpc;
        rep("staged1", bpc, timeit(staged<1, 0>, blocks, 0, 5, c));
        rep("staged2", bpc, timeit(staged<2, 0>, blocks, 0, 5, c));
        rep("staged3", bpc, timeit(staged<3, 0>, blocks, 0, 5, c));
        rep("staged2 c40", bpc, timeit(staged<2, 40>, blocks, 0, 5, c));
    }
    for (int bpc : {2, 4, 6}) {
        const int blocks = 256 * bpc;
        rep("ring2 nt", bpc, timeit(ring<2, 0, true, false>, blocks, 8 * SLOT, 5, c));
        rep("ring2 strided", bpc, timeit(ring<2, 0, false, true>, blocks, 8 * SLOT, 5, c));
        rep("ring2 nt strided", bpc, timeit(ring<2, 0, true, true>, blocks, 8 * SLOT, 5, c));
        rep("ring1 nt strided", bpc, timeit(ring<1, 0, true, true>, blocks, 4 * SLOT, 5, c));
        rep("ring2 nt strided c40", bpc, timeit(ring<2, 40, true, true>, blocks, 8 * SLOT, 5, c));
    }
    for (int bpc : {2, 4, 5, 6}) {
        const int blocks = 256 * bpc;
        rep("ring1", bpc, timeit(ring<1, 0>, blocks, 4 * SLOT, 5, c));
        rep("ring2", bpc, timeit(ring<2, 0>, blocks, 8 * SLOT, 5, c));
        if (bpc <= 3) rep("ring3", bpc, timeit(ring<3, 0>, blocks, 12 * SLOT, 5, c));
        rep("ring2 c40", bpc, timeit(ring<2, 40>, blocks, 8 * SLOT, 5, c));
    }
    return 0;
}
