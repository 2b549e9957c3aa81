// Memory-pipeline probe for the flow kernel (development tool, not part of the
// engine): 512-vote chunks of the 14 B/vote SoA staged by LDS-DMA into a D-slot ring
// per wave, 1 B/vote written back, VAL dependent-ish VALU ops per chunk standing in
// for the tally, waves per CU set by the LDS each wave claims.
//   hipcc --offload-arch=gfx950 -O3 -o tools/flow_probe tools/flow_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <initializer_list>

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

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void sdma16(const void* base, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(base), "s"(lds) : "memory");
}
__device__ __forceinline__ void sdma4(const void* base, uint32_t voff, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(base), "s"(lds) : "memory");
}
template <int N> __device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

constexpr uint32_t SLOT = 7168, CH = 512;

template <int D, int VAL>
__global__ __launch_bounds__(256) void flowp(Cols c, uint32_t lpw) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    unsigned char* const base = smem + wave * lpw;
    const uint32_t bl = lds_addr(base);
    const uint64_t W = (uint64_t)gridDim.x * 4;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + wave;
    const uint64_t nck = c.n / CH;
    const uint64_t per = (nck + W - 1) / W;
    const uint64_t k0 = w * per < nck ? w * per : nck, k1 = k0 + per < nck ? k0 + per : nck;
    const uint32_t o16 = 16u * lane, o4 = 4u * lane, o32 = 32u * lane, o8 = 8u * lane;
    auto issue = [&](uint64_t k, uint32_t s) {
        const uint64_t j = k * CH;
        const uint32_t l = bl + s * SLOT;
        __builtin_amdgcn_s_waitcnt(0xC07F);
        sdma16(c.inst + j, o16, l);
        sdma16(c.inst + j + 256, o16, l + 1024);
        sdma16(c.value + j, o16, l + 2048);
        sdma16(c.value + j + 256, o16, l + 3072);
        sdma16(c.val + j, o16, l + 4096);
        sdma16(c.val + j + 256, o16, l + 5120);
        sdma4(c.round + j, o4, l + 6144);
        sdma4(c.round + j + 256, o4, l + 6400);
        sdma4(c.type + j, o4, l + 6656);
        sdma4(c.type + j + 256, o4, l + 6912);
    };
    for (int d = 0; d < D; ++d)
        if (k0 + d < k1) issue(k0 + d, d);
    uint32_t s = 0;
    for (uint64_t k = k0; k < k1; ++k) {
        if (D == 1 || k + 1 >= k1) vm_wait<0>();
        else vm_wait<11>(); /* the younger chunk's 10 DMAs + the last store in flight */
        unsigned char* p = base + s * SLOT;
        const uint4 a0 = *(const uint4*)(p + o32), a1 = *(const uint4*)(p + o32 + 16);
        const uint4 v0 = *(const uint4*)(p + 2048 + o32), v1 = *(const uint4*)(p + 2048 + o32 + 16);
        const uint4 x0 = *(const uint4*)(p + 4096 + o32), x1 = *(const uint4*)(p + 4096 + o32 + 16);
        const uint2 r = *(const uint2*)(p + 6144 + o8), t = *(const uint2*)(p + 6656 + o8);
        uint32_t q[8] = {a0.x ^ v0.x, a0.y ^ v0.y, a0.z ^ x0.z, a0.w ^ x0.w, a1.x ^ v1.x, a1.y ^ x1.y, a1.z ^ r.x, a1.w ^ t.y};
        if (k + D < k1) issue(k + D, s);
        s = s + 1 == D ? 0 : s + 1;
#pragma unroll
        for (int i = 0; i < VAL / 16; ++i)
#pragma unroll
            for (int u = 0; u < 8; ++u) q[u] = (q[u] ^ (0x9E37u + i)) + (q[u] >> 3);
        const uint32_t o0 = q[0] ^ q[1] ^ q[2] ^ q[3], o1 = q[4] ^ q[5] ^ q[6] ^ q[7];
        *(uint2*)(c.out + k * CH + o8) = make_uint2(o0, o1);
    }
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

template <int D, int VAL>
static void run(Cols c, const char* name, std::initializer_list<int> wpcs = {8, 12, 16}) {
    for (int wpc : wpcs) {
        /* LDS per wave so that wpc waves fit a CU (4 waves per block) */
        const uint32_t lpw = (160u * 1024u / wpc) & ~15u;
        if (lpw < D * SLOT) continue;
        const int blocks = 256 * (wpc / 4);
        const float ms = timeit(flowp<D, VAL>, blocks, (size_t)lpw * 4, 5, c, lpw);
        printf("%-10s D=%d VAL=%4d waves/CU %2d  %.3f ms  %.0f GB/s\n", name, D, VAL, wpc, ms, 15.0 * c.n / ms / 1e6);
    }
}

int main() {
    const uint64_t n = 200000000ull;
    Cols c;
    CK(hipMalloc((void**)&c.inst, n * 4)); CK(hipMalloc((void**)&c.value, n * 4)); CK(hipMalloc((void**)&c.val, n * 4));
    CK(hipMalloc((void**)&c.round, n)); CK(hipMalloc((void**)&c.type, n)); CK(hipMalloc((void**)&c.out, n));
    CK(hipMemset((void*)c.inst, 1, n * 4)); CK(hipMemset((void*)c.value, 2, n * 4)); CK(hipMemset((void*)c.val, 3, n * 4));
    CK(hipMemset((void*)c.round, 4, n)); CK(hipMemset((void*)c.type, 5, n));
    c.n = n;
    run<1, 0>(c, "ring1", {16});
    run<1, 320>(c, "ring1", {12, 16});
    /* every chunk 4 votes off the 128-vote (u8 column line) alignment */
    Cols m = c;
    m.inst += 4; m.value += 4; m.val += 4; m.round += 4; m.type += 4; m.out += 4; m.n -= 512;
    run<1, 0>(m, "ring1 mis4", {16});
    run<1, 320>(m, "ring1 mis4", {12, 16});
    m = c;
    m.inst += 32; m.value += 32; m.val += 32; m.round += 32; m.type += 32; m.out += 32; m.n -= 512;
    run<1, 320>(m, "ring1 mis32", {12, 16});
    return 0;
}
