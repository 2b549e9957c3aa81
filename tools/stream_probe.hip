// Standalone bandwidth probe for the vote-stream access shape (14 B SoA in, 1 B out):
// how much HBM bandwidth do per-lane loads vs. dwordx4 register staging reach at a
// given number of votes in flight per wave?  Development tool, not part of the engine.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/sp tools/stream_probe.hip && /tmp/sp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

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

// (A) one vote per lane, UNROLL chunks of 64 in flight per wave, contiguous range per wave
template <int UNROLL>
__global__ __launch_bounds__(256) void per_lane(Cols c) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t per = (c.n + W - 1) / W;
    const uint64_t b = w * per, e = b + per < c.n ? b + per : c.n;
    for (uint64_t j0 = b; j0 < e; j0 += 64 * UNROLL) {
        uint32_t a[UNROLL], v[UNROLL], x[UNROLL], r[UNROLL], t[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t j = j0 + u * 64 + lane;
            if (j < e) { a[u] = c.inst[j]; v[u] = c.value[j]; x[u] = c.val[j]; r[u] = c.round[j]; t[u] = c.type[j]; }
            else { a[u] = v[u] = x[u] = r[u] = t[u] = 0; }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t j = j0 + u * 64 + lane;
            if (j < e) c.out[j] = (uint8_t)(a[u] ^ v[u] ^ x[u] ^ r[u] ^ t[u]);
        }
    }
}

// (B) dwordx4 staging: each lane loads 4 consecutive votes of each column (256 votes / wave-load)
template <int UNROLL>
__global__ __launch_bounds__(256) void staged(Cols c) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = (uint64_t)gridDim.x * 4;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    uint64_t per = (c.n + W - 1) / W;
    per = (per + 255) & ~255ull;
    const uint64_t b = w * per, e = b + per < c.n ? b + per : c.n;
    for (uint64_t j0 = b; j0 < e; j0 += 256 * UNROLL) {
        uint4 a[UNROLL], v[UNROLL], x[UNROLL];
        uint32_t r[UNROLL], t[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t j = j0 + u * 256 + lane * 4;
            if (j + 3 < e) {
                a[u] = *(const uint4*)(c.inst + j); v[u] = *(const uint4*)(c.value + j); x[u] = *(const uint4*)(c.val + j);
                r[u] = *(const uint32_t*)(c.round + j); t[u] = *(const uint32_t*)(c.type + j);
            } else { a[u] = v[u] = x[u] = make_uint4(0, 0, 0, 0); r[u] = t[u] = 0; }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint64_t j = j0 + u * 256 + lane * 4;
            if (j + 3 < e) {
                uint32_t o = 0;
                o |= (uint8_t)(a[u].x ^ v[u].x ^ x[u].x ^ r[u]);
                o |= (uint32_t)(uint8_t)(a[u].y ^ v[u].y ^ x[u].y ^ (r[u] >> 8)) << 8;
                o |= (uint32_t)(uint8_t)(a[u].z ^ v[u].z ^ x[u].z ^ (t[u])) << 16;
                o |= (uint32_t)(uint8_t)(a[u].w ^ v[u].w ^ x[u].w ^ (t[u] >> 8)) << 24;
                *(uint32_t*)(c.out + j) = o;
            }
        }
    }
}

template <typename K>
static float timeit(K k, int blocks, Cols c, int reps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, c);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, c);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
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
    for (int bpc : {2, 4, 8}) {
        const int blocks = 256 * bpc;
        printf("blocks/CU %d (waves/CU %d)\n", bpc, bpc * 4);
        printf("  per_lane x1  %.1f GB/s\n", bytes / timeit(per_lane<1>, blocks, c, 5) / 1e6);
        printf("  per_lane x2  %.1f GB/s\n", bytes / timeit(per_lane<2>, blocks, c, 5) / 1e6);
        printf("  per_lane x4  %.1f GB/s\n", bytes / timeit(per_lane<4>, blocks, c, 5) / 1e6);
        printf("  per_lane x8  %.1f GB/s\n", bytes / timeit(per_lane<8>, blocks, c, 5) / 1e6);
        printf("  staged   x1  %.1f GB/s\n", bytes / timeit(staged<1>, blocks, c, 5) / 1e6);
        printf("  staged   x2  %.1f GB/s\n", bytes / timeit(staged<2>, blocks, c, 5) / 1e6);
        printf("  staged   x4  %.1f GB/s\n", bytes / timeit(staged<4>, blocks, c, 5) / 1e6);
    }
    return 0;
}
