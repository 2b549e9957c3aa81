// Bandwidth probe: 64 independent per-lane sequential vote streams per wave (each
// lane walks its own contiguous range), 14 B SoA in + 1 B out per vote.
// Development tool, not part of the engine.
//   hipcc --offload-arch=gfx950 -O3 -o tools/lane_probe tools/lane_probe.hip
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

// each lane: contiguous range of n/(threads) votes, D votes loaded ahead per step
template <int D>
__global__ __launch_bounds__(256) void lane_seq(Cols c) {
    const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t per = (c.n + T - 1) / T;
    const uint64_t b = tid * per, e = b + per < c.n ? b + per : c.n;
    uint32_t acc = 0;
    for (uint64_t j = b; j < e; j += D) {
        uint32_t a[D], v[D], x[D], r[D], t[D];
#pragma unroll
        for (int u = 0; u < D; ++u) {
            const uint64_t q = j + u;
            const bool in = q < e;
            a[u] = in ? c.inst[q] : 0; v[u] = in ? c.value[q] : 0; x[u] = in ? c.val[q] : 0;
            r[u] = in ? c.round[q] : 0; t[u] = in ? c.type[q] : 0;
        }
#pragma unroll
        for (int u = 0; u < D; ++u) {
            const uint64_t q = j + u;
            acc = acc * 3u + (a[u] ^ v[u] ^ x[u] ^ r[u] ^ t[u]);  // sequential dependency, like a tally
            if (q < e) c.out[q] = (uint8_t)acc;
        }
    }
}

template <typename K>
static float timeit(K k, int blocks, Cols c, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, c);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, c);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
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
        printf("  lane_seq D1  %.1f GB/s\n", bytes / timeit(lane_seq<1>, blocks, c, 3) / 1e6);
        printf("  lane_seq D4  %.1f GB/s\n", bytes / timeit(lane_seq<4>, blocks, c, 3) / 1e6);
        printf("  lane_seq D8  %.1f GB/s\n", bytes / timeit(lane_seq<8>, blocks, c, 3) / 1e6);
        printf("  lane_seq D16 %.1f GB/s\n", bytes / timeit(lane_seq<16>, blocks, c, 3) / 1e6);
    }
    return 0;
}
