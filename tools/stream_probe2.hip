// Bandwidth ceiling probe for the vote-stream access shape (development tool, not
// part of the engine): which load shape moves the 14 B/vote SoA in + 1 B/vote out
// fastest on MI355X?  Every variant walks a contiguous vote range per wave.
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_probe2 tools/stream_probe2.hip
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

__device__ __forceinline__ void wave_range(uint64_t n, uint64_t align, uint64_t& b, uint64_t& e) {
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    uint64_t per = (n + W - 1) / W;
    per = (per + align - 1) / align * align;
    b = w * per;
    e = b + per < n ? b + per : n;
    if (b > n) b = n;
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t ld(const uint32_t* p, bool nt) { return nt ? __builtin_nontemporal_load(p) : *p; }
__device__ __forceinline__ uint4 ld(const uint4* p, bool nt) {
    if (!nt) return *p;
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st(uint4 o, uint4* p, bool nt) {
    if (!nt) { *p = o; return; }
    v4u v = {o.x, o.y, o.z, o.w};
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
}

// (B) 4 votes per lane per column (dwordx4 / dword), U chunks of 256 in flight
template <int U, bool NT>
__global__ __launch_bounds__(256) void staged(Cols c) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t b, e;
    wave_range(c.n, 256, b, e);
    for (uint64_t j0 = b; j0 + 256 * U <= e; j0 += 256 * U) {
        uint4 a[U], v[U], x[U];
        uint32_t r[U], t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = j0 + u * 256 + lane * 4;
            a[u] = ld((const uint4*)(c.inst + j), NT);
            v[u] = ld((const uint4*)(c.value + j), NT);
            x[u] = ld((const uint4*)(c.val + j), NT);
            r[u] = ld((const uint32_t*)(c.round + j), NT);
            t[u] = ld((const uint32_t*)(c.type + j), NT);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = j0 + u * 256 + lane * 4;
            const uint32_t o = (a[u].x ^ v[u].y ^ x[u].z ^ a[u].w) + r[u] + t[u];
            if (NT) __builtin_nontemporal_store(o, (uint32_t*)(c.out + j));
            else *(uint32_t*)(c.out + j) = o;
        }
    }
}

// (D) 16 votes per lane: u32 columns 4 x dwordx4, u8 columns 1 x dwordx4, out 1 x dwordx4
template <bool NT>
__global__ __launch_bounds__(256) void wide16(Cols c) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t b, e;
    wave_range(c.n, 1024, b, e);
    for (uint64_t j0 = b; j0 + 1024 <= e; j0 += 1024) {
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k) { /* u32 columns: 4 consecutive 256-vote slabs, lane-contiguous */
            const uint64_t j = j0 + k * 256 + lane * 4;
            const uint4 a = ld((const uint4*)(c.inst + j), NT);
            const uint4 v = ld((const uint4*)(c.value + j), NT);
            const uint4 x = ld((const uint4*)(c.val + j), NT);
            acc.x += a.x ^ v.x ^ x.x; acc.y += a.y ^ v.y ^ x.y; acc.z += a.z ^ v.z; acc.w += x.w;
        }
        const uint64_t jb = j0 + lane * 16;
        const uint4 r = ld((const uint4*)(c.round + jb), NT);
        const uint4 t = ld((const uint4*)(c.type + jb), NT);
        uint4 o = make_uint4(acc.x + r.x + t.x, acc.y + r.y + t.y, acc.z + r.z + t.z, acc.w + r.w + t.w);
        st(o, (uint4*)(c.out + jb), NT);
    }
}

// (E) read only: staged loads, no output stream (one store per wave at the end)
template <int U>
__global__ __launch_bounds__(256) void readonly(Cols c) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t b, e;
    wave_range(c.n, 256, b, e);
    uint32_t s = 0;
    for (uint64_t j0 = b; j0 + 256 * U <= e; j0 += 256 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = j0 + u * 256 + lane * 4;
            const uint4 a = *(const uint4*)(c.inst + j), v = *(const uint4*)(c.value + j), x = *(const uint4*)(c.val + j);
            s += a.x ^ v.y ^ x.z ^ *(const uint32_t*)(c.round + j) ^ *(const uint32_t*)(c.type + j);
        }
    }
    if (s == 0x12345678u) c.out[lane] = 1;
}

// (A) float4 copy: inst -> out region reinterpretation (bytes = 2 x 16 B per element)
__global__ __launch_bounds__(256) void copy4(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

template <typename K, typename... A>
static float timeit(K k, int blocks, int reps, A... args) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, args...);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, args...);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

int main() {
    const uint64_t n = 200000000ull;
    Cols c;
    CK(hipMalloc((void**)&c.inst, n * 4)); CK(hipMalloc((void**)&c.value, n * 4)); CK(hipMalloc((void**)&c.val, n * 4));
    CK(hipMalloc((void**)&c.round, n)); CK(hipMalloc((void**)&c.type, n)); CK(hipMalloc((void**)&c.out, n * 4));
    CK(hipMemset((void*)c.inst, 1, n * 4)); CK(hipMemset((void*)c.value, 2, n * 4)); CK(hipMemset((void*)c.val, 3, n * 4));
    CK(hipMemset((void*)c.round, 4, n)); CK(hipMemset((void*)c.type, 5, n));
    c.n = n;
    const double bytes = 15.0 * n;
    const uint64_t n4 = n / 4; /* copy 800 MB -> 800 MB */
    for (int bpc : {4, 8}) {
        const int blocks = 256 * bpc;
        printf("blocks/CU %d\n", bpc);
        printf("  copy float4 (r+w)      %.1f GB/s\n", 32.0 * n4 / timeit(copy4, blocks, 5, (const uint4*)c.inst, (uint4*)c.out, n4) / 1e6);
        printf("  staged x1              %.1f GB/s\n", bytes / timeit(staged<1, false>, blocks, 5, c) / 1e6);
        printf("  staged x2              %.1f GB/s\n", bytes / timeit(staged<2, false>, blocks, 5, c) / 1e6);
        printf("  staged x1 nt           %.1f GB/s\n", bytes / timeit(staged<1, true>, blocks, 5, c) / 1e6);
        printf("  staged x2 nt           %.1f GB/s\n", bytes / timeit(staged<2, true>, blocks, 5, c) / 1e6);
        printf("  wide16                 %.1f GB/s\n", bytes / timeit(wide16<false>, blocks, 5, c) / 1e6);
        printf("  wide16 nt              %.1f GB/s\n", bytes / timeit(wide16<true>, blocks, 5, c) / 1e6);
        printf("  readonly x1 (14 B)     %.1f GB/s\n", 14.0 * n / timeit(readonly<1>, blocks, 5, c) / 1e6);
        printf("  readonly x2 (14 B)     %.1f GB/s\n", 14.0 * n / timeit(readonly<2>, blocks, 5, c) / 1e6);
    }
    return 0;
}
