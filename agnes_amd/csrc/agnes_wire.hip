/*
 * agnes_wire.hip — wire-format ingest: 104-byte signed vote records -> the tally's
 * SoA columns, every signature checked (include/agnes.h
 * agnes_wire_ingest).  The vote fields are those of Vote (lib.rs:22-39) plus the
 * instance, height and validator a network message names; the key is the
 * validator's (validators.rs:4-8, 15-17).
 *
 * One record per lane: an Ed25519 verification is ~4k field products of integer
 * multiply-adds with no data shared between votes (the fixed-base table, 123 KB,
 * is read from L2), so the kernel is VALU bound and simply needs every lane busy
 * (agnes_ed25519.h).  The record and
 * the key are read once (136 B per vote), the columns written once (14 B + the
 * verdict byte).
 */
#include <hip/hip_runtime.h>

#include "agnes_ed25519.h"
#include "agnes_internal.h"

namespace agnes {
namespace wire {

__global__ __launch_bounds__(256) void ingest_kernel(agnes_wire_args a) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    /* the record: 13 x 8 B */
    uint8_t rec[104];
    {
        const uint64_t* src = reinterpret_cast<const uint64_t*>(a.records + i);
#pragma unroll
        for (int k = 0; k < 13; ++k) {
            const uint64_t w = src[k];
#pragma unroll
            for (int b = 0; b < 8; ++b) rec[8 * k + b] = (uint8_t)(w >> (8 * b));
        }
    }
    auto u32at = [&](int o) -> uint32_t {
        return (uint32_t)rec[o] | ((uint32_t)rec[o + 1] << 8) | ((uint32_t)rec[o + 2] << 16) | ((uint32_t)rec[o + 3] << 24);
    };
    auto i64at = [&](int o) -> int64_t { return (int64_t)(((uint64_t)u32at(o + 4) << 32) | u32at(o)); };
    const uint32_t magic = u32at(0), inst = u32at(4), val = u32at(24), value = u32at(28);
    const int64_t height = i64at(8), rnd = i64at(16);
    const uint32_t typ = rec[32];
    uint32_t pad = 0;
#pragma unroll
    for (int k = 33; k < 40; ++k) pad |= rec[k];

    uint32_t verdict = AGNES_WIRE_OK;
    if (magic != AGNES_WIRE_MAGIC || typ > 1u || pad != 0u || rnd < 0 || rnd >= (int64_t)a.max_rounds) {
        verdict = AGNES_WIRE_BAD_FORMAT;
    } else if (height != a.height) {
        verdict = AGNES_WIRE_BAD_HEIGHT;
    } else {
        uint32_t set = 0;
        bool ok = true;
        if (a.instance_set) {
            ok = inst < a.n_instances;
            set = ok ? a.instance_set[inst] : 0u;
        } else {
            set = a.n_sets ? inst % a.n_sets : 0u;
        }
        if (!ok || set >= a.n_sets || val >= a.n_vals) {
            verdict = AGNES_WIRE_BAD_VALIDATOR;
        } else {
            uint8_t pub[32];
            const uint4* kp = reinterpret_cast<const uint4*>(a.pubkeys + ((uint64_t)set * a.n_vals + val) * 32u);
            const uint4 k0 = kp[0], k1 = kp[1];
            const uint32_t kw[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
#pragma unroll
            for (int b = 0; b < 32; ++b) pub[b] = (uint8_t)(kw[b >> 2] >> (8 * (b & 3)));
            if (!ed::verify(pub, rec, AGNES_WIRE_SIGNED_BYTES, rec + AGNES_WIRE_SIGNED_BYTES, a.base_table))
                verdict = AGNES_WIRE_BAD_SIGNATURE;
        }
    }
    const bool acc = verdict == AGNES_WIRE_OK;
    a.instance[i] = inst;
    a.value[i] = value;
    a.validator[i] = val;
    a.round[i] = acc ? (uint8_t)rnd : (uint8_t)0;
    a.type[i] = acc ? (uint8_t)typ : (uint8_t)0xFF;
    a.verdict[i] = (uint8_t)verdict;
}

/* the fixed-base table: row i = j 16^i B, j = 0..15, one thread a row */
__global__ __launch_bounds__(64) void table_kernel(int32_t* tab) {
    const int i = (int)threadIdx.x;
    if (i < 64) ed::build_base_row(i, tab + i * ed::BASE_ROW_WORDS);
}

} // namespace wire
} // namespace agnes

size_t agnes_wire_table_bytes(void) { return 64u * agnes::ed::BASE_ROW_WORDS * sizeof(int32_t); }

hipError_t agnes_launch_wire_table(int32_t* table, hipStream_t st) {
    hipLaunchKernelGGL(agnes::wire::table_kernel, dim3(1), dim3(64), 0, st, table);
    return hipGetLastError();
}

hipError_t agnes_launch_wire_ingest(const agnes_wire_args* a, hipStream_t st) {
    if (a->n == 0) return hipSuccess;
    const uint64_t blocks = (a->n + 255u) / 256u;
    hipLaunchKernelGGL(agnes::wire::ingest_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, *a);
    return hipGetLastError();
}
