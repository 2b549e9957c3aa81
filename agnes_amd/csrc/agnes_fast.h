/*
 * agnes_fast.h — pieces shared by the u32 fast-path tally kernels
 * (agnes_fast.hip: one instance per chunk; agnes_stream.hip: instance-straddling
 * chunks): chunk geometry, the LDS-DMA prefetch layout, the work-queue constants
 * and the vote-event view of the State.
 */
#ifndef AGNES_FAST_H
#define AGNES_FAST_H

#include "agnes_device.h"
#include "agnes_internal.h"

namespace agnes {
namespace fast {

constexpr uint32_t VPL = 4;
constexpr uint32_t CHUNK = 64u * VPL;
constexpr uint32_t SL = 16u; /* State dword k lives in lane SL + k of a State VGPR */
constexpr uint32_t BQ = 4u;  /* instances per work-queue batch (agnes_fast.hip)   */
constexpr uint32_t QN = AGNES_QUEUE_N;          /* work-queue counters (at most)  */
constexpr uint32_t NONE = 0xFFFFFFFFu;
#ifndef AGNES_FAST_NT
#define AGNES_FAST_NT 0 /* cache policy of the streamed vote/code traffic (2 = nt: slower here, the
                            * over-fetched tail of a chunk is re-read as the next instance's start) */
#endif

/* The u32 domain of the fast kernels, per instance: every power of its set in [0, 2^31),
 * fewer than 2^30 votes and len * maxpow < 2^31, so no running sum reaches 2^31.  An
 * instance outside it goes to the i64 LIST kernel; the u32 tally kernels and the apply
 * pass (agnes_apply.hip), which skips the LIST kernel's instances, test it alike. */
__host__ __device__ __forceinline__ bool defer_to_list(uint32_t fast, uint32_t maxpow, uint64_t len) {
    return !fast || len >= (1ull << 30) || len * (uint64_t)maxpow >= (1ull << 31);
}

/* The u64 domain (agnes_tally_args.w64, sets with agnes_set_info.w64): non-negative
 * powers, fewer than 2^30 votes and len * maxpow < 2^61, so every running sum stays
 * below 2^61 and 3 * sum never wraps (round_votes.rs:31-33).  The instance test of the
 * kernel's domain, u32 or u64: outside it, the i64 LIST kernel's. */
__device__ __forceinline__ bool defer_si(const agnes_set_info& si, uint64_t len, bool w64) {
    if (!w64) return defer_to_list(si.fast, si.maxpow, len);
    return !si.w64 || len >= (1ull << 30) || __umul64hi(len, si.maxw) != 0ull || len * si.maxw >= (1ull << 61);
}

/* LDS-DMA prefetch buffer of one chunk: instance, value, validator (1 KiB each,
 * lane l's 16 B at 16 l), round, type (256 B each, lane l's 4 B at 4 l) */
constexpr uint32_t PF_INST = 0, PF_VALUE = 1024, PF_VAL = 2048, PF_ROUND = 3072, PF_TYPE = 3328,
                   PF_BYTES = 3584;

/* LDS-DMA (global_load_lds) issued by inline asm.  With the builtin the compiler
 * cannot tell the DMA target from the carry / State rows and waits vmcnt(0) before
 * every later LDS read, which drains the prefetch; here the reader of the DMA
 * target waits itself (dma_wait) and nothing else waits for the DMA. */
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void glds16(const void* g, unsigned char* l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(rfl(lds_addr(l)))
                 : "memory");
}
__device__ __forceinline__ void glds4(const void* g, unsigned char* l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(rfl(lds_addr(l)))
                 : "memory");
}
/* non-temporal forms (the streamed vote columns are read once: keep them out of L2) */
__device__ __forceinline__ void glds16nt(const void* g, unsigned char* l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(rfl(lds_addr(l)))
                 : "memory");
}
__device__ __forceinline__ void glds4nt(const void* g, unsigned char* l) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(rfl(lds_addr(l)))
                 : "memory");
}
/* every outstanding vector-memory op (the LDS-DMAs included) has retired */
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ uint32_t byte_of(uint32_t x, uint32_t s) { return (x >> (8u * s)) & 0xFFu; }

/* the uniform view of the State that vote events read (state_machine.rs:196-211) */
struct View {
    uint32_t flags; /* State dword 13: step | locked << 8 | valid << 16 | decided << 24 */
    uint32_t eq8;   /* State.round when in [0, 255], else 0x100 (no u8 vote round equals it) */
    int32_t rlt;    /* clamp(State.round, -1, 256): u8 round r > rlt <=> State.round < r     */
    uint32_t vval;  /* valid.value                                                           */
    uint32_t vsame; /* valid == Some{round: State.round, ..}                                 */
    uint32_t chg;   /* bit idx: the event changes the State (idx = event | eqr << 3)          */
    uint32_t mt;    /* 2-bit message of a non-changing event at idx (1 TimeoutPrevote, 2 TimeoutPrecommit) */
    uint32_t pvchk; /* Precommit with valid at this round: PolkaValue changes iff its value differs */
};

__device__ __forceinline__ int64_t lanes64(uint32_t stv, uint32_t k) {
    return (int64_t)(((uint64_t)rdl(stv, SL + k + 1u) << 32) | rdl(stv, SL + k));
}

__device__ __forceinline__ void view_tables(View& v) {
    const uint32_t step = v.flags & 0xFFu;
    v.chg = (1u << AGNES_CODE_PRECOMMIT_VALUE) | (1u << (AGNES_CODE_PRECOMMIT_VALUE | 8u)); /* :211 */
    v.mt = 2u << (2u * (AGNES_CODE_PRECOMMIT_ANY | 8u));                                       /* :208 */
    v.pvchk = 0;
    if (step == AGNES_STEP_PREVOTE) { /* :196-199 */
        v.chg |= (1u << (AGNES_CODE_POLKA_NIL | 8u)) | (1u << (AGNES_CODE_POLKA_VALUE | 8u));
        v.mt |= 1u << (2u * (AGNES_CODE_POLKA_ANY | 8u));
    } else if (step == AGNES_STEP_PRECOMMIT) { /* :202 set_valid_value */
        if (v.vsame) v.pvchk = 1;
        else v.chg |= 1u << (AGNES_CODE_POLKA_VALUE | 8u);
    }
}

__device__ __forceinline__ void view_round(View& v, int64_t round, uint32_t stv) {
    v.eq8 = (round >= 0 && round <= 255) ? (uint32_t)round : 0x100u;
    v.rlt = round < -1 ? -1 : (round > 256 ? 256 : (int32_t)round);
    v.vsame = ((v.flags >> 16) & 0xFFu) != 0u && lanes64(stv, 6) == round;
}

__device__ __forceinline__ View view_of(uint32_t stv) {
    View v;
    v.flags = rdl(stv, SL + 13u);
    v.vval = rdl(stv, SL + 11u);
    view_round(v, lanes64(stv, 2), stv);
    view_tables(v);
    return v;
}

/* Apply one state-changing vote event (RoundSkip first, then the tally event at
 * the vote's round; state_machine.rs:196-211 via consensus_executor.rs:64-68)
 * to the State lanes; returns the message nibble.  Mirrors sm_vote in
 * agnes_kernels.hip. */
__device__ __forceinline__ uint32_t apply_change(uint32_t& stv, View& v, uint32_t code, uint32_t r,
                                                 uint32_t lab) {
    uint32_t step = v.flags & 0xFFu;
    bool nr = false;
    if ((code & AGNES_CODE_SKIP) && (int32_t)r > v.rlt) { /* :210 round_skip(s, r) */
        stv = wrl<SL + 2u>(stv, r);
        stv = wrl<SL + 3u>(stv, 0u);
        step = AGNES_STEP_NEW_ROUND;
        view_round(v, (int64_t)r, stv);
        nr = true;
    }
    const bool eqr = r == v.eq8;
    uint32_t b = AGNES_VMSG_NONE;
    switch (code & AGNES_CODE_EVENT_MASK) {
    case AGNES_CODE_POLKA_ANY: /* :196 */
        if (eqr && step == AGNES_STEP_PREVOTE) b = AGNES_VMSG_TIMEOUT_PREVOTE;
        break;
    case AGNES_CODE_POLKA_NIL: /* :197 */
        if (eqr && step == AGNES_STEP_PREVOTE) {
            step = AGNES_STEP_PRECOMMIT;
            b = AGNES_VMSG_PRECOMMIT_NIL;
        }
        break;
    case AGNES_CODE_POLKA_VALUE:
        if (eqr && (step == AGNES_STEP_PREVOTE || step == AGNES_STEP_PRECOMMIT)) {
            const uint32_t rl = rdl(stv, SL + 2u), rh = rdl(stv, SL + 3u);
            if (step == AGNES_STEP_PREVOTE) { /* :198 precommit: locked = valid = {round, v} */
                stv = wrl<SL + 4u>(stv, rl);
                stv = wrl<SL + 5u>(stv, rh);
                stv = wrl<SL + 10u>(stv, lab);
                v.flags = (v.flags & ~0xFF00u) | 0x100u;
                step = AGNES_STEP_PRECOMMIT;
                b = AGNES_VMSG_PRECOMMIT_VALUE;
            }
            stv = wrl<SL + 6u>(stv, rl); /* :202 set_valid_value */
            stv = wrl<SL + 7u>(stv, rh);
            stv = wrl<SL + 11u>(stv, lab);
            v.flags = (v.flags & ~0xFF0000u) | 0x10000u;
            v.vval = lab;
            v.vsame = 1;
        }
        break;
    case AGNES_CODE_PRECOMMIT_ANY: /* :208 */
        if (eqr) b = AGNES_VMSG_TIMEOUT_PRECOMMIT;
        break;
    case AGNES_CODE_PRECOMMIT_VALUE: /* :211 commit */
        step = AGNES_STEP_COMMIT;
        v.flags = (v.flags & 0x00FFFFFFu) | 0x01000000u;
        stv = wrl<SL + 8u>(stv, r);
        stv = wrl<SL + 9u>(stv, 0u);
        stv = wrl<SL + 12u>(stv, lab);
        b = AGNES_VMSG_DECISION;
        break;
    default:
        break;
    }
    v.flags = (v.flags & ~0xFFu) | step;
    stv = wrl<SL + 13u>(stv, v.flags);
    view_tables(v);
    if (nr) return b == AGNES_VMSG_TIMEOUT_PRECOMMIT ? AGNES_VMSG_NEW_ROUND_TIMEOUT_PRECOMMIT
                 : b == AGNES_VMSG_DECISION           ? AGNES_VMSG_NEW_ROUND_DECISION
                                                      : AGNES_VMSG_NEW_ROUND;
    return b;
}

template <typename T>
__device__ __forceinline__ T sel4(const T (&x)[VPL], uint32_t s) { /* s wave-uniform */
    if (s == 0) return x[0];
    if (s == 1) return x[1];
    if (s == 2) return x[2];
    return x[3];
}

/* lanes whose vote s lies at a chunk position in [lo, hi) */
__device__ __forceinline__ uint64_t win(uint32_t s, uint32_t lo, uint32_t hi) {
    const uint32_t a0 = lo > s ? (lo - s + 3u) >> 2 : 0u;
    const uint32_t a1 = hi > s ? (hi - s + 3u) >> 2 : 0u;
    const uint64_t m1 = a1 >= 64u ? ~0ull : ((1ull << a1) - 1ull);
    const uint64_t m0 = a0 >= 64u ? ~0ull : ((1ull << a0) - 1ull);
    return m1 & ~m0;
}

/* the first chunk position in [lo, hi) whose vote s is set in ballot b[s]; CHUNK if none */
__device__ __forceinline__ uint32_t first_of(const uint64_t (&b)[VPL], uint32_t lo, uint32_t hi) {
    uint32_t f = CHUNK;
#pragma unroll
    for (uint32_t s = 0; s < VPL; ++s) {
        const uint64_t m = b[s] & win(s, lo, hi);
        if (m) {
            const uint32_t p = 4u * (uint32_t)__builtin_ctzll(m) + s;
            f = p < f ? p : f;
        }
    }
    return f;
}

/* the last chunk position in [lo, hi) whose vote s is set in ballot b[s]; CHUNK if none */
__device__ __forceinline__ uint32_t last_of(const uint64_t (&b)[VPL], uint32_t lo, uint32_t hi) {
    uint32_t f = CHUNK;
#pragma unroll
    for (uint32_t s = 0; s < VPL; ++s) {
        const uint64_t m = b[s] & win(s, lo, hi);
        if (m) {
            const uint32_t p = 4u * (63u - (uint32_t)__builtin_clzll(m)) + s;
            f = (f == CHUNK || p > f) ? p : f;
        }
    }
    return f;
}

} // namespace fast
} // namespace agnes

#endif
