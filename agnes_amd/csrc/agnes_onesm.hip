/*
 * agnes_onesm.hip — the State machine of ONE instance whose vote stream is split
 * into slices over waves and GPUs (C5; include/agnes.h agnes_one_sm_*,
 * agnes_amd/dist.py one_instance_states).
 *
 * Without RoundSkip, State.round never moves under vote events, so whether a vote
 * is at State.round (eqr, state_machine.rs:184) is fixed per vote, and the vote
 * events drive a three-state automaton (state_machine.rs:196-211): Prevote
 * --first PolkaNil / PolkaValue at eqr (P1)--> Precommit, any step --first
 * PrecommitValue (C, any round)--> Commit (:205: nothing after).  Every vote's
 * message then follows from its position relative to P1 and C:
 *   PolkaAny at eqr before P1 (in Prevote)      TimeoutPrevote       (:196)
 *   PolkaNil / PolkaValue at P1                  precommit nil / v    (:197-198)
 *   PrecommitAny at eqr before C                 TimeoutPrecommit     (:208)
 *   PrecommitValue at C                          Decision             (:211)
 * and the State's values from three votes: locked = P1's value (a PolkaValue,
 * :198), valid = the last non-nil PolkaValue at eqr from P1 on (from the start when
 * the State enters in Precommit) before C (:198, :202), the decision = C's vote
 * (:211).  (A nil PolkaValue's value is its bucket's last non-nil one,
 * round_votes.rs:50-54, which is an earlier candidate with the same value; the
 * crossing votes P1 (PolkaValue) and C are non-nil.)
 *
 * Three launches per slice, two exchanges between them over the ranks:
 *   scan    marks[0] = min (position << 32 | lock value or NIL) of the P1
 *           candidates, marks[1] = min (position << 32 | value) of the C
 *           candidates -- the lowest candidate lane of each wave, one atomic;
 *   (all_reduce MIN of marks[0..1])
 *   apply   the message nibbles into the codes; marks[2] = max ((position + 1)
 *           << 32 | value) of the valid candidates, marks[3] = C's round + 1
 *           (written by the slice holding C);
 *   (all_reduce MAX of marks[2..3])
 *   finish  the State (one thread).
 * Positions are global (the slice's base + index) and below 2^31, so the packed
 * marks are non-negative int64.  HBM bound: 6 B/vote (code, round, value) per
 * pass, plus the code bytes rewritten where a message lands.
 */
#include <hip/hip_runtime.h>

#include <cstdint>

#include "agnes_device.h"
#include "agnes_internal.h"

namespace agnes {
namespace onesm {

constexpr uint32_t T = 256u;
constexpr int64_t MAXM = INT64_MAX;

struct View {
    int64_t eq;    /* State.round */
    uint32_t step; /* State.step */
};

__device__ __forceinline__ View view_of(const agnes_state* s) { return View{s->round, s->step}; }

__global__ __launch_bounds__(T) void scan_kernel(const uint8_t* codes, const uint8_t* round, const uint32_t* value,
                                                 uint64_t n, uint64_t base, const agnes_state* st, int64_t* marks) {
    const View v = view_of(st);
    if (v.step == AGNES_STEP_COMMIT) return; /* :205 */
    const uint32_t lane = lane_id();
    for (uint64_t j0 = (uint64_t)blockIdx.x * T; j0 < n; j0 += (uint64_t)gridDim.x * T) {
        const uint64_t j = j0 + threadIdx.x;
        uint32_t e = AGNES_CODE_INVALID, r = 0, x = 0;
        if (j < n) {
            e = codes[j] & AGNES_CODE_EVENT_MASK;
            r = round[j];
            x = value[j];
        }
        const bool eqr = (int64_t)r == v.eq;
        const bool p1 = v.step == AGNES_STEP_PREVOTE && eqr && (e == AGNES_CODE_POLKA_NIL || e == AGNES_CODE_POLKA_VALUE);
        const bool cc = e == AGNES_CODE_PRECOMMIT_VALUE;
        const uint64_t bp = ballot(p1), bc = ballot(cc);
        /* positions grow with the lane: a wave's first candidate is its minimum */
        const int64_t pos = (int64_t)(base + j);
        if (bp && lane == (uint32_t)__builtin_ctzll(bp))
            atomicMin(reinterpret_cast<long long*>(marks), (long long)((pos << 32) | (e == AGNES_CODE_POLKA_VALUE ? x : AGNES_NIL)));
        if (bc && lane == (uint32_t)__builtin_ctzll(bc))
            atomicMin(reinterpret_cast<long long*>(marks + 1), (long long)((pos << 32) | x));
    }
}

__global__ __launch_bounds__(T) void apply_kernel(uint8_t* codes, const uint8_t* round, const uint32_t* value,
                                                  uint64_t n, uint64_t base, const agnes_state* st, int64_t* marks) {
    const View v = view_of(st);
    if (v.step == AGNES_STEP_COMMIT) return;
    const int64_t m0 = marks[0], m1 = marks[1];
    const int64_t C = m1 == MAXM ? MAXM : (m1 >> 32);
    int64_t P1 = m0 == MAXM ? MAXM : (m0 >> 32);
    if (P1 >= C) P1 = MAXM; /* the commit came first: Prevote never left at P1 */
    const uint32_t lane = lane_id();
    for (uint64_t j0 = (uint64_t)blockIdx.x * T; j0 < n; j0 += (uint64_t)gridDim.x * T) {
        const uint64_t j = j0 + threadIdx.x;
        uint32_t e = AGNES_CODE_INVALID, r = 0, x = AGNES_NIL, cb = 0;
        if (j < n) {
            cb = codes[j];
            e = cb & AGNES_CODE_EVENT_MASK;
            r = round[j];
            x = value[j];
        }
        const int64_t pos = (int64_t)(base + j);
        const bool eqr = (int64_t)r == v.eq;
        uint32_t msg = AGNES_VMSG_NONE;
        if (pos < C) {
            if (e == AGNES_CODE_PRECOMMIT_ANY && eqr) msg = AGNES_VMSG_TIMEOUT_PRECOMMIT;
            if (e == AGNES_CODE_POLKA_ANY && eqr && v.step == AGNES_STEP_PREVOTE && pos < P1)
                msg = AGNES_VMSG_TIMEOUT_PREVOTE;
            if (pos == P1) msg = e == AGNES_CODE_POLKA_VALUE ? AGNES_VMSG_PRECOMMIT_VALUE : AGNES_VMSG_PRECOMMIT_NIL;
        } else if (pos == C) {
            msg = AGNES_VMSG_DECISION;
        }
        if (msg) codes[j] = (uint8_t)(cb | (msg << AGNES_CODE_MSG_SHIFT));
        const bool vc = e == AGNES_CODE_POLKA_VALUE && eqr && x != AGNES_NIL && pos < C &&
                        ((v.step == AGNES_STEP_PREVOTE && pos >= P1) || v.step == AGNES_STEP_PRECOMMIT);
        const uint64_t bv = ballot(vc);
        if (bv && lane == 63u - (uint32_t)__builtin_clzll(bv)) /* a wave's last candidate is its maximum */
            atomicMax(reinterpret_cast<long long*>(marks + 2), (long long)(((pos + 1) << 32) | x));
        if (pos == C) atomicMax(reinterpret_cast<long long*>(marks + 3), (long long)r + 1);
    }
}

__global__ void finish_kernel(const int64_t* marks, agnes_state* st) {
    if (threadIdx.x != 0) return;
    agnes_state s = *st;
    if (s.step == AGNES_STEP_COMMIT) return;
    const int64_t m0 = marks[0], m1 = marks[1], m2 = marks[2], m3 = marks[3];
    const int64_t C = m1 == MAXM ? MAXM : (m1 >> 32);
    const int64_t P1 = m0 == MAXM ? MAXM : (m0 >> 32);
    if (P1 < C) { /* Prevote -> Precommit (:197-198); a PolkaValue locks (:198) */
        s.step = AGNES_STEP_PRECOMMIT;
        const uint32_t lv = (uint32_t)m0;
        if (lv != AGNES_NIL) {
            s.locked_present = 1;
            s.locked_round = s.round;
            s.locked_value = lv;
        }
    }
    if (m2 != 0) { /* the last valid candidate (:198, :202) */
        s.valid_present = 1;
        s.valid_round = s.round;
        s.valid_value = (uint32_t)m2;
    }
    if (C != MAXM) { /* commit (:211) */
        s.step = AGNES_STEP_COMMIT;
        s.decided = 1;
        s.decision_round = m3 - 1;
        s.decision_value = (uint32_t)m1;
    }
    *st = s;
}

} // namespace onesm
} // namespace agnes

static dim3 onesm_grid(uint64_t n, int num_cus) {
    const uint64_t blocks = (n + agnes::onesm::T - 1u) / agnes::onesm::T;
    const uint64_t cap = (uint64_t)(num_cus > 0 ? num_cus : 256) * 8u;
    return dim3((uint32_t)(blocks < cap ? (blocks ? blocks : 1u) : cap));
}

hipError_t agnes_launch_one_sm(int pass, const uint8_t* codes, const uint8_t* round, const uint32_t* value, uint64_t n,
                               uint64_t base, agnes_state* state, int64_t* marks, int num_cus, hipStream_t st) {
    using namespace agnes::onesm;
    if (pass == 2) {
        AgnesKt kt("one_sm_finish", st);
        hipLaunchKernelGGL(finish_kernel, dim3(1), dim3(64), 0, st, marks, state);
        return hipGetLastError();
    }
    if (n == 0) return hipSuccess;
    if (pass == 0) {
        AgnesKt kt("one_sm_scan", st);
        hipLaunchKernelGGL(scan_kernel, onesm_grid(n, num_cus), dim3(T), 0, st, codes, round, value, n, base, state, marks);
    } else {
        AgnesKt kt("one_sm_apply", st);
        hipLaunchKernelGGL(apply_kernel, onesm_grid(n, num_cus), dim3(T), 0, st, const_cast<uint8_t*>(codes), round,
                           value, n, base, state, marks);
    }
    return hipGetLastError();
}
