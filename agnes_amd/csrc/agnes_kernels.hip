/*
 * agnes_kernels.hip — gfx950 kernels of the Agnes vote-tally engine.
 *
 * K1-K4 fused (tally_kernel): each wave64 owns a contiguous range of instances
 * and tallies them one at a time in 256-vote chunks = 4 rows of 64 (every load
 * a coalesced 64-lane row; the next chunk's loads in flight while one computes):
 *
 *   K1 ingest   coalesced SoA loads (instance, round, type, value, validator)
 *               + gather w = power[set][validator]          (consensus_executor.rs:62-63
 *                                                             replaced by validators.rs:7)
 *   dedup       first-vote-wins per (round, type, validator): ds_min_u32 of the vote's
 *               local index into an LDS table, then read back — order-independent, so
 *               the lowest index (= first in stream order) wins deterministically
 *   K2 tally    per distinct (round, type) key present in the 64 lanes: a masked
 *               wave64 inclusive scan (DPP row_shr 1/2/4/8 + row_bcast 15/31) of the
 *               value-bucket and nil-bucket weights, plus the key's carry from LDS —
 *               exactly VoteCount::add_vote's running sums in stream order
 *               (round_votes.rs:48-56), last value label via ballot + ds_bpermute
 *   K3 quorum   is_quorum precedence Value > Nil > Any > Init (round_votes.rs:58-66),
 *               to_event (vote_executor.rs:26-36), RoundSkip +1/3 (extension)
 *   K4 state    State::apply (state_machine.rs:183-322) on the wave-uniform state:
 *               each pass classifies every pending lane against the current state
 *               in parallel; lanes before the first state-CHANGING event get their
 *               messages at once, the changing lane is applied on the scalar path,
 *               then the pass repeats — sequential semantics, ~1 pass per change.
 *
 * Two arithmetic paths per instance (wave-uniform branch):
 *   fast  all sums provably < 2^31 (non-negative powers, len * maxpow < 2^31):
 *         u32 scans, quorum as `s > floor(2t/3)` (exact, see agnes_internal.h)
 *   wide  anything else (caller weights, negative/huge powers, carried state):
 *         u64 scans, literal wrapping `3*v > 2*t` in two's complement.
 *
 * No MFMA: the path is HBM-bound integer work.
 */
#include "agnes_device.h"
#include "agnes_gen.h"
#include "agnes_internal.h"

namespace agnes {

/* ------------------------------------------------------------------ */
/* State machine (state_machine.rs:183-322)                            */

struct Sm {
    int64_t height, round, locked_round, valid_round, decision_round;
    uint32_t locked_value, valid_value, decision_value;
    uint32_t step, locked, valid, decided;
};

struct MsgOut {
    int64_t round, pol_round;
    uint32_t value, kind, vote_type, timeout_step;
};

__device__ __forceinline__ Sm sm_load(const agnes_state* p) {
    Sm s;
    s.height = p->height;
    s.round = p->round;
    s.locked_round = p->locked_round;
    s.valid_round = p->valid_round;
    s.decision_round = p->decision_round;
    s.locked_value = p->locked_value;
    s.valid_value = p->valid_value;
    s.decision_value = p->decision_value;
    s.step = p->step;
    s.locked = p->locked_present;
    s.valid = p->valid_present;
    s.decided = p->decided;
    return s;
}

__device__ __forceinline__ void sm_store(agnes_state* p, const Sm& s) {
    p->height = s.height;
    p->round = s.round;
    p->locked_round = s.locked_round;
    p->valid_round = s.valid_round;
    p->decision_round = s.decision_round;
    p->locked_value = s.locked_value;
    p->valid_value = s.valid_value;
    p->decision_value = s.decision_value;
    p->step = (uint8_t)s.step;
    p->locked_present = (uint8_t)s.locked;
    p->valid_present = (uint8_t)s.valid;
    p->decided = (uint8_t)s.decided;
}

__device__ __forceinline__ void sm_next_step(Sm& s) { /* :58-66 */
    if (s.step == AGNES_STEP_NEW_ROUND) s.step = AGNES_STEP_PROPOSE;
    else if (s.step == AGNES_STEP_PROPOSE) s.step = AGNES_STEP_PREVOTE;
    else if (s.step == AGNES_STEP_PREVOTE) s.step = AGNES_STEP_PRECOMMIT;
}

/* fn apply (:183-214); returns whether a Message was produced */
__device__ bool sm_apply(Sm& s, int64_t round, uint32_t k, uint32_t v, int64_t pol,
                         uint32_t flags, MsgOut& m) {
    m.round = 0;
    m.pol_round = 0;
    m.value = 0;
    m.kind = AGNES_MSG_NONE;
    m.vote_type = 0;
    m.timeout_step = 0;
    const bool eqr = s.round == round;
    if (s.step == AGNES_STEP_COMMIT) return false; /* :205 (no earlier arm matches Commit) */
    if (s.step == AGNES_STEP_NEW_ROUND && eqr) {
        if (k == AGNES_EV_NEW_ROUND_PROPOSER) { /* :187 propose :222-229 */
            sm_next_step(s);
            m.kind = AGNES_MSG_PROPOSAL;
            m.round = s.round;
            m.value = s.valid ? s.valid_value : v;
            m.pol_round = s.valid ? s.valid_round : -1;
            return true;
        }
        if (k == AGNES_EV_NEW_ROUND) { /* :188 :278-281 */
            sm_next_step(s);
            m.kind = AGNES_MSG_TIMEOUT;
            m.round = s.round;
            m.timeout_step = AGNES_TIMEOUT_PROPOSE;
            return true;
        }
    }
    if (s.step == AGNES_STEP_PROPOSE && eqr) {
        if (k == AGNES_EV_PROPOSAL && pol >= -1 && pol < s.round) { /* :191 prevote :237-246 */
            sm_next_step(s);
            uint32_t out = v;
            if (s.locked && !(s.locked_round <= pol)) {
                const bool same = (flags & AGNES_FLAG_DISTINCT_VALUES) ? s.locked_value == v : true;
                out = same ? v : AGNES_NIL;
            }
            m.kind = AGNES_MSG_VOTE;
            m.vote_type = AGNES_PREVOTE;
            m.round = s.round;
            m.value = out;
            return true;
        }
        if (k == AGNES_EV_PROPOSAL_INVALID || k == AGNES_EV_TIMEOUT_PROPOSE) { /* :192-193 */
            sm_next_step(s);
            m.kind = AGNES_MSG_VOTE;
            m.vote_type = AGNES_PREVOTE;
            m.round = s.round;
            m.value = AGNES_NIL;
            return true;
        }
    }
    if (s.step == AGNES_STEP_PREVOTE && eqr) {
        if (k == AGNES_EV_POLKA_ANY) { /* :196 */
            m.kind = AGNES_MSG_TIMEOUT;
            m.round = s.round;
            m.timeout_step = AGNES_TIMEOUT_PREVOTE;
            return true;
        }
        if (k == AGNES_EV_POLKA_NIL || k == AGNES_EV_TIMEOUT_PREVOTE) { /* :197,:199 */
            sm_next_step(s);
            m.kind = AGNES_MSG_VOTE;
            m.vote_type = AGNES_PRECOMMIT;
            m.round = s.round;
            m.value = AGNES_NIL;
            return true;
        }
        if (k == AGNES_EV_POLKA_VALUE) { /* :198 precommit :261-264 */
            s.locked = 1;
            s.locked_round = s.round;
            s.locked_value = v;
            s.valid = 1;
            s.valid_round = s.round;
            s.valid_value = v;
            sm_next_step(s);
            m.kind = AGNES_MSG_VOTE;
            m.vote_type = AGNES_PRECOMMIT;
            m.round = s.round;
            m.value = v;
            return true;
        }
    }
    if (s.step == AGNES_STEP_PRECOMMIT && eqr && k == AGNES_EV_POLKA_VALUE) { /* :202 */
        s.valid = 1;
        s.valid_round = s.round;
        s.valid_value = v;
        return false;
    }
    if (k == AGNES_EV_PRECOMMIT_ANY && eqr) { /* :208 */
        m.kind = AGNES_MSG_TIMEOUT;
        m.round = s.round;
        m.timeout_step = AGNES_TIMEOUT_PRECOMMIT;
        return true;
    }
    if (k == AGNES_EV_TIMEOUT_PRECOMMIT && eqr) { /* :209 round_skip(s, round + 1) */
        const int64_t r = (int64_t)((uint64_t)round + 1u);
        s.round = r;
        s.step = AGNES_STEP_NEW_ROUND;
        m.kind = AGNES_MSG_NEW_ROUND;
        m.round = r;
        return true;
    }
    if (k == AGNES_EV_ROUND_SKIP && s.round < round) { /* :210 */
        s.round = round;
        s.step = AGNES_STEP_NEW_ROUND;
        m.kind = AGNES_MSG_NEW_ROUND;
        m.round = round;
        return true;
    }
    if (k == AGNES_EV_PRECOMMIT_VALUE) { /* :211 commit :320-322 */
        s.step = AGNES_STEP_COMMIT;
        s.decided = 1;
        s.decision_round = round;
        s.decision_value = v;
        m.kind = AGNES_MSG_DECISION;
        m.round = round;
        m.value = v;
        return true;
    }
    return false; /* :212 */
}

/* Vote events against a wave-uniform state, vectorised by per-state lookup masks.
 * idx = code*2 + eqr (code 1..5 = PolkaAny..PrecommitValue, eqr = s.round == r).
 * chg bit idx: the event changes the state (applied on the scalar path);
 * msg nibble idx: the message a NON-changing event produces. */
struct SmTab {
    uint32_t chg;   /* bit idx: the event changes the state (applied on the scalar path) */
    uint32_t pv;    /* step == Prevote                                               */
    uint32_t pc;    /* step == Precommit: PolkaValue at eqr changes iff valid differs (:202) */
    uint32_t vsame; /* valid == Some{round: s.round, ..}                             */
    uint32_t vval;  /* valid value                                                   */
    uint32_t r8;    /* s.round when in [0,255], else 0x100 (never a u8 round)        */
    int32_t rlt;    /* clamp(s.round, -1, 256): u8 round r > rlt <=> s.round < r      */
};

__device__ __forceinline__ SmTab sm_tab(const Sm& s) {
    SmTab t;
    t.pv = s.step == AGNES_STEP_PREVOTE;
    t.pc = s.step == AGNES_STEP_PRECOMMIT;
    t.chg = (1u << (AGNES_CODE_PRECOMMIT_VALUE * 2)) | (1u << (AGNES_CODE_PRECOMMIT_VALUE * 2 + 1)); /* :211 */
    if (t.pv) t.chg |= (1u << (AGNES_CODE_POLKA_NIL * 2 + 1)) | (1u << (AGNES_CODE_POLKA_VALUE * 2 + 1));
    t.vsame = s.valid && s.valid_round == s.round;
    t.vval = s.valid_value;
    t.r8 = (s.round >= 0 && s.round <= 255) ? (uint32_t)s.round : 0x100u;
    t.rlt = s.round < -1 ? -1 : (s.round > 256 ? 256 : (int32_t)s.round);
    return t;
}

/* Vote events against a wave-uniform state, branch-free.  idx = code*2 + eqr
 * (code 1..5 = PolkaAny..PrecommitValue, eqr = s.round == r).  change: the event
 * changes the state; msg: the message of a NON-changing event — TimeoutPrevote for
 * PolkaAny at eqr in Prevote (:196), TimeoutPrecommit for PrecommitAny at eqr (:208). */
__device__ __forceinline__ void sm_classify(const SmTab& t, uint32_t r, uint32_t code, uint32_t lab,
                                            uint32_t skip, uint32_t& change, uint32_t& msg) {
    const uint32_t idx = code * 2u + (uint32_t)(r == t.r8);
    const uint32_t pvpc = t.pc & (uint32_t)(idx == AGNES_CODE_POLKA_VALUE * 2u + 1u) &
                          ((t.vsame & (uint32_t)(t.vval == lab)) ^ 1u);
    change = ((t.chg >> idx) & 1u) | (skip & (uint32_t)((int32_t)r > t.rlt)) | pvpc;
    const uint32_t m = (idx == AGNES_CODE_POLKA_ANY * 2u + 1u) ? (t.pv ? AGNES_VMSG_TIMEOUT_PREVOTE : 0u)
                     : (idx == AGNES_CODE_PRECOMMIT_ANY * 2u + 1u) ? AGNES_VMSG_TIMEOUT_PRECOMMIT
                                                                    : 0u;
    msg = change ? 0u : m;
}

__device__ __forceinline__ uint32_t vmsg_of(bool h1, bool h2, const MsgOut& m2) {
    uint32_t b = AGNES_VMSG_NONE;
    if (h2) {
        if (m2.kind == AGNES_MSG_TIMEOUT)
            b = m2.timeout_step == AGNES_TIMEOUT_PREVOTE ? AGNES_VMSG_TIMEOUT_PREVOTE
                                                         : AGNES_VMSG_TIMEOUT_PRECOMMIT;
        else if (m2.kind == AGNES_MSG_VOTE)
            b = m2.value == AGNES_NIL ? AGNES_VMSG_PRECOMMIT_NIL : AGNES_VMSG_PRECOMMIT_VALUE;
        else
            b = AGNES_VMSG_DECISION;
    }
    if (h1) {
        if (b == AGNES_VMSG_TIMEOUT_PRECOMMIT) return AGNES_VMSG_NEW_ROUND_TIMEOUT_PRECOMMIT;
        if (b == AGNES_VMSG_DECISION) return AGNES_VMSG_NEW_ROUND_DECISION;
        return AGNES_VMSG_NEW_ROUND;
    }
    return b;
}

template <typename T>
__device__ __forceinline__ T pick4(const T (&x)[4], uint32_t e) {
    return e == 0 ? x[0] : (e == 1 ? x[1] : (e == 2 ? x[2] : x[3]));
}

/* State::apply for the events a vote can produce (RoundSkip, then the tally
 * event at the vote's round), state_machine.rs:196-211 restricted to those arms;
 * returns the message nibble.  Equivalent to sm_apply + vmsg_of for these events. */
__device__ __forceinline__ uint32_t sm_vote(Sm& s, int64_t r, uint32_t code, uint32_t lab) {
    if (s.step == AGNES_STEP_COMMIT) return AGNES_VMSG_NONE; /* :205 */
    bool nr = false;
    if ((code & AGNES_CODE_SKIP) && s.round < r) { /* :210 round_skip */
        s.round = r;
        s.step = AGNES_STEP_NEW_ROUND;
        nr = true;
    }
    uint32_t b = AGNES_VMSG_NONE;
    const bool eqr = s.round == r;
    switch (code & AGNES_CODE_EVENT_MASK) {
    case AGNES_CODE_POLKA_ANY: /* :196 */
        if (eqr && s.step == AGNES_STEP_PREVOTE) b = AGNES_VMSG_TIMEOUT_PREVOTE;
        break;
    case AGNES_CODE_POLKA_NIL: /* :197 precommit_nil */
        if (eqr && s.step == AGNES_STEP_PREVOTE) {
            s.step = AGNES_STEP_PRECOMMIT;
            b = AGNES_VMSG_PRECOMMIT_NIL;
        }
        break;
    case AGNES_CODE_POLKA_VALUE:
        if (eqr && s.step == AGNES_STEP_PREVOTE) { /* :198 precommit */
            s.locked = 1;
            s.locked_round = s.round;
            s.locked_value = lab;
            s.valid = 1;
            s.valid_round = s.round;
            s.valid_value = lab;
            s.step = AGNES_STEP_PRECOMMIT;
            b = AGNES_VMSG_PRECOMMIT_VALUE;
        } else if (eqr && s.step == AGNES_STEP_PRECOMMIT) { /* :202 set_valid_value */
            s.valid = 1;
            s.valid_round = s.round;
            s.valid_value = lab;
        }
        break;
    case AGNES_CODE_PRECOMMIT_ANY: /* :208 */
        if (eqr) b = AGNES_VMSG_TIMEOUT_PRECOMMIT;
        break;
    case AGNES_CODE_PRECOMMIT_VALUE: /* :211 commit */
        s.step = AGNES_STEP_COMMIT;
        s.decided = 1;
        s.decision_round = r;
        s.decision_value = lab;
        b = AGNES_VMSG_DECISION;
        break;
    default:
        break;
    }
    if (nr) return b == AGNES_VMSG_TIMEOUT_PRECOMMIT ? AGNES_VMSG_NEW_ROUND_TIMEOUT_PRECOMMIT
                 : b == AGNES_VMSG_DECISION           ? AGNES_VMSG_NEW_ROUND_DECISION
                                                      : AGNES_VMSG_NEW_ROUND;
    return b;
}

/* The State of the instance being tallied lives lane-distributed in one VGPR
 * (lane 16 + k = dword k of agnes_state, k < 14), so it costs no scalar registers
 * outside the state-machine loop; unpacked to scalars only while events apply. */
constexpr uint32_t SM_LANE = 16u;
__device__ __forceinline__ Sm sm_unpack(uint32_t v) {
    Sm s;
    s.height = (int64_t)(((uint64_t)rdl(v, SM_LANE + 1u) << 32) | rdl(v, SM_LANE + 0u));
    s.round = (int64_t)(((uint64_t)rdl(v, SM_LANE + 3u) << 32) | rdl(v, SM_LANE + 2u));
    s.locked_round = (int64_t)(((uint64_t)rdl(v, SM_LANE + 5u) << 32) | rdl(v, SM_LANE + 4u));
    s.valid_round = (int64_t)(((uint64_t)rdl(v, SM_LANE + 7u) << 32) | rdl(v, SM_LANE + 6u));
    s.decision_round = (int64_t)(((uint64_t)rdl(v, SM_LANE + 9u) << 32) | rdl(v, SM_LANE + 8u));
    s.locked_value = rdl(v, SM_LANE + 10u);
    s.valid_value = rdl(v, SM_LANE + 11u);
    s.decision_value = rdl(v, SM_LANE + 12u);
    const uint32_t f = rdl(v, SM_LANE + 13u);
    s.step = f & 0xFFu;
    s.locked = (f >> 8) & 0xFFu;
    s.valid = (f >> 16) & 0xFFu;
    s.decided = f >> 24;
    return s;
}
__device__ __forceinline__ uint32_t sm_pack(const Sm& s, uint32_t v) {
    v = wrl<SM_LANE + 0u>(v, (uint32_t)s.height);
    v = wrl<SM_LANE + 1u>(v, (uint32_t)((uint64_t)s.height >> 32));
    v = wrl<SM_LANE + 2u>(v, (uint32_t)s.round);
    v = wrl<SM_LANE + 3u>(v, (uint32_t)((uint64_t)s.round >> 32));
    v = wrl<SM_LANE + 4u>(v, (uint32_t)s.locked_round);
    v = wrl<SM_LANE + 5u>(v, (uint32_t)((uint64_t)s.locked_round >> 32));
    v = wrl<SM_LANE + 6u>(v, (uint32_t)s.valid_round);
    v = wrl<SM_LANE + 7u>(v, (uint32_t)((uint64_t)s.valid_round >> 32));
    v = wrl<SM_LANE + 8u>(v, (uint32_t)s.decision_round);
    v = wrl<SM_LANE + 9u>(v, (uint32_t)((uint64_t)s.decision_round >> 32));
    v = wrl<SM_LANE + 10u>(v, s.locked_value);
    v = wrl<SM_LANE + 11u>(v, s.valid_value);
    v = wrl<SM_LANE + 12u>(v, s.decision_value);
    v = wrl<SM_LANE + 13u>(v, (s.step & 0xFFu) | ((s.locked & 0xFFu) << 8) | ((s.valid & 0xFFu) << 16) |
                                  (s.decided << 24));
    return v;
}

/* ------------------------------------------------------------------ */
/* LDS of one wave: the executors of the instance being tallied        */

/* RoundVotes of every round of the current instance (round_votes.rs:74-80):
 * value / nil weight and last value label per (round, type) slot, plus the
 * RoundSkip weight per round; and the first-vote tables. */
struct WaveLds {
    uint64_t* vw;      /* [2R] */
    uint64_t* vn;      /* [2R] */
    uint64_t* skw;     /* [R]  */
    uint32_t* lv;      /* [2R] */
    uint32_t* first_v; /* DEDUP [2R][nv]: epoch << lb | (LMASK - local) of the first vote */
    uint32_t* first_s; /* SKIP  [R][nv]:  same per (round, validator)                    */
};

__host__ __device__ inline void lds_layout(uint32_t mode, uint32_t flags, uint32_t R, uint32_t nv,
                                           uint64_t* o_first_v, uint64_t* o_first_s,
                                           uint64_t* total) {
    uint64_t o = align16(48ull * R); /* vw 16R + vn 16R + skw 8R + lv 8R */
    *o_first_v = o;
    if (mode == AGNES_MODE_DEDUP) o = align16(o + 2ull * R * nv * 4u);
    *o_first_s = o;
    if (flags & AGNES_FLAG_ROUND_SKIP) o = align16(o + (uint64_t)R * nv * 4u);
    *total = o;
}

/* ------------------------------------------------------------------ */
/* fused tally kernel                                                  */

constexpr uint32_t VPL = 4;             /* consecutive votes per lane          */
constexpr uint32_t CHUNK = 64u * VPL;   /* votes per chunk (one instance pass) */

/* One chunk of the canonical SoA, lane-major: lane l holds votes c + 4l .. c + 4l + 3
 * (c 4-aligned), so the u32 columns arrive as one 16-B load per lane and the u8
 * columns as one 4-B load per lane (vote s in byte s). */
struct Raw {
    uint32_t inst[VPL], value[VPL], val[VPL];
    uint32_t r4, t4;
};

__device__ __forceinline__ void load_raw(const agnes_vote_batch& vb, uint64_t c, Raw& x) {
    const uint64_t j = c + 4u * lane_id();
    const uint64_t NV = vb.n_votes;
    if (c + CHUNK <= NV) { /* wave-uniform: the whole chunk lies inside the columns */
        const uint4 a = *reinterpret_cast<const uint4*>(vb.instance + j);
        const uint4 v = *reinterpret_cast<const uint4*>(vb.value + j);
        const uint4 d = *reinterpret_cast<const uint4*>(vb.validator + j);
        x.inst[0] = a.x; x.inst[1] = a.y; x.inst[2] = a.z; x.inst[3] = a.w;
        x.value[0] = v.x; x.value[1] = v.y; x.value[2] = v.z; x.value[3] = v.w;
        x.val[0] = d.x; x.val[1] = d.y; x.val[2] = d.z; x.val[3] = d.w;
        x.r4 = *reinterpret_cast<const uint32_t*>(vb.round + j);
        x.t4 = *reinterpret_cast<const uint32_t*>(vb.type + j);
    } else { /* the batch's last chunk */
        x.r4 = x.t4 = 0;
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s) {
            const bool in = j + s < NV;
            x.inst[s] = in ? vb.instance[j + s] : 0u;
            x.value[s] = in ? vb.value[j + s] : 0u;
            x.val[s] = in ? vb.validator[j + s] : 0u;
            x.r4 |= (in ? (uint32_t)vb.round[j + s] : 0u) << (8u * s);
            x.t4 |= (in ? (uint32_t)vb.type[j + s] : 0u) << (8u * s);
        }
    }
}

/* inclusive stream-order prefix of a[0..3] over the wave (vote 4l+s); returns the
 * chunk total.  Lane-local serial sums + one wave scan of the lane totals. */
template <typename W>
__device__ __forceinline__ W scan4(const W (&a)[VPL], W (&o)[VPL]) {
    const W l0 = a[0], l1 = l0 + a[1], l2 = l1 + a[2], l3 = l2 + a[3];
    const W inc = scan(l3);
    const W ex = inc - l3;
    o[0] = ex + l0;
    o[1] = ex + l1;
    o[2] = ex + l2;
    o[3] = ex + l3;
    return rdl(inc, 63u);
}

/* uniform facts of the instance being tallied */
struct Inst {
    uint64_t beg, end; /* its votes                        */
    uint32_t i;        /* its index                        */
    uint32_t pbase;    /* set * n_vals                     */
    uint32_t q2, q1;   /* fast-path thresholds             */
    int64_t total;     /* total_weight (wide path)         */
    uint32_t ep;       /* epoch tag of its first-vote rows */
    bool set_ok;
};

/* per-vote facts of one chunk pass, computed before anything else so that the
 * weight gather is the first memory operation issued for the chunk */
template <typename W>
struct Pre {
    uint32_t rr[VPL], tt[VPL];
    uint32_t f_valid, f_ok, f_nil; /* bit s = vote s of the lane */
    W w[VPL]; /* meaningful only where f_ok */
};

/* validation (the vote belongs to the instance, round < max_rounds, type in
 * {0,1}, validator in the set) and the K1 weight gather
 * (consensus_executor.rs:62-63 -> validators.rs:7), branch-free; the gather reads
 * the block's LDS copy of the power table when the launcher staged one */
template <bool WIDE, uint32_t MODE, bool SKIP, bool PC>
__device__ __forceinline__ void prep_chunk(const agnes_tally_args& a, const Inst& in_, uint64_t c,
                                           const Raw& x, uint32_t pc_off, Pre<
                                           typename std::conditional<WIDE, uint64_t, uint32_t>::type>& P,
                                           uint32_t& bad_lane) {
    using W = typename std::conditional<WIDE, uint64_t, uint32_t>::type;
    const uint32_t R = a.max_rounds;
    const uint32_t nv = a.n_vals;
    const agnes_vote_batch& vb = a.vb;
    const bool has_w = WIDE && vb.weight != nullptr; /* caller weights run on the i64 kernels */
    /* AGNES_FLAG_WEIGHTS_CACHED: the weights agnes_tally_partials gathered, validated as without them */
    const bool cached = has_w && (a.flags & AGNES_FLAG_WEIGHTS_CACHED);
    const bool need_val = !has_w || cached || MODE == AGNES_MODE_DEDUP || SKIP;
    /* uniform part of the checks: the validator must index the set's row when the
     * vote needs it; the weight needs a valid set unless the caller supplied it */
    const bool set_ok = in_.set_ok;
    const bool vote_ok_u = (has_w && !cached) || set_ok;
    const bool table = !has_w && (uint64_t)a.n_sets * nv > 0u;
    /* the instance's votes in this chunk: positions [lo, hi) */
    const uint32_t lo = c < in_.beg ? (uint32_t)(in_.beg - c) : 0u;
    const uint32_t hi = in_.end - c < CHUNK ? (uint32_t)(in_.end - c) : CHUNK;
    const uint32_t p0 = 4u * lane_id();
    P.f_valid = P.f_ok = P.f_nil = 0;
#pragma unroll
    for (uint32_t s = 0; s < VPL; ++s) {
        P.rr[s] = (x.r4 >> (8u * s)) & 0xFFu;
        P.tt[s] = (x.t4 >> (8u * s)) & 0xFFu;
        /* bitwise, not short-circuit: no divergent branches */
        const uint32_t valid = (uint32_t)(p0 + s >= lo) & (uint32_t)(p0 + s < hi);
        const uint32_t vidx_ok = need_val ? ((uint32_t)set_ok & (uint32_t)(x.val[s] < nv)) : 1u;
        const uint32_t ok = valid & (uint32_t)(x.inst[s] == (a.one_inst ? a.one_id : in_.i)) & (uint32_t)(P.rr[s] < R) &
                            (uint32_t)(P.tt[s] <= 1u) & vidx_ok & (uint32_t)vote_ok_u;
        bad_lane += valid & (ok ^ 1u);
        P.f_valid |= valid << s;
        P.f_ok |= ok << s;
        P.f_nil |= (uint32_t)(x.value[s] == AGNES_NIL) << s;
    }
    if (has_w) {
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s)
            P.w[s] = ((P.f_ok >> s) & 1u) ? (W)vb.weight[c + p0 + s] : (W)0;
    } else if (!table) {
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s) P.w[s] = 0;
    } else if (!WIDE && PC) { /* LDS copy of the table (lgkmcnt) */
        const uint32_t* pc = reinterpret_cast<const uint32_t*>(agnes_smem + pc_off);
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s) {
            const bool ok = (P.f_ok >> s) & 1u;
            P.w[s] = (W)pc[ok ? in_.pbase + x.val[s] : 0u]; /* used only under f_acc <= f_ok */
        }
    } else { /* HBM table; entry 0 exists, so every lane loads (no divergence) */
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s) {
            const bool ok = (P.f_ok >> s) & 1u;
            const uint32_t idx = ok ? in_.pbase + x.val[s] : 0u;
            P.w[s] = WIDE ? (W)a.power[idx] : (W)a.power32[idx]; /* used only under f_acc */
        }
    }
}

/* One pass over chunk [c, c + CHUNK) for instance in_ (votes outside
 * [in_.beg, in_.end) untouched); returns the lane's 4 code bytes, packed. */
template <bool WIDE, uint32_t MODE, bool SKIP, bool SM>
__device__ __forceinline__ uint32_t process_chunk(const agnes_tally_args& a, const WaveLds& L,
                                                  const Inst& in_, uint64_t c, const Raw& x,
                                                  const Pre<typename std::conditional<WIDE, uint64_t, uint32_t>::type>& P,
                                                  uint32_t& stv, uint32_t lb, bool ld_carry, bool st_carry) {
    using W = typename std::conditional<WIDE, uint64_t, uint32_t>::type;
    const uint32_t lane = lane_id();
    const uint32_t nv = a.n_vals;
    const bool track = SM || a.carry != nullptr; /* labels: state machine / carried executors */
    const uint32_t p0 = 4u * lane;
    const W(&w)[VPL] = P.w;
    const uint32_t f_ok = P.f_ok, f_nil = P.f_nil;
    uint32_t f_acc = f_ok;
    /* quorum tests of a running sum (round_votes.rs:32, fast path: s > floor(2t/3)) */
    auto q23 = [&](W v) -> bool {
        if (WIDE) return (int64_t)(3ull * (uint64_t)v) > (int64_t)(2ull * (uint64_t)in_.total);
        return (uint32_t)v > in_.q2;
    };

    /* first-vote-wins (DEDUP) / distinct-validator (RoundSkip) tables: atomic max of
     * (epoch << lb | LMASK - local index): the earliest vote of the instance wins,
     * entries of earlier instances (smaller epochs) are simply overwritten */
    uint32_t f_sfirst = 0;
    if (MODE == AGNES_MODE_DEDUP || SKIP) {
        const uint32_t lmask = (1u << lb) - 1u;
        const uint32_t loc0 = (uint32_t)(c - in_.beg) + p0; /* wraps only for votes before beg */
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s) {
            const uint32_t enc = (in_.ep << lb) | (lmask - (loc0 + s));
            if ((f_ok >> s) & 1u) {
                if (MODE == AGNES_MODE_DEDUP)
                    atomicMax(&L.first_v[(P.rr[s] * 2u + P.tt[s]) * nv + x.val[s]], enc);
                if (SKIP) atomicMax(&L.first_s[P.rr[s] * nv + x.val[s]], enc);
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (MODE == AGNES_MODE_DEDUP) f_acc = 0;
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s) {
            const uint32_t enc = (in_.ep << lb) | (lmask - (loc0 + s));
            if ((f_ok >> s) & 1u) {
                if (MODE == AGNES_MODE_DEDUP)
                    f_acc |= (uint32_t)(*(volatile uint32_t*)&L.first_v[(P.rr[s] * 2u + P.tt[s]) * nv + x.val[s]] ==
                                        enc) << s;
                if (SKIP) f_sfirst |= (uint32_t)(*(volatile uint32_t*)&L.first_s[P.rr[s] * nv + x.val[s]] == enc) << s;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }

    /* K2+K3: per (round,type) slot present, one stream-order scan of the value and
     * nil buckets over the chunk plus the running executor — VoteCount::add_vote's
     * sums (round_votes.rs:48-56) — and at once is_quorum with precedence
     * Value > Nil > Any > Init (:58-66) and to_event (vote_executor.rs:26-36).
     * codes: byte s = vote s's code; lab[s]: the Thresh::Value payload. */
    uint32_t codes = 0;
    uint32_t lab[VPL];
#pragma unroll
    for (uint32_t s = 0; s < VPL; ++s) lab[s] = 0;
    uint32_t rem = f_acc;
    for (;;) {
        const uint64_t lm = ballot(rem != 0u);
        if (!lm) break;
        const uint32_t kl = (uint32_t)__builtin_ctzll(lm);
        const uint32_t ks = (uint32_t)__builtin_ctz(rdl(rem, kl));
        const uint32_t key = rdl(pick4(P.rr, ks) * 2u + pick4(P.tt, ks), kl);
        const uint32_t kt = key & 1u; /* the slot's vote type */
        uint32_t inb = 0;
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s)
            inb |= (uint32_t)(((rem >> s) & 1u) && P.rr[s] * 2u + P.tt[s] == key) << s;
        rem &= ~inb;
        W cv = 0, cn = 0;
        uint32_t lbl = 0;
        if (ld_carry) {
            cv = (W)L.vw[key];
            cn = (W)L.vn[key];
            if (track) lbl = L.lv[key];
        }
        W av[VPL], an[VPL], ov[VPL], on[VPL];
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s) {
            const bool in = (inb >> s) & 1u, nil = (f_nil >> s) & 1u;
            av[s] = (in && !nil) ? w[s] : (W)0;
            an[s] = (in && nil) ? w[s] : (W)0;
        }
        const W tv = scan4(av, ov);
        const W tn = scan4(an, on);
        uint32_t qvb = 0;
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s) {
            const W pv = cv + ov[s], pn = cn + on[s];
            const bool qv = q23(pv), qn = q23(pn), qa = q23(pv + pn);
            const uint32_t ev = qv ? (kt ? AGNES_CODE_PRECOMMIT_VALUE : AGNES_CODE_POLKA_VALUE)
                              : qn ? (kt ? AGNES_CODE_NONE : AGNES_CODE_POLKA_NIL)
                              : qa ? (kt ? AGNES_CODE_PRECOMMIT_ANY : AGNES_CODE_POLKA_ANY)
                                   : AGNES_CODE_NONE;
            const bool in = (inb >> s) & 1u;
            codes |= (in ? ev : 0u) << (8u * s);
            qvb |= (uint32_t)(in && qv) << s;
        }
        if (track) { /* Thresh::Value payload: the last value written (round_votes.rs:53) */
            const uint32_t nnb = inb & ~f_nil; /* this key's value votes in the lane */
            const uint32_t lastv = nnb ? pick4(x.value, 31u - (uint32_t)__builtin_clz(nnb)) : 0u;
            const uint64_t lanes_nn = ballot(nnb != 0u);
            /* a nil vote needs a propagated label only when its value bucket is at quorum */
            if (ballot((qvb & f_nil) != 0u)) {
                const uint64_t le = lanes_nn & lanemask_lt(lane);
                const uint32_t got = shfl(lastv, le ? 63u - (uint32_t)__builtin_clzll(le) : 0u);
                uint32_t run = le ? got : lbl;
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s) {
                    if ((nnb >> s) & 1u) run = x.value[s];
                    if ((inb >> s) & 1u) lab[s] = run;
                }
            } else {
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s)
                    if ((nnb >> s) & 1u) lab[s] = x.value[s];
            }
            if (lanes_nn) lbl = rdl(lastv, 63u - (uint32_t)__builtin_clzll(lanes_nn));
        }
        if (st_carry) {
            L.vw[key] = (uint64_t)(cv + tv);
            L.vn[key] = (uint64_t)(cn + tn);
            if (track) L.lv[key] = lbl;
        }
        __builtin_amdgcn_wave_barrier();
    }

    /* RoundSkip (+1/3 of distinct validators of the vote's round, extension):
     * the same scheme keyed by round over each validator's first vote */
    if (SKIP) {
        uint32_t rs = f_acc;
        for (;;) {
            const uint64_t lm = ballot(rs != 0u);
            if (!lm) break;
            const uint32_t kl = (uint32_t)__builtin_ctzll(lm);
            const uint32_t ks = (uint32_t)__builtin_ctz(rdl(rs, kl));
            const uint32_t kr = rdl(pick4(P.rr, ks), kl);
            uint32_t inb = 0;
#pragma unroll
            for (uint32_t s = 0; s < VPL; ++s) inb |= (uint32_t)(((rs >> s) & 1u) && P.rr[s] == kr) << s;
            rs &= ~inb;
            const W cs = ld_carry ? (W)L.skw[kr] : (W)0;
            W as[VPL], os[VPL];
#pragma unroll
            for (uint32_t s = 0; s < VPL; ++s) as[s] = ((inb & f_sfirst) >> s) & 1u ? w[s] : (W)0;
            const W ts = scan4(as, os);
#pragma unroll
            for (uint32_t s = 0; s < VPL; ++s) {
                const W ps = cs + os[s];
                bool q3;
                if (WIDE) q3 = (int64_t)(3ull * (uint64_t)ps) > in_.total;
                else q3 = (uint32_t)ps > in_.q1;
                codes |= (uint32_t)(((inb >> s) & 1u) && q3) << (8u * s + 3u);
            }
            if (st_carry) L.skw[kr] = (uint64_t)(cs + ts);
            __builtin_amdgcn_wave_barrier();
        }
    }

    /* votes that are not tallied (AGNES_FLAG_MASKED_REJECTED, carried calls: a vote the
     * DEDUP mask took out is REJECTED, what agnes_dedup_reject would write after us) */
    const bool mrej = WIDE && (a.flags & AGNES_FLAG_MASKED_REJECTED) != 0u;
#pragma unroll
    for (uint32_t s = 0; s < VPL; ++s) {
        if (!((f_ok >> s) & 1u))
            codes |= (mrej && P.tt[s] == AGNES_TYPE_MASKED ? AGNES_CODE_REJECTED : AGNES_CODE_INVALID) << (8u * s);
        else if (!((f_acc >> s) & 1u)) codes |= AGNES_CODE_REJECTED << (8u * s);
    }

    /* K4: State::apply(v.round, event) in stream order (consensus_executor.rs:64-68):
     * each pass classifies every pending vote of the chunk against the current
     * (wave-uniform) state; votes before the first state change get their message,
     * the changing vote is applied on the scalar path, repeat */
    if (SM) {
        uint32_t msgs = 0; /* nibble s: vote s's message */
        uint32_t pend = 0;
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s)
            pend |= (uint32_t)(((f_acc >> s) & 1u) && ((codes >> (8u * s)) & 0x0Fu) != 0u) << s;
        if (ballot(pend != 0u) && (rdl(stv, SM_LANE + 13u) & 0xFFu) != AGNES_STEP_COMMIT) {
            Sm st = sm_unpack(stv); /* scalar State for this chunk's passes */
            bool changed = false;
            while (st.step != AGNES_STEP_COMMIT && ballot(pend != 0u)) { /* :205 */
                const SmTab tb = sm_tab(st);
                uint32_t chb = 0, cm = 0;
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s) {
                    uint32_t chg, m;
                    const uint32_t cd = (codes >> (8u * s)) & 0xFFu;
                    sm_classify(tb, P.rr[s], cd & AGNES_CODE_EVENT_MASK, lab[s], (cd >> 3) & 1u, chg, m);
                    chb |= chg << s;
                    cm |= m << (4u * s);
                }
                chb &= pend;
                const uint64_t bk = ballot(chb != 0u);
                uint32_t first = 0xFFFFFFFFu; /* chunk position 4*lane+s of the first change */
                uint32_t fl = 0, fs = 0;
                if (bk) {
                    fl = (uint32_t)__builtin_ctzll(bk);
                    fs = (uint32_t)__builtin_ctz(rdl(chb, fl));
                    first = 4u * fl + fs;
                }
                /* votes before the change: their message under this state */
                uint32_t before = 0;
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s) before |= (uint32_t)(p0 + s < first) << s;
                before &= pend;
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s)
                    if ((before >> s) & 1u) msgs = (msgs & ~(0xFu << (4u * s))) | (cm & (0xFu << (4u * s)));
                if (!bk) break;
                const int64_t fr = (int64_t)rdl(pick4(P.rr, fs), fl);
                const uint32_t fcode = (rdl(codes, fl) >> (8u * fs)) & 0xFFu;
                const uint32_t flab = rdl(pick4(lab, fs), fl);
                const uint32_t vm = sm_vote(st, fr, fcode, flab);
                changed = true;
#pragma unroll
                for (uint32_t s = 0; s < VPL; ++s) {
                    if (p0 + s == first) msgs = (msgs & ~(0xFu << (4u * s))) | (vm << (4u * s));
                    if (p0 + s <= first) pend &= ~(1u << s); /* drop every vote up to the change */
                }
            }
            if (changed) stv = sm_pack(st, stv);
        }
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s)
            codes |= ((msgs >> (4u * s)) & 0xFu) << (8u * s + AGNES_CODE_MSG_SHIFT);
    }
    return codes;
}

/* the lane's 4 code bytes of chunk c: one 4-B store when all 4 belong to the pass */
__device__ __forceinline__ void store_codes(uint8_t* codes, uint64_t c, uint32_t packed, uint32_t f_valid) {
    const uint64_t j = c + 4u * lane_id();
    if (f_valid == 0xFu) {
        *reinterpret_cast<uint32_t*>(codes + j) = packed;
    } else {
#pragma unroll
        for (uint32_t s = 0; s < VPL; ++s)
            if ((f_valid >> s) & 1u) codes[j + s] = (uint8_t)(packed >> (8u * s));
    }
}

/* set constants cached in LDS (block-shared) when the table is small */
constexpr uint32_t SET_CACHE_MAX = 1024u;
__host__ __device__ inline uint32_t set_cache_bytes(uint32_t n_sets) {
    return n_sets <= SET_CACHE_MAX ? (uint32_t)align16(20ull * n_sets) : 0u;
}
/* the u32 power table cached in LDS when it is at most 32 KB */
constexpr uint64_t POWER_CACHE_MAX = 32u * 1024u;
__host__ __device__ inline uint32_t power_cache_bytes(uint32_t n_sets, uint32_t n_vals) {
    const uint64_t b = align16(4ull * n_sets * n_vals);
    return b <= POWER_CACHE_MAX ? (uint32_t)b : 0u;
}

/* Per wave: a contiguous range of instances (or, LIST, the deferred instances
 * grid-strided), one instance at a time, 256-vote chunks; the next chunk's votes
 * and the next instance's header and State are in flight while one computes.
 * FAST kernels defer instances whose sums could reach 2^31 (or whose set is not
 * fast) to the WIDE LIST kernel. */
template <bool WIDE, uint32_t MODE, bool SKIP, bool SM, bool LIST, bool PC>
__global__ __launch_bounds__(256) void tally_kernel(agnes_tally_args a, uint32_t lds_per_wave) {
    unsigned char* const smem = agnes_smem;
    const uint32_t lane = lane_id();
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint32_t R = a.max_rounds;
    const uint32_t nv = a.n_vals;
    const agnes_vote_batch& vb = a.vb;
    const uint32_t n = vb.n_instances;
    const uint64_t NV = vb.n_votes;
    const uint32_t Wn = gridDim.x * AGNES_WAVES_PER_BLOCK;
    const uint32_t gw = blockIdx.x * AGNES_WAVES_PER_BLOCK + wave;
    /* the deferred list empty (every instance fit the u32 kernels): leave before staging */
    if (LIST && *(volatile const uint32_t*)a.list_count == 0u) return;

    /* block-shared set cache: q2[ns] q1[ns] mp[ns] (maxpow | fast<<31) tot[ns] (u64) */
    const uint32_t ns = a.n_sets;
    const uint32_t scb = a.set_cache;
    uint32_t* sc_q2 = reinterpret_cast<uint32_t*>(smem);
    uint32_t* sc_q1 = sc_q2 + ns;
    uint32_t* sc_mp = sc_q1 + ns;
    uint32_t* sc_tot = sc_mp + ns; /* lo, hi pairs */
    if (scb) {
        for (uint32_t k = threadIdx.x; k < ns; k += blockDim.x) {
            const agnes_set_info si = a.sets[k];
            sc_q2[k] = si.q2;
            sc_q1[k] = si.q1;
            sc_mp[k] = si.maxpow | (si.fast ? 0x80000000u : 0u);
            sc_tot[2 * k] = (uint32_t)si.total;
            sc_tot[2 * k + 1] = (uint32_t)((uint64_t)si.total >> 32);
        }
    }
    /* block-shared power table (u32, fast kernels) when the launcher staged one: the
     * gather is then an LDS read, waited on by lgkmcnt, not behind the vector
     * memory queue of prefetches and stores */
    uint32_t pc_off = 0xFFFFFFFFu;
    if (!WIDE && PC) {
        uint32_t* pc = reinterpret_cast<uint32_t*>(smem + scb);
        const uint32_t np = ns * nv;
        for (uint32_t k = threadIdx.x; k < np; k += blockDim.x) pc[k] = a.power32[k];
        pc_off = scb;
    }
    if (scb || (!WIDE && PC)) __syncthreads();

    uint32_t q0, qend, qstep;
    if (LIST) {
        q0 = gw;
        qend = rfl(*(volatile uint32_t*)a.list_count);
        qstep = Wn;
    } else {
        q0 = (uint32_t)(((uint64_t)n * gw) / Wn);
        qend = (uint32_t)(((uint64_t)n * (gw + 1u)) / Wn);
        qstep = 1;
    }
    if (q0 >= qend) return;

    uint64_t o_fv, o_fs, o_tot;
    lds_layout(MODE, SKIP ? AGNES_FLAG_ROUND_SKIP : 0u, R, nv, &o_fv, &o_fs, &o_tot);
    unsigned char* base = smem + scb + a.power_cache + (uint64_t)wave * lds_per_wave;
    WaveLds L;
    L.vw = reinterpret_cast<uint64_t*>(base);
    L.vn = L.vw + 2u * R;
    L.skw = L.vn + 2u * R;
    L.lv = reinterpret_cast<uint32_t*>(L.skw + R);
    L.first_v = reinterpret_cast<uint32_t*>(base + o_fv);
    L.first_s = reinterpret_cast<uint32_t*>(base + o_fs);
    const bool tables = MODE == AGNES_MODE_DEDUP || SKIP;
    if (MODE == AGNES_MODE_DEDUP) fill_u32(L.first_v, 2ull * R * nv, 0u, lane);
    if (SKIP) fill_u32(L.first_s, (uint64_t)R * nv, 0u, lane);
    const uint32_t lb = a.epoch_shift;                                /* bits of a local vote index */
    const uint32_t emax = lb >= 31u ? 1u : ((1u << (32u - lb)) - 1u); /* epochs per table fill      */
    uint32_t ep = 0;

    /* the wave's votes end at vend (contiguous mode): the next chunk is prefetched */
    const uint64_t vend = LIST ? NV : (vb.offsets[qend] < NV ? rfl64(vb.offsets[qend]) : NV);
    uint64_t pf_at = ~0ull;
    Raw pf;
    uint32_t bad_lane = 0;
    /* stores deferred until the next chunk's gather is issued (gfx9 vmcnt retires
     * in issue order: a store ahead of a load delays every wait on that load) */
    uint64_t dc_at = ~0ull;      /* chunk whose codes are pending                  */
    uint32_t dc_code = 0, dc_valid = 0;
    uint32_t ds_i = 0xFFFFFFFFu; /* instance whose State (lanes 16..29) is pending */
    uint32_t ds_word = 0;
    auto flush = [&]() {
        if (dc_at != ~0ull) store_codes(a.codes, dc_at, dc_code, dc_valid);
        dc_at = ~0ull;
        if (SM && ds_i != 0xFFFFFFFFu && lane >= SM_LANE && lane < SM_LANE + 14u)
            reinterpret_cast<uint32_t*>(&a.states[ds_i])[lane - SM_LANE] = ds_word;
        ds_i = 0xFFFFFFFFu;
    };

    /* header of instance k, spread over lanes: 0,1 = offsets[k]; 2,3 = offsets[k+1];
     * 4 = its set; 16..29 = its State (dwords 0..13) */
    auto load_hdr = [&](uint32_t k) -> uint32_t {
        uint32_t h = 0;
        if (lane < 4u) h = reinterpret_cast<const uint32_t*>(vb.offsets + k)[lane];
        else if (lane == 4u) h = vb.instance_set ? vb.instance_set[k] : (ns ? (a.one_inst ? a.one_id : k) % ns : 0u);
        else if (SM && lane >= 16u && lane < 30u) h = reinterpret_cast<const uint32_t*>(&a.states[k])[lane - 16u];
        return h;
    };
    uint32_t qi = LIST ? rfl(a.list[q0]) : q0;
    uint32_t hdr = load_hdr(qi);

    for (uint32_t q = q0; q < qend; q += qstep) {
        Inst I;
        I.i = qi;
        const uint32_t h = hdr;
        /* next instance's header in flight while this one is tallied */
        if (q + qstep < qend) {
            qi = LIST ? rfl(a.list[q + qstep]) : q + qstep;
            hdr = load_hdr(qi);
        }
        uint64_t b = ((uint64_t)rdl(h, 1u) << 32) | rdl(h, 0u);
        uint64_t e = ((uint64_t)rdl(h, 3u) << 32) | rdl(h, 2u);
        b = b < NV ? b : NV;
        e = e < NV ? e : NV;
        I.beg = b;
        I.end = e > b ? e : b;
        const uint32_t set = rdl(h, 4u);
        I.set_ok = set < ns;
        uint32_t mp = 0;
        if (!I.set_ok) {
            I.q2 = I.q1 = 0;
            I.total = 0;
        } else if (scb) {
            I.q2 = sc_q2[set];
            I.q1 = sc_q1[set];
            mp = sc_mp[set];
            I.total = (int64_t)(((uint64_t)sc_tot[2 * set + 1] << 32) | sc_tot[2 * set]);
        } else {
            const agnes_set_info si = a.sets[set];
            I.q2 = si.q2;
            I.q1 = si.q1;
            mp = si.maxpow | (si.fast ? 0x80000000u : 0u);
            I.total = si.total;
        }
        I.pbase = set * nv;
        const uint64_t len = I.end - I.beg;
        if (!WIDE) { /* sums provably < 2^31: u32 arithmetic; otherwise defer to WIDE */
            const bool fast = !I.set_ok || ((mp >> 31) && len < (1ull << 32) &&
                                            len * (uint64_t)(mp & 0x7FFFFFFFu) < (1ull << 31));
            if (!fast) {
                if (lane == 0) a.list[atomicAdd(a.list_count, 1u)] = I.i;
                continue;
            }
        }
        if (len == 0) continue; /* no votes: executors and State untouched */

        /* RoundVotes::new for every round (round_votes.rs:83-90): zero carries are
         * implicit in an instance's first chunk; LDS holds them only across chunks */
        if (tables) {
            if (++ep > emax) { /* epoch space used up: recycle the tables */
                if (MODE == AGNES_MODE_DEDUP) fill_u32(L.first_v, 2ull * R * nv, 0u, lane);
                if (SKIP) fill_u32(L.first_s, (uint64_t)R * nv, 0u, lane);
                ep = 1;
            }
        }
        I.ep = ep;
        const uint64_t c0 = I.beg & ~3ull; /* chunks are 4-aligned in the stream */
        const bool multi = I.end - c0 > CHUNK || a.carry != nullptr;
        if (multi) {
            for (uint32_t k = lane; k < 2u * R; k += 64) {
                if (a.carry) {
                    const agnes_carry_rec cr = a.carry[(uint64_t)I.i * 2u * R + k];
                    L.vw[k] = (uint64_t)cr.value_w;
                    L.vn[k] = (uint64_t)cr.nil_w;
                    L.lv[k] = cr.value;
                } else {
                    L.vw[k] = 0;
                    L.vn[k] = 0;
                    L.lv[k] = 0;
                }
            }
            for (uint32_t k = lane; k < R; k += 64) L.skw[k] = 0;
        }
        uint32_t stv = h; /* State: header lanes 16..29 */
        __builtin_amdgcn_wave_barrier();

        for (uint64_t c = c0; c < I.end; c += CHUNK) {
            Raw x;
            if (pf_at == c) {
                x = pf;
            } else {
                load_raw(vb, c, x);
            }
            /* issue order: gather of this chunk, the previous chunk's stores, then the
             * next chunk (this instance's, or the next instance's first) */
            Pre<typename std::conditional<WIDE, uint64_t, uint32_t>::type> P;
            prep_chunk<WIDE, MODE, SKIP, PC>(a, I, c, x, pc_off, P, bad_lane);
            flush();
            const uint64_t nc = c + CHUNK < I.end ? c + CHUNK : (I.end & ~3ull);
            if (!LIST && nc < vend) {
                load_raw(vb, nc, pf);
                pf_at = nc;
            }
            dc_code = process_chunk<WIDE, MODE, SKIP, SM>(a, L, I, c, x, P, stv, lb,
                                                          /*ld_carry=*/c != c0 || a.carry != nullptr,
                                                          /*st_carry=*/c + CHUNK < I.end || a.carry != nullptr);
            dc_valid = P.f_valid;
            dc_at = c;
            __builtin_amdgcn_wave_barrier();
        }
        if (SM) { /* State back (deferred) */
            ds_word = stv;
            ds_i = I.i;
        }
        if (a.carry) { /* persist the executors */
            for (uint32_t k = lane; k < 2u * R; k += 64) {
                agnes_carry_rec cr;
                cr.value_w = (int64_t)L.vw[k];
                cr.nil_w = (int64_t)L.vn[k];
                cr.value = L.lv[k];
                cr.pad = 0;
                a.carry[(uint64_t)I.i * 2u * R + k] = cr;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    flush();
    const uint32_t nb = rdl(scan(bad_lane), 63u);
    if (lane == 0 && nb) add_invalid(a.n_invalid, (unsigned long long)nb);
}

/* ------------------------------------------------------------------ */
/* batched State::apply over explicit events: one instance per lane    */

/* ------------------------------------------------------------------ */
/* ConsensusExecutor::apply_msg over a batch of message streams        */
/* (consensus_executor.rs:54-79), one instance per lane.               */

/* is_quorum in the reference's wrapping i64 (round_votes.rs:31-33) */
__device__ __forceinline__ bool q23_wrap(int64_t v, int64_t total) {
    return (int64_t)((uint64_t)v * 3u) > (int64_t)((uint64_t)total * 2u);
}

struct MsgArgs {
    agnes_vote_batch vb; /* the messages: instance, round, type (vote type / timeout step), value, validator */
    const uint8_t* kind; /* AGNES_IN_* per message */
    const int32_t* pol;  /* Proposal.pol_round per message (NULL: -1) */
    const int64_t* power;
    const agnes_set_info* sets;
    uint32_t n_sets, n_vals, max_rounds, flags;
    agnes_state* states;
    agnes_message* msgs;
    uint8_t* codes;
    unsigned long long* n_invalid;
};

/* Per lane: its instance's VoteCounts (round_votes.rs:15-19) in LDS, [key][lane] for
 * value_w, nil_w and the value slot; the State in registers.  Every message in
 * stream order: a Vote through VoteExecutor::apply (:61-69; the engine's
 * validation and power-table weight, vote_executor.rs:20-36) then its event, a
 * Proposal as Event::Proposal(pol_round, value) (:56-60), a Timeout as its Timeout
 * event (:70-77), a NewRound input as Event::NewRound / NewRoundProposer(value)
 * (the executor's answer to its own NewRound message, :31-33) — each applied at
 * the message's round (apply_event, :82-86). */
__global__ __launch_bounds__(64) void apply_msgs_kernel(MsgArgs a) {
    const uint32_t lane = threadIdx.x, i = blockIdx.x * 64u + lane;
    const uint32_t K = 2u * a.max_rounds;
    int64_t* const vw = reinterpret_cast<int64_t*>(agnes_smem);
    int64_t* const nw = vw + (size_t)K * 64u;
    uint32_t* const lab = reinterpret_cast<uint32_t*>(nw + (size_t)K * 64u);
    if (i >= a.vb.n_instances) return;
    for (uint32_t k = 0; k < K; ++k) { /* RoundVotes::new (round_votes.rs:36-45, 83-90) */
        vw[k * 64u + lane] = 0;
        nw[k * 64u + lane] = 0;
        lab[k * 64u + lane] = 0u;
    }
    const uint32_t set = a.vb.instance_set ? a.vb.instance_set[i] : (a.n_sets ? i % a.n_sets : 0u);
    const bool set_ok = set < a.n_sets;
    const int64_t total = set_ok ? a.sets[set].total : 0;
    Sm s = sm_load(&a.states[i]);
    uint64_t bad = 0;
    const uint64_t NV = a.vb.n_votes;
    uint64_t lo = a.vb.offsets[i], hi = a.vb.offsets[i + 1u];
    lo = lo < NV ? lo : NV;
    hi = hi < NV ? hi : NV;
    for (uint64_t j = lo; j < hi; ++j) {
        const uint32_t kd = a.kind[j], r = a.vb.round[j], t = a.vb.type[j], v = a.vb.value[j];
        uint32_t code = AGNES_CODE_NONE, ev = AGNES_EV_NONE, ev_val = 0;
        int64_t pol = 0;
        if (kd == AGNES_IN_VOTE) {
            const uint32_t x = a.vb.validator[j];
            const bool need_val = a.vb.weight == nullptr;
            if (a.vb.instance[j] != i || r >= a.max_rounds || t > 1u || (need_val && (!set_ok || x >= a.n_vals))) {
                code = AGNES_CODE_INVALID;
                ++bad;
            } else {
                const int64_t w = a.vb.weight ? a.vb.weight[j] : a.power[(uint64_t)set * a.n_vals + x];
                const uint32_t key = (r * 2u + t) * 64u + lane;
                if (v != AGNES_NIL) { /* add_vote :50-54, one value slot */
                    vw[key] = (int64_t)((uint64_t)vw[key] + (uint64_t)w);
                    lab[key] = v;
                } else {
                    nw[key] = (int64_t)((uint64_t)nw[key] + (uint64_t)w);
                }
                const int64_t sv = vw[key], sn = nw[key];
                uint32_t level = 0; /* :58-66 */
                if (q23_wrap(sv, total)) level = 3;
                else if (q23_wrap(sn, total)) level = 2;
                else if (q23_wrap((int64_t)((uint64_t)sv + (uint64_t)sn), total)) level = 1;
                /* to_event, vote_executor.rs:26-36 */
                if (level) {
                    if (t == AGNES_PREVOTE) ev = level == 3 ? AGNES_EV_POLKA_VALUE : (level == 2 ? AGNES_EV_POLKA_NIL : AGNES_EV_POLKA_ANY);
                    else ev = level == 3 ? AGNES_EV_PRECOMMIT_VALUE : (level == 2 ? AGNES_EV_NONE : AGNES_EV_PRECOMMIT_ANY);
                }
                ev_val = lab[key];
                code = ev == AGNES_EV_NONE ? AGNES_CODE_NONE : ev - AGNES_EV_POLKA_ANY + AGNES_CODE_POLKA_ANY;
            }
        } else if (kd == AGNES_IN_PROPOSAL) {
            ev = AGNES_EV_PROPOSAL;
            ev_val = v;
            pol = a.pol ? (int64_t)a.pol[j] : -1;
        } else if (kd == AGNES_IN_TIMEOUT && t <= 2u) {
            ev = t == AGNES_TIMEOUT_PROPOSE ? AGNES_EV_TIMEOUT_PROPOSE
                                            : (t == AGNES_TIMEOUT_PREVOTE ? AGNES_EV_TIMEOUT_PREVOTE : AGNES_EV_TIMEOUT_PRECOMMIT);
        } else if (kd == AGNES_IN_NEW_ROUND) {
            ev = v != AGNES_NIL ? AGNES_EV_NEW_ROUND_PROPOSER : AGNES_EV_NEW_ROUND;
            ev_val = v;
        } else {
            code = AGNES_CODE_INVALID; /* not a message kind */
            ++bad;
        }
        MsgOut m;
        const bool has = ev != AGNES_EV_NONE && sm_apply(s, (int64_t)r, ev, ev_val, pol, a.flags, m);
        agnes_message o;
        o.round = has ? m.round : 0;
        o.pol_round = has ? m.pol_round : 0;
        o.value = has ? m.value : 0;
        o.kind = (uint8_t)(has ? m.kind : AGNES_MSG_NONE);
        o.vote_type = (uint8_t)(has ? m.vote_type : 0);
        o.timeout_step = (uint8_t)(has ? m.timeout_step : 0);
        o.pad = 0;
        a.msgs[j] = o;
        a.codes[j] = (uint8_t)code;
    }
    sm_store(&a.states[i], s);
    if (bad) add_invalid(a.n_invalid, (unsigned long long)bad);
}

__global__ __launch_bounds__(256) void apply_events_kernel(agnes_state* states, uint32_t n,
                                                           const uint64_t* off,
                                                           const agnes_event* ev,
                                                           agnes_message* msgs, uint32_t flags) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Sm s = sm_load(&states[i]);
    for (uint64_t k = off[i]; k < off[i + 1]; ++k) {
        const agnes_event e = ev[k];
        MsgOut m;
        const bool has = sm_apply(s, e.round, e.kind, e.value, e.pol_round, flags, m);
        agnes_message o;
        o.round = has ? m.round : 0;
        o.pol_round = has ? m.pol_round : 0;
        o.value = has ? m.value : 0;
        o.kind = (uint8_t)(has ? m.kind : AGNES_MSG_NONE);
        o.vote_type = (uint8_t)(has ? m.vote_type : 0);
        o.timeout_step = (uint8_t)(has ? m.timeout_step : 0);
        o.pad = 0;
        msgs[k] = o;
    }
    sm_store(&states[i], s);
}

/* ------------------------------------------------------------------ */
/* synthetic stream generator (agnes_gen.h)                            */

__global__ __launch_bounds__(256) void gen_kernel(agnes_gen_params p, agnes_gen_shape sh,
                                                  const uint64_t* off, uint64_t n_votes,
                                                  uint32_t* instance, uint8_t* round,
                                                  uint8_t* type, uint32_t* value,
                                                  uint32_t* validator) {
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n_votes;
         j += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = p.n_instances; /* last i with off[i] <= j */
        while (hi - lo > 1u) {
            const uint32_t mid = (lo + hi) >> 1;
            if (off[mid] <= j) lo = mid;
            else hi = mid;
        }
        const agnes_gen_vote v =
            agnes_gen_vote_at(p.seed, p.instance_base + lo, j - off[lo], sh, p.nil_permille, p.order,
                              p.absent_permille);
        instance[j] = lo;
        round[j] = (uint8_t)v.round;
        type[j] = (uint8_t)v.type;
        value[j] = v.value;
        validator[j] = v.validator;
    }
}

} // namespace agnes

/* ------------------------------------------------------------------ */
/* launchers                                                           */

int64_t agnes_lds_per_wave(uint32_t mode, uint32_t flags, uint32_t max_rounds, uint32_t n_vals) {
    uint64_t fv, fs, tot;
    agnes::lds_layout(mode, flags, max_rounds, n_vals, &fv, &fs, &tot);
    return (int64_t)tot;
}

template <bool WIDE, uint32_t MODE, bool SKIP, bool SM, bool LIST>
static hipError_t launch_k(const agnes_tally_args* a, uint32_t lpw, int num_cus, hipStream_t st) {
    const uint32_t n = a->vb.n_instances;
    if (n == 0) return hipSuccess;
    const void* fn = reinterpret_cast<const void*>(&agnes::tally_kernel<WIDE, MODE, SKIP, SM, LIST, false>);
    const uint64_t wave_lds = (uint64_t)lpw * AGNES_WAVES_PER_BLOCK;
    const uint32_t scb = agnes::set_cache_bytes(a->n_sets);
    const uint32_t pcb = WIDE ? 0u : agnes::power_cache_bytes(a->n_sets, a->n_vals);
    /* every wave owns an equal slice of the instances: launch the resident grid
     * (blocks per CU from the occupancy query).  The set and power caches are
     * used only where they do not lower the blocks per CU.  Cached per (kernel,
     * LDS shape). */
    struct Occ { const void* fn; uint64_t wave_lds; uint32_t scb, pcb; int per_cu; uint32_t use_s, use_p; };
    static thread_local Occ occ[8];
    static thread_local unsigned occ_next = 0;
    Occ* o = nullptr;
    for (auto& c : occ)
        if (c.fn == fn && c.wave_lds == wave_lds && c.scb == scb && c.pcb == pcb) o = &c;
    if (!o) {
        auto blocks_per_cu = [&](uint64_t lds) -> int {
            if (lds > 160u * 1024u) return 0;
            if (lds > 48u * 1024u &&
                hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
                return 0;
            int per_cu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, (size_t)lds) != hipSuccess)
                per_cu = 0;
            return per_cu;
        };
        const int base = blocks_per_cu(wave_lds);
        o = &occ[occ_next++ % 8];
        *o = Occ{fn, wave_lds, scb, pcb, base > 0 ? base : 1, 0u, 0u};
        /* preference: both caches, power only, set only, none */
        const uint32_t cand[3][2] = {{scb, pcb}, {0u, pcb}, {scb, 0u}};
        for (const auto& cd : cand) {
            if (!cd[0] && !cd[1]) continue;
            if ((cd[0] && !scb) || (cd[1] && !pcb)) continue;
            const int pc = blocks_per_cu(wave_lds + cd[0] + cd[1]);
            if (pc > 0 && pc >= base) {
                o->per_cu = pc;
                o->use_s = cd[0];
                o->use_p = cd[1];
                break;
            }
        }
    }
    agnes_tally_args b = *a;
    b.set_cache = o->use_s;
    b.power_cache = o->use_p;
    const uint64_t lds = wave_lds + o->use_s + o->use_p;
    if (lds > 48u * 1024u) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    const uint64_t ncu = (uint64_t)(num_cus > 0 ? num_cus : 256);
    const uint64_t cap = ncu * (uint64_t)o->per_cu;
    uint64_t blocks = (n + AGNES_WAVES_PER_BLOCK - 1) / AGNES_WAVES_PER_BLOCK;
    if (blocks > cap) blocks = cap;
    if (LIST && blocks > ncu) blocks = ncu;
    bool launched = false;
    if constexpr (!WIDE) {
      if (o->use_p) {
        const void* fp = reinterpret_cast<const void*>(&agnes::tally_kernel<WIDE, MODE, SKIP, SM, LIST, true>);
        if (lds > 48u * 1024u) {
            hipError_t e = hipFuncSetAttribute(fp, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL((agnes::tally_kernel<WIDE, MODE, SKIP, SM, LIST, true>), dim3((uint32_t)blocks),
                           dim3(256), (size_t)lds, st, b, lpw);
        launched = true;
      }
    }
    if (!launched)
        hipLaunchKernelGGL((agnes::tally_kernel<WIDE, MODE, SKIP, SM, LIST, false>), dim3((uint32_t)blocks),
                           dim3(256), (size_t)lds, st, b, lpw);
    return hipGetLastError();
}

template <uint32_t MODE, bool SKIP, bool SM>
static hipError_t launch_mode(const agnes_tally_args* a, uint32_t lpw, int num_cus, bool wide_all,
                              hipStream_t st) {
    if (wide_all || ((a->flags >> AGNES_ROUTE_SHIFT) & AGNES_ROUTE_MASK) == AGNES_ROUTE_WIDE) {
        AgnesKt kt("tally_wide", st);
        return launch_k<true, MODE, SKIP, SM, false>(a, lpw, num_cus, st);
    }
    hipError_t e = hipSuccess; /* (the work-queue counters were zeroed with the invalid count) */
    {
        /* REFERENCE without RoundSkip: the fused sweep (tally + State machine in one
         * pass over the votes, agnes_sweep.hip).  DEDUP / RoundSkip: the per-instance
         * kernel, with the State machine either fused or in the one-instance-per-lane
         * apply pass (agnes_apply.hip).  AGNES_ROUTE_* in cfg->flags overrides the
         * choice (diagnostics and the route-equivalence tests; results are identical). */
        const uint32_t route = (a->flags >> AGNES_ROUTE_SHIFT) & AGNES_ROUTE_MASK;
        const bool sweep = route == AGNES_ROUTE_AUTO && MODE == AGNES_MODE_REFERENCE && !SKIP &&
                           agnes_sweep_supported(a);
        if (sweep) {
            e = agnes_launch_sweep(a, num_cus, st); /* the stream and walk kernels */
        } else {
            /* per-instance route: split (C4 1.04 vs 1.11 ms fused) unless forced fused */
            const bool split = SM && route != AGNES_ROUTE_INSTANCE && agnes_apply_codes_supported(a);
            agnes_tally_args b = *a;
            if (split) b.flags &= ~AGNES_FLAG_STATE_MACHINE;
            {
                AgnesKt kt("tally_fast", st);
                e = agnes_launch_tally_fast(&b, MODE, num_cus, st);
            }
            if (e == hipSuccess && split) {
                AgnesKt kt("apply_codes", st);
                e = agnes_launch_apply_codes(a, st);
            }
        }
    }
    if (e == hipSuccess) {
        AgnesKt kt("tally_list", st);
        e = launch_k<true, MODE, SKIP, SM, true>(a, lpw, num_cus, st);
    }
    return e;
}

hipError_t agnes_launch_tally(const agnes_tally_args* a, uint32_t mode, int num_cus, bool wide_all,
                              hipStream_t st) {
    const bool skip = (a->flags & AGNES_FLAG_ROUND_SKIP) != 0;
    const bool sm = (a->flags & AGNES_FLAG_STATE_MACHINE) != 0 && a->states != nullptr;
    const uint32_t lpw = (uint32_t)agnes_lds_per_wave(mode, a->flags, a->max_rounds, a->n_vals);
    if (mode == AGNES_MODE_DEDUP) {
        if (skip) return sm ? launch_mode<1, true, true>(a, lpw, num_cus, wide_all, st)
                            : launch_mode<1, true, false>(a, lpw, num_cus, wide_all, st);
        return sm ? launch_mode<1, false, true>(a, lpw, num_cus, wide_all, st)
                  : launch_mode<1, false, false>(a, lpw, num_cus, wide_all, st);
    }
    if (skip) return sm ? launch_mode<0, true, true>(a, lpw, num_cus, wide_all, st)
                        : launch_mode<0, true, false>(a, lpw, num_cus, wide_all, st);
    return sm ? launch_mode<0, false, true>(a, lpw, num_cus, wide_all, st)
              : launch_mode<0, false, false>(a, lpw, num_cus, wide_all, st);
}

hipError_t agnes_launch_apply_msgs(const agnes_vote_batch* vb, const uint8_t* kind, const int32_t* pol,
                                  const int64_t* power, const agnes_set_info* sets, uint32_t n_sets, uint32_t n_vals,
                                  uint32_t max_rounds, uint32_t flags, agnes_state* states, agnes_message* msgs,
                                  uint8_t* codes, unsigned long long* n_invalid, hipStream_t st) {
    const uint32_t n = vb->n_instances;
    if (n == 0) return hipSuccess;
    agnes::MsgArgs a{*vb, kind, pol, power, sets, n_sets, n_vals, max_rounds, flags, states, msgs, codes, n_invalid};
    const size_t lds = (size_t)2u * max_rounds * 64u * (2u * sizeof(int64_t) + sizeof(uint32_t));
    AgnesKt kt("apply_msgs", st);
    hipLaunchKernelGGL(agnes::apply_msgs_kernel, dim3((n + 63u) / 64u), dim3(64), lds, st, a);
    return hipGetLastError();
}

hipError_t agnes_launch_apply_events(agnes_state* states, uint32_t n, const uint64_t* off,
                                     const agnes_event* ev, agnes_message* msgs, uint32_t flags,
                                     hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(agnes::apply_events_kernel, dim3((n + 255) / 256), dim3(256), 0, st, states,
                       n, off, ev, msgs, flags);
    return hipGetLastError();
}

hipError_t agnes_launch_gen(const agnes_gen_params* p, const uint64_t* d_offsets, uint64_t n_votes,
                            uint32_t* instance, uint8_t* round, uint8_t* type, uint32_t* value,
                            uint32_t* validator, hipStream_t st) {
    if (n_votes == 0) return hipSuccess;
    const agnes_gen_shape sh =
        agnes_gen_shape_of(p->n_vals, p->dup_permille, p->equiv_permille, p->higher_permille);
    uint64_t blocks = (n_votes + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(agnes::gen_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, *p, sh,
                       d_offsets, n_votes, instance, round, type, value, validator);
    return hipGetLastError();
}
