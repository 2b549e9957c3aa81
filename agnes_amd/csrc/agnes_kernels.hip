/*
 * agnes_kernels.hip — gfx950 kernels of the Agnes vote-tally engine.
 *
 * K1-K4 fused (tally_kernel): one wave64 per instance (grid-stride over
 * instances), 64 consecutive votes of the instance per step, one vote per lane:
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
#include "agnes_gen.h"
#include "agnes_internal.h"

namespace agnes {

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t rdl(uint32_t x, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l);
}
__device__ __forceinline__ uint64_t rdl(uint64_t x, uint32_t l) {
    uint32_t lo = rdl((uint32_t)x, l), hi = rdl((uint32_t)(x >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t rfl(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
    return ((uint64_t)rfl((uint32_t)(x >> 32)) << 32) | rfl((uint32_t)x);
}
__device__ __forceinline__ uint64_t lanemask_le(uint32_t l) { return (2ull << l) - 1ull; }

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

__device__ __forceinline__ uint64_t scan(uint64_t x) {
    x = dpp_step64<0x111, 0xf>(x);
    x = dpp_step64<0x112, 0xf>(x);
    x = dpp_step64<0x114, 0xf>(x);
    x = dpp_step64<0x118, 0xf>(x);
    x = dpp_step64<0x142, 0xa>(x);
    x = dpp_step64<0x143, 0xc>(x);
    return x;
}

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

/* Does the vote-derived event (skip flag, tally code 1..5) change the state, and
 * which message does it produce when it does not? */
__device__ __forceinline__ void sm_classify(const Sm& s, int64_t r, uint32_t ev, uint32_t lab,
                                            bool skip, bool& change, uint32_t& msg) {
    change = false;
    msg = AGNES_VMSG_NONE;
    if (s.step == AGNES_STEP_COMMIT) return;
    if (skip && s.round < r) {
        change = true;
        return;
    }
    const bool eqr = s.round == r;
    if (!eqr) {
        change = ev == AGNES_CODE_PRECOMMIT_VALUE;
        return;
    }
    switch (ev) {
    case AGNES_CODE_POLKA_ANY:
        if (s.step == AGNES_STEP_PREVOTE) msg = AGNES_VMSG_TIMEOUT_PREVOTE;
        break;
    case AGNES_CODE_POLKA_NIL:
        change = s.step == AGNES_STEP_PREVOTE;
        break;
    case AGNES_CODE_POLKA_VALUE:
        if (s.step == AGNES_STEP_PREVOTE) change = true;
        else if (s.step == AGNES_STEP_PRECOMMIT)
            change = !(s.valid && s.valid_round == s.round && s.valid_value == lab);
        break;
    case AGNES_CODE_PRECOMMIT_ANY:
        msg = AGNES_VMSG_TIMEOUT_PRECOMMIT;
        break;
    case AGNES_CODE_PRECOMMIT_VALUE:
        change = true;
        break;
    default:
        break;
    }
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

/* ------------------------------------------------------------------ */
/* LDS layout of one wave                                              */

struct WaveLds {
    uint64_t* vw;       /* [2R] value-bucket weight per (round,type)        */
    uint64_t* vn;       /* [2R] nil-bucket weight                           */
    uint64_t* skw;      /* [R]  RoundSkip weight of distinct validators      */
    uint32_t* lv;       /* [2R] last value label                            */
    uint32_t* first_v;  /* [2R][nv] DEDUP: first local index per (r,t,val)  */
    uint32_t* first_s;  /* [R][nv]  SKIP:  first local index per (r,val)    */
};

__host__ __device__ inline uint64_t align16(uint64_t x) { return (x + 15u) & ~15ull; }

__host__ __device__ inline void lds_layout(uint32_t mode, uint32_t flags, uint32_t R, uint32_t nv,
                                           uint64_t* o_first_v, uint64_t* o_first_s,
                                           uint64_t* total) {
    uint64_t o = 0;
    o += 2ull * R * 8u;          /* vw  */
    o += 2ull * R * 8u;          /* vn  */
    o += (uint64_t)R * 8u;       /* skw */
    o += 2ull * R * 4u;          /* lv  */
    o = align16(o);
    *o_first_v = o;
    if (mode == AGNES_MODE_DEDUP) o = align16(o + 2ull * R * nv * 4u);
    *o_first_s = o;
    if (flags & AGNES_FLAG_ROUND_SKIP) o = align16(o + (uint64_t)R * nv * 4u);
    *total = o;
}

__device__ inline void fill_u32(uint32_t* p, uint64_t n, uint32_t v, uint32_t lane) {
    const uint64_t n4 = n >> 2;
    uint4* q = reinterpret_cast<uint4*>(p);
    const uint4 vv = make_uint4(v, v, v, v);
    for (uint64_t k = lane; k < n4; k += 64) q[k] = vv;
    for (uint64_t k = (n4 << 2) + lane; k < n; k += 64) p[k] = v;
}

/* ------------------------------------------------------------------ */
/* fused tally kernel                                                  */

template <bool WIDE, uint32_t MODE, bool SKIP, bool SM>
__device__ __forceinline__ void run_instance(const agnes_tally_args& a, const WaveLds& L,
                                             uint32_t i, uint32_t set, bool set_ok,
                                             const agnes_set_info& si, uint64_t beg, uint64_t end,
                                             uint64_t& n_bad) {
    using W = typename std::conditional<WIDE, uint64_t, uint32_t>::type;
    const uint32_t lane = lane_id();
    const uint32_t R = a.max_rounds;
    const uint32_t nv = a.n_vals;
    const agnes_vote_batch& vb = a.vb;
    const bool need_val = vb.weight == nullptr || MODE == AGNES_MODE_DEDUP || SKIP;
    const bool has_w = vb.weight != nullptr;
    const uint64_t pbase = (uint64_t)set * nv;
    const int64_t total = si.total;
    const bool track_label = a.carry != nullptr; /* carried executors keep their label */

    Sm s;
    if (SM) s = sm_load(&a.states[i]);

    for (uint64_t c = beg; c < end; c += 64) {
        const uint64_t j = c + lane;
        const bool valid = j < end;
        uint32_t inst = 0, value = 0, val = 0, r = 0, t = 0;
        if (valid) {
            inst = vb.instance[j];
            r = vb.round[j];
            t = vb.type[j];
            value = vb.value[j];
            val = vb.validator[j];
        }
        const bool ok = valid && inst == i && r < R && t <= 1u &&
                        (!need_val || (set_ok && val < nv)) && (has_w || set_ok);
        W w = 0;
        if (ok) {
            if (has_w) w = (W)vb.weight[j];
            else if (WIDE) w = (W)a.power[pbase + val];
            else w = (W)a.power32[pbase + val];
        }
        const uint32_t local = (uint32_t)(j - beg);
        bool acc = ok;
        if (MODE == AGNES_MODE_DEDUP) {
            uint32_t* e = &L.first_v[(r * 2u + t) * nv + val];
            if (ok) atomicMin(e, local);
            __builtin_amdgcn_wave_barrier();
            if (ok) acc = *(volatile uint32_t*)e == local;
        }
        bool sfirst = false;
        if (SKIP) {
            uint32_t* e = &L.first_s[r * nv + val];
            if (ok) atomicMin(e, local);
            __builtin_amdgcn_wave_barrier();
            if (ok) sfirst = *(volatile uint32_t*)e == local;
        }
        n_bad += __builtin_popcountll(ballot(valid && !ok));

        const bool isnil = value == AGNES_NIL;
        const uint32_t slot = r * 2u + t;
        W pv = 0, pn = 0;
        uint32_t lab = 0;
        uint64_t rem = ballot(acc);
        while (rem) {
            const uint32_t k = rdl(slot, (uint32_t)__builtin_ctzll(rem));
            const bool in = acc && slot == k;
            const uint64_t m = ballot(in);
            rem &= ~m;
            const W sv = scan((W)((in && !isnil) ? w : (W)0));
            const W sn = scan((W)((in && isnil) ? w : (W)0));
            const W cv = (W)L.vw[k], cn = (W)L.vn[k];
            if (in) {
                pv = cv + sv;
                pn = cn + sn;
            }
            L.vw[k] = (uint64_t)(W)(cv + rdl(sv, 63u));
            L.vn[k] = (uint64_t)(W)(cn + rdl(sn, 63u));
            if (SM || track_label) { /* Thresh::Value payload: last value written (round_votes.rs:53) */
                const uint64_t mv = ballot(in && !isnil);
                const uint64_t le = mv & lanemask_le(lane);
                const uint32_t src = le ? 63u - (uint32_t)__builtin_clzll(le) : 0u;
                const uint32_t got = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)value);
                const uint32_t cl = L.lv[k];
                if (in) lab = le ? got : cl;
                if (mv) L.lv[k] = rdl(value, 63u - (uint32_t)__builtin_clzll(mv));
            }
            __builtin_amdgcn_wave_barrier();
        }
        W ps = 0;
        if (SKIP) {
            rem = ballot(acc);
            while (rem) {
                const uint32_t kr = rdl(r, (uint32_t)__builtin_ctzll(rem));
                const bool in = acc && r == kr;
                rem &= ~ballot(in);
                const W ss = scan((W)((in && sfirst) ? w : (W)0));
                const W cs = (W)L.skw[kr];
                if (in) ps = cs + ss;
                L.skw[kr] = (uint64_t)(W)(cs + rdl(ss, 63u));
                __builtin_amdgcn_wave_barrier();
            }
        }

        uint32_t code;
        if (!ok) {
            code = AGNES_CODE_INVALID;
        } else if (!acc) {
            code = AGNES_CODE_REJECTED;
        } else {
            bool qv, qn, qa, q3;
            if (WIDE) { /* literal i64 wrapping: round_votes.rs:32 */
                const int64_t t2 = (int64_t)(2ull * (uint64_t)total);
                qv = (int64_t)(3ull * (uint64_t)pv) > t2;
                qn = (int64_t)(3ull * (uint64_t)pn) > t2;
                qa = (int64_t)(3ull * ((uint64_t)pv + (uint64_t)pn)) > t2;
                q3 = (int64_t)(3ull * (uint64_t)ps) > total;
            } else {
                qv = (uint32_t)pv > si.q2;
                qn = (uint32_t)pn > si.q2;
                qa = (uint32_t)pv + (uint32_t)pn > si.q2;
                q3 = (uint32_t)ps > si.q1;
            }
            /* to_event, vote_executor.rs:26-36 */
            const uint32_t ev = qv ? (t ? AGNES_CODE_PRECOMMIT_VALUE : AGNES_CODE_POLKA_VALUE)
                              : qn ? (t ? AGNES_CODE_NONE : AGNES_CODE_POLKA_NIL)
                              : qa ? (t ? AGNES_CODE_PRECOMMIT_ANY : AGNES_CODE_POLKA_ANY)
                                   : AGNES_CODE_NONE;
            code = ev | ((SKIP && q3) ? AGNES_CODE_SKIP : 0u);
        }

        if (SM) { /* consensus_executor.rs:64-68: State::apply(v.round, event) */
            const uint32_t evc = code & AGNES_CODE_EVENT_MASK;
            const bool skp = (code & AGNES_CODE_SKIP) != 0;
            const bool pend = acc && (code & 0x0Fu) != 0u;
            uint64_t P = ballot(pend);
            uint32_t msg = 0;
            while (P) {
                bool change;
                uint32_t cm;
                sm_classify(s, (int64_t)r, evc, lab, skp, change, cm);
                const bool inP = (P >> lane) & 1ull;
                const uint64_t Cm = ballot(inP && change);
                const uint32_t first = Cm ? (uint32_t)__builtin_ctzll(Cm) : 64u;
                if (inP && lane < first) msg = cm;
                if (!Cm) break;
                const int64_t fr = (int64_t)rdl(r, first);
                const uint32_t fev = rdl(evc, first);
                const uint32_t flab = rdl(lab, first);
                const bool fsk = rdl((uint32_t)skp, first) != 0u;
                MsgOut m1, m2;
                bool h1 = false, h2 = false;
                if (fsk) h1 = sm_apply(s, fr, AGNES_EV_ROUND_SKIP, 0u, 0, a.flags, m1);
                if (fev) h2 = sm_apply(s, fr, fev + 3u, flab, 0, a.flags, m2);
                const uint32_t vm = vmsg_of(h1, h2, m2);
                if (lane == first) msg = vm;
                P = first >= 63u ? 0ull : (P & (~0ull << (first + 1u)));
            }
            code |= msg << AGNES_CODE_MSG_SHIFT;
        }
        if (valid) a.codes[j] = (uint8_t)code;
    }
    if (SM && lane == 0) sm_store(&a.states[i], s);
}

template <uint32_t MODE, bool SKIP, bool SM>
__global__ __launch_bounds__(256) void tally_kernel(agnes_tally_args a, uint32_t lds_per_wave) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t lane = lane_id();
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint32_t R = a.max_rounds;
    const uint32_t nv = a.n_vals;

    uint64_t o_fv, o_fs, o_tot;
    lds_layout(MODE, SKIP ? AGNES_FLAG_ROUND_SKIP : 0u, R, nv, &o_fv, &o_fs, &o_tot);
    unsigned char* base = smem + (uint64_t)wave * lds_per_wave;
    WaveLds L;
    L.vw = reinterpret_cast<uint64_t*>(base);
    L.vn = L.vw + 2u * R;
    L.skw = L.vn + 2u * R;
    L.lv = reinterpret_cast<uint32_t*>(L.skw + R);
    L.first_v = reinterpret_cast<uint32_t*>(base + o_fv);
    L.first_s = reinterpret_cast<uint32_t*>(base + o_fs);

    uint64_t n_bad = 0;
    const uint32_t n_inst = a.vb.n_instances;
    const uint32_t stride = gridDim.x * AGNES_WAVES_PER_BLOCK;
    for (uint32_t i = blockIdx.x * AGNES_WAVES_PER_BLOCK + wave; i < n_inst; i += stride) {
        /* clamp: malformed offsets never make the kernel read or write past n_votes */
        uint64_t end = rfl64(a.vb.offsets[i + 1]);
        end = end < a.vb.n_votes ? end : a.vb.n_votes;
        uint64_t beg = rfl64(a.vb.offsets[i]);
        beg = beg < end ? beg : end;
        uint32_t set = a.vb.instance_set ? a.vb.instance_set[i] : (a.n_sets ? i % a.n_sets : 0u);
        set = rfl(set);
        const bool set_ok = set < a.n_sets;
        agnes_set_info si;
        if (set_ok) {
            si = a.sets[set];
        } else {
            si.total = 0;
            si.q2 = si.q1 = 0;
            si.maxpow = 0;
            si.fast = 0;
        }
        const uint64_t len = end - beg;
        const bool fast = a.vb.weight == nullptr && a.carry == nullptr && set_ok && si.fast &&
                          len < (1ull << 32) && len * (uint64_t)si.maxpow < (1ull << 31);

        /* per-instance executors: RoundVotes::new for every round (round_votes.rs:83-90) */
        for (uint32_t k = lane; k < 2u * R; k += 64) {
            if (a.carry) {
                const agnes_carry_rec cr = a.carry[(uint64_t)i * 2u * R + k];
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
        if (MODE == AGNES_MODE_DEDUP) fill_u32(L.first_v, 2ull * R * nv, 0xFFFFFFFFu, lane);
        if (SKIP) fill_u32(L.first_s, (uint64_t)R * nv, 0xFFFFFFFFu, lane);
        __builtin_amdgcn_wave_barrier();

        if (fast) run_instance<false, MODE, SKIP, SM>(a, L, i, set, set_ok, si, beg, end, n_bad);
        else run_instance<true, MODE, SKIP, SM>(a, L, i, set, set_ok, si, beg, end, n_bad);

        __builtin_amdgcn_wave_barrier();
        if (a.carry) {
            for (uint32_t k = lane; k < 2u * R; k += 64) {
                agnes_carry_rec cr;
                cr.value_w = (int64_t)L.vw[k];
                cr.nil_w = (int64_t)L.vn[k];
                cr.value = L.lv[k];
                cr.pad = 0;
                a.carry[(uint64_t)i * 2u * R + k] = cr;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0 && n_bad) atomicAdd(a.n_invalid, (unsigned long long)n_bad);
}

/* ------------------------------------------------------------------ */
/* batched State::apply over explicit events: one instance per lane    */

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
            agnes_gen_vote_at(p.seed, p.instance_base + lo, j - off[lo], sh, p.nil_permille, p.order);
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

template <uint32_t MODE, bool SKIP, bool SM>
static hipError_t launch_t(const agnes_tally_args* a, uint32_t lpw, int num_cus, hipStream_t st) {
    const uint32_t n = a->vb.n_instances;
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + AGNES_WAVES_PER_BLOCK - 1) / AGNES_WAVES_PER_BLOCK;
    const uint64_t lds = (uint64_t)lpw * AGNES_WAVES_PER_BLOCK;
    uint64_t per_cu = 8;
    if (lds) {
        const uint64_t by_lds = (160ull * 1024ull) / lds;
        if (by_lds < per_cu) per_cu = by_lds ? by_lds : 1;
    }
    const uint64_t cap = (uint64_t)(num_cus > 0 ? num_cus : 256) * per_cu;
    if (blocks > cap) blocks = cap;
    if (lds > 48u * 1024u) {
        hipError_t e = hipFuncSetAttribute(
            reinterpret_cast<const void*>(&agnes::tally_kernel<MODE, SKIP, SM>),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((agnes::tally_kernel<MODE, SKIP, SM>), dim3((uint32_t)blocks), dim3(256),
                       (size_t)lds, st, *a, lpw);
    return hipGetLastError();
}

hipError_t agnes_launch_tally(const agnes_tally_args* a, uint32_t mode, int num_cus,
                              hipStream_t st) {
    const bool skip = (a->flags & AGNES_FLAG_ROUND_SKIP) != 0;
    const bool sm = (a->flags & AGNES_FLAG_STATE_MACHINE) != 0 && a->states != nullptr;
    const uint32_t lpw = (uint32_t)agnes_lds_per_wave(mode, a->flags, a->max_rounds, a->n_vals);
    if (mode == AGNES_MODE_DEDUP) {
        if (skip) return sm ? launch_t<1, true, true>(a, lpw, num_cus, st)
                            : launch_t<1, true, false>(a, lpw, num_cus, st);
        return sm ? launch_t<1, false, true>(a, lpw, num_cus, st)
                  : launch_t<1, false, false>(a, lpw, num_cus, st);
    }
    if (skip) return sm ? launch_t<0, true, true>(a, lpw, num_cus, st)
                        : launch_t<0, true, false>(a, lpw, num_cus, st);
    return sm ? launch_t<0, false, true>(a, lpw, num_cus, st)
              : launch_t<0, false, false>(a, lpw, num_cus, st);
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
