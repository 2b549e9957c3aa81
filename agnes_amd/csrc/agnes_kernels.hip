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
/* x of lane `src` (ds_bpermute) */
__device__ __forceinline__ uint32_t shfl(uint32_t x, uint32_t src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)x);
}
__device__ __forceinline__ uint64_t shfl(uint64_t x, uint32_t src) {
    return ((uint64_t)shfl((uint32_t)(x >> 32), src) << 32) | shfl((uint32_t)x, src);
}

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

/* Vote events against a wave-uniform state, vectorised by per-state lookup masks.
 * idx = code*2 + eqr (code 1..5 = PolkaAny..PrecommitValue, eqr = s.round == r).
 * chg bit idx: the event changes the state (applied on the scalar path);
 * msg nibble idx: the message a NON-changing event produces. */
struct SmTab {
    uint64_t msg;
    uint32_t chg;
    uint32_t pv_pc;      /* PolkaValue at eqr in Precommit: change iff valid differs (:202) */
    uint32_t vsame;      /* valid == Some{round: s.round, ..}                           */
    uint32_t vval;       /* valid value                                                 */
    uint32_t r8;         /* s.round when in [0,255], else 0x100 (never a u8 round)      */
    int32_t rlt;         /* clamp(s.round, -1, 256): u8 round r > rlt <=> s.round < r   */
};

__device__ __forceinline__ SmTab sm_tab(const Sm& s) {
    SmTab t;
    const bool pv = s.step == AGNES_STEP_PREVOTE;
    t.msg = (uint64_t)AGNES_VMSG_TIMEOUT_PRECOMMIT << ((AGNES_CODE_PRECOMMIT_ANY * 2 + 1) * 4); /* :208 */
    t.chg = (1u << (AGNES_CODE_PRECOMMIT_VALUE * 2)) | (1u << (AGNES_CODE_PRECOMMIT_VALUE * 2 + 1)); /* :211 */
    if (pv) {
        t.msg |= (uint64_t)AGNES_VMSG_TIMEOUT_PREVOTE << ((AGNES_CODE_POLKA_ANY * 2 + 1) * 4); /* :196 */
        t.chg |= (1u << (AGNES_CODE_POLKA_NIL * 2 + 1)) | (1u << (AGNES_CODE_POLKA_VALUE * 2 + 1));
    }
    t.pv_pc = s.step == AGNES_STEP_PRECOMMIT;
    t.vsame = s.valid && s.valid_round == s.round;
    t.vval = s.valid_value;
    t.r8 = (s.round >= 0 && s.round <= 255) ? (uint32_t)s.round : 0x100u;
    t.rlt = s.round < -1 ? -1 : (s.round > 256 ? 256 : (int32_t)s.round);
    return t;
}

__device__ __forceinline__ void sm_classify(const SmTab& t, uint32_t r, uint32_t code, uint32_t lab,
                                            bool skip, bool& change, uint32_t& msg) {
    const uint32_t idx = code * 2u + (r == t.r8 ? 1u : 0u);
    const bool pvpc = t.pv_pc && idx == AGNES_CODE_POLKA_VALUE * 2u + 1u && !(t.vsame && t.vval == lab);
    change = ((t.chg >> idx) & 1u) || (skip && (int32_t)r > t.rlt) || pvpc;
    msg = change ? 0u : (uint32_t)(t.msg >> (idx * 4u)) & 0xFu;
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
/* LDS of one wave                                                     */

/* Two carry buffers (ping-pong): the executors of the instance left open at a
 * chunk end live in buffer `pp`; a chunk that opens a new instance writes that
 * instance's carries into the other buffer.  Per buffer: RoundVotes of every
 * round = value/nil weights + last value label per (round, type) slot, and the
 * RoundSkip weight per round. */
struct CarryBuf {
    uint64_t* vw;  /* [2R] */
    uint64_t* vn;  /* [2R] */
    uint64_t* skw; /* [R]  */
    uint32_t* lv;  /* [2R] */
};

struct WaveLds {
    unsigned char* cbase; /* carry buffer 0; buffer 1 at cbase + cbytes */
    uint32_t cbytes;
    uint32_t R;
    uint32_t* first_v; /* DEDUP [2R][nv]: epoch<<LB | (LMASK - local) of the first vote */
    uint32_t* first_s; /* SKIP  [R][nv]:  same, per (round, validator)                  */
};

__device__ __forceinline__ CarryBuf carry_buf(const WaveLds& L, uint32_t b) {
    CarryBuf cb;
    cb.vw = reinterpret_cast<uint64_t*>(L.cbase + b * L.cbytes);
    cb.vn = cb.vw + 2u * L.R;
    cb.skw = cb.vn + 2u * L.R;
    cb.lv = reinterpret_cast<uint32_t*>(cb.skw + L.R);
    return cb;
}

__host__ __device__ inline uint64_t align16(uint64_t x) { return (x + 15u) & ~15ull; }

__host__ __device__ inline void lds_layout(uint32_t mode, uint32_t flags, uint32_t R, uint32_t nv,
                                           uint64_t* o_first_v, uint64_t* o_first_s,
                                           uint64_t* total) {
    uint64_t o = 2ull * align16(48ull * R); /* 2 x (vw 16R + vn 16R + skw 8R + lv 8R) */
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

__device__ inline void zero_carry(const CarryBuf& b, uint32_t R, uint32_t lane) {
    for (uint32_t k = lane; k < 2u * R; k += 64) {
        b.vw[k] = 0;
        b.vn[k] = 0;
        b.lv[k] = 0;
    }
    for (uint32_t k = lane; k < R; k += 64) b.skw[k] = 0;
}

/* ------------------------------------------------------------------ */
/* fused tally kernel                                                  */

/* Per-lane view of the instances vbase + lane of the wave's range (a 64-wide
 * window, reloaded as the stream advances; read back with v_readlane). */
struct Window {
    uint64_t end;  /* offsets[k+1] (clamped to n_votes)          */
    int64_t tot;   /* total_weight of the instance's set          */
    uint32_t q2;   /* fast-path quorum threshold floor(2t/3)     */
    uint32_t q1;   /* fast-path RoundSkip threshold floor(t/3)   */
    uint32_t pb;   /* set * n_vals: row of the power table       */
    uint32_t fl;   /* bit0: set exists; bit1: fast path provable */
};

struct Fields {
    uint32_t inst, value, val, r, t;
};

__device__ __forceinline__ Fields load_fields(const agnes_vote_batch& vb, uint64_t j, bool in) {
    Fields f = {0u, 0u, 0u, 0u, 0u};
    if (in) {
        f.inst = vb.instance[j];
        f.r = vb.round[j];
        f.t = vb.type[j];
        f.value = vb.value[j];
        f.val = vb.validator[j];
    }
    return f;
}

/* Everything a chunk needs besides its fields. */
struct Chunk {
    uint64_t c;        /* first vote of the chunk            */
    uint32_t nvalid;   /* votes in the chunk (cl - c)         */
    uint32_t cur;      /* instance of lane 0                  */
    uint32_t last;     /* instance of the last valid lane     */
    uint32_t m;        /* instance boundaries inside          */
    uint32_t hl;       /* first lane of `last` (m > 0)        */
    uint64_t cur_start;
    uint32_t ebase;
    bool last_continues;
};

template <bool WIDE, uint32_t MODE, bool SKIP, bool SM>
__device__ __forceinline__ void process_chunk(const agnes_tally_args& a, const WaveLds& L,
                                              uint32_t pp, const Chunk& ch, const Fields& f,
                                              uint32_t myi, uint32_t head, uint32_t q2l,
                                              uint32_t q1l, int64_t totl, uint32_t pbl,
                                              bool setok, Sm& st, const Sm& st_next,
                                              uint32_t lb, uint64_t& n_bad) {
    using W = typename std::conditional<WIDE, uint64_t, uint32_t>::type;
    const uint32_t lane = lane_id();
    const uint32_t R = a.max_rounds;
    const uint32_t nv = a.n_vals;
    const agnes_vote_batch& vb = a.vb;
    const bool has_w = vb.weight != nullptr;
    const bool need_val = !has_w || MODE == AGNES_MODE_DEDUP || SKIP;
    const bool track = SM || a.carry != nullptr; /* carried executors keep their label */
    const CarryBuf P = carry_buf(L, pp);
    const CarryBuf Q = carry_buf(L, pp ^ 1u);
    const uint64_t j = ch.c + lane;
    const bool valid = lane < ch.nvalid;

    const bool ok = valid && f.inst == myi && f.r < R && f.t <= 1u &&
                    (!need_val || (setok && f.val < nv)) && (has_w || setok);
    n_bad += __builtin_popcountll(ballot(valid && !ok));
    W w = 0;
    if (ok) {
        if (has_w) w = (W)vb.weight[j];
        else if (WIDE) w = (W)a.power[(uint64_t)pbl + f.val];
        else w = (W)a.power32[(uint64_t)pbl + f.val];
    }

    /* first-vote-wins tables (DEDUP) and distinct-validator tables (RoundSkip):
     * atomic max of (epoch << lb | LMASK - local); instances of one chunk in
     * stream order, so a later instance never overwrites an earlier one's
     * entry before that one has read it back. */
    bool acc = ok, sfirst = false;
    if (MODE == AGNES_MODE_DEDUP || SKIP) {
        const uint32_t lmask = (lb >= 32u) ? 0xFFFFFFFFu : ((1u << lb) - 1u);
        const uint64_t start = (myi == ch.cur) ? ch.cur_start : ch.c + head;
        const uint32_t loc = (uint32_t)(j - start);
        for (uint32_t k = ch.cur; k <= ch.last; ++k) {
            const bool inseg = ok && myi == k;
            if (!ballot(inseg)) continue;
            const uint32_t enc = ((k - ch.ebase + 1u) << lb) | (lmask - loc);
            uint32_t* ev = nullptr;
            uint32_t* es = nullptr;
            if (MODE == AGNES_MODE_DEDUP) ev = &L.first_v[(f.r * 2u + f.t) * nv + f.val];
            if (SKIP) es = &L.first_s[f.r * nv + f.val];
            if (inseg) {
                if (MODE == AGNES_MODE_DEDUP) atomicMax(ev, enc);
                if (SKIP) atomicMax(es, enc);
            }
            __builtin_amdgcn_wave_barrier();
            if (inseg) {
                if (MODE == AGNES_MODE_DEDUP) acc = *(volatile uint32_t*)ev == enc;
                if (SKIP) sfirst = *(volatile uint32_t*)es == enc;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }

    /* K2: per (round,type) slot present: unsegmented inclusive scans; a lane's
     * prefix = scan - scan[just before its instance's first lane], or + the
     * carried executor for the instance open since an earlier chunk. */
    const bool isnil = f.value == AGNES_NIL;
    const uint32_t slot = f.r * 2u + f.t;
    const uint32_t hidx = head ? head - 1u : 0u;
    const uint64_t ge_head = ~((1ull << head) - 1ull);
    const bool multi = ch.m != 0u;
    /* carries are needed after the chunk when the last instance continues, or
     * when they are persisted (carry mode: one instance per chunk) */
    const bool upd = ch.last_continues || a.carry != nullptr;
    W pv = 0, pn = 0;
    uint32_t lab = 0;
    uint64_t rem = ballot(acc);
    while (rem) {
        const uint32_t k = rdl(slot, (uint32_t)__builtin_ctzll(rem));
        const bool in = acc && slot == k;
        rem &= ~ballot(in);
        const W sv = scan((W)((in && !isnil) ? w : (W)0));
        const W sn = scan((W)((in && isnil) ? w : (W)0));
        const W cv = (W)P.vw[k], cn = (W)P.vn[k];
        W bv = cv, bn = cn;
        if (multi) {
            const W gv = shfl(sv, hidx), gn = shfl(sn, hidx);
            bv = head ? (W)(0 - gv) : cv;
            bn = head ? (W)(0 - gn) : cn;
        }
        if (in) {
            pv = sv + bv;
            pn = sn + bn;
        }
        if (upd) {
            const W tv = rdl(sv, 63u), tn = rdl(sn, 63u);
            if (!multi) {
                P.vw[k] = (uint64_t)(W)(cv + tv);
                P.vn[k] = (uint64_t)(W)(cn + tn);
            } else {
                Q.vw[k] = (uint64_t)(W)(tv - rdl(sv, ch.hl - 1u));
                Q.vn[k] = (uint64_t)(W)(tn - rdl(sn, ch.hl - 1u));
            }
        }
        if (track) { /* Thresh::Value payload: last value written (round_votes.rs:53) */
            const uint64_t mv = ballot(in && !isnil);
            const uint64_t le = mv & lanemask_le(lane) & ge_head;
            const uint32_t src = le ? 63u - (uint32_t)__builtin_clzll(le) : 0u;
            const uint32_t got = shfl(f.value, src);
            const uint32_t cl = (head == 0u) ? P.lv[k] : 0u;
            if (in) lab = isnil ? (le ? got : cl) : f.value;
            if (upd) {
                const uint64_t mvl = multi ? (mv & ~((1ull << ch.hl) - 1ull)) : mv;
                if (mvl) (multi ? Q : P).lv[k] = rdl(f.value, 63u - (uint32_t)__builtin_clzll(mvl));
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    W ps = 0;
    if (SKIP) { /* RoundSkip weight of distinct validators per round, same scheme */
        rem = ballot(acc);
        while (rem) {
            const uint32_t kr = rdl(f.r, (uint32_t)__builtin_ctzll(rem));
            const bool in = acc && f.r == kr;
            rem &= ~ballot(in);
            const W ss = scan((W)((in && sfirst) ? w : (W)0));
            const W cs = (W)P.skw[kr];
            W bs = cs;
            if (multi) { /* bpermute with every lane active: inactive sources read as 0 */
                const W gs = shfl(ss, hidx);
                bs = head ? (W)(0 - gs) : cs;
            }
            if (in) ps = ss + bs;
            if (upd) {
                const W ts = rdl(ss, 63u);
                if (!multi) P.skw[kr] = (uint64_t)(W)(cs + ts);
                else Q.skw[kr] = (uint64_t)(W)(ts - rdl(ss, ch.hl - 1u));
            }
            __builtin_amdgcn_wave_barrier();
        }
    }

    /* K3: is_quorum precedence (round_votes.rs:58-66) and to_event (vote_executor.rs:26-36) */
    uint32_t code;
    if (!ok) {
        code = AGNES_CODE_INVALID;
    } else if (!acc) {
        code = AGNES_CODE_REJECTED;
    } else {
        bool qv, qn, qa, q3;
        if (WIDE) {
            const int64_t t2 = (int64_t)(2ull * (uint64_t)totl);
            qv = (int64_t)(3ull * (uint64_t)pv) > t2;
            qn = (int64_t)(3ull * (uint64_t)pn) > t2;
            qa = (int64_t)(3ull * ((uint64_t)pv + (uint64_t)pn)) > t2;
            q3 = (int64_t)(3ull * (uint64_t)ps) > totl;
        } else {
            qv = (uint32_t)pv > q2l;
            qn = (uint32_t)pn > q2l;
            qa = (uint32_t)pv + (uint32_t)pn > q2l;
            q3 = (uint32_t)ps > q1l;
        }
        const uint32_t ev = qv ? (f.t ? AGNES_CODE_PRECOMMIT_VALUE : AGNES_CODE_POLKA_VALUE)
                          : qn ? (f.t ? AGNES_CODE_NONE : AGNES_CODE_POLKA_NIL)
                          : qa ? (f.t ? AGNES_CODE_PRECOMMIT_ANY : AGNES_CODE_POLKA_ANY)
                               : AGNES_CODE_NONE;
        code = ev | ((SKIP && q3) ? AGNES_CODE_SKIP : 0u);
    }

    /* K4: State::apply(v.round, event) per instance in stream order
     * (consensus_executor.rs:64-68) */
    if (SM) {
        const uint32_t evc = code & AGNES_CODE_EVENT_MASK;
        const bool skp = (code & AGNES_CODE_SKIP) != 0u;
        const bool pend_any = acc && (code & 0x0Fu) != 0u;
        uint32_t msg = 0;
        for (uint32_t k = ch.cur; k <= ch.last; ++k) {
            Sm s = (k == ch.cur) ? st : (k == ch.cur + 1u ? st_next : sm_load(&a.states[k]));
            uint64_t P2 = ballot(pend_any && myi == k);
            while (P2 && s.step != AGNES_STEP_COMMIT) {
                const SmTab tb = sm_tab(s);
                bool change;
                uint32_t cm;
                sm_classify(tb, f.r, evc, lab, skp, change, cm);
                const bool inP = (P2 >> lane) & 1ull;
                const uint64_t Cm = ballot(inP && change);
                const uint32_t first = Cm ? (uint32_t)__builtin_ctzll(Cm) : 64u;
                if (inP && lane < first) msg = cm;
                if (!Cm) break;
                const int64_t fr = (int64_t)rdl(f.r, first);
                const uint32_t fev = rdl(evc, first);
                const uint32_t flab = rdl(lab, first);
                const bool fsk = rdl((uint32_t)skp, first) != 0u;
                MsgOut m1, m2;
                bool h1 = false, h2 = false;
                if (fsk) h1 = sm_apply(s, fr, AGNES_EV_ROUND_SKIP, 0u, 0, a.flags, m1);
                if (fev) h2 = sm_apply(s, fr, fev + 3u, flab, 0, a.flags, m2);
                const uint32_t vm = vmsg_of(h1, h2, m2);
                if (lane == first) msg = vm;
                P2 = first >= 63u ? 0ull : (P2 & (~0ull << (first + 1u)));
            }
            if (k == ch.last && ch.last_continues) st = s;
            else if (lane == 0) sm_store(&a.states[k], s);
        }
        code |= msg << AGNES_CODE_MSG_SHIFT;
    }
    if (valid) a.codes[j] = (uint8_t)code;
}

template <uint32_t MODE, bool SKIP, bool SM>
__global__ __launch_bounds__(256) void tally_kernel(agnes_tally_args a, uint32_t lds_per_wave) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t lane = lane_id();
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint32_t R = a.max_rounds;
    const uint32_t nv = a.n_vals;
    const agnes_vote_batch& vb = a.vb;
    const uint32_t n = vb.n_instances;
    const uint64_t NV = vb.n_votes;

    /* contiguous instance range of this wave: one vote stream */
    const uint32_t Wn = gridDim.x * AGNES_WAVES_PER_BLOCK;
    const uint32_t gw = blockIdx.x * AGNES_WAVES_PER_BLOCK + wave;
    const uint32_t ia = (uint32_t)(((uint64_t)n * gw) / Wn);
    const uint32_t ib = (uint32_t)(((uint64_t)n * (gw + 1u)) / Wn);
    if (ia >= ib) return;

    uint64_t o_fv, o_fs, o_tot;
    lds_layout(MODE, SKIP ? AGNES_FLAG_ROUND_SKIP : 0u, R, nv, &o_fv, &o_fs, &o_tot);
    unsigned char* base = smem + (uint64_t)wave * lds_per_wave;
    WaveLds L;
    L.cbase = base;
    L.cbytes = (uint32_t)align16(48ull * R);
    L.R = R;
    L.first_v = reinterpret_cast<uint32_t*>(base + o_fv);
    L.first_s = reinterpret_cast<uint32_t*>(base + o_fs);
    if (MODE == AGNES_MODE_DEDUP) fill_u32(L.first_v, 2ull * R * nv, 0u, lane);
    if (SKIP) fill_u32(L.first_s, (uint64_t)R * nv, 0u, lane);

    const uint32_t lb = a.epoch_shift;               /* bits of the local vote index */
    const uint32_t emax = lb >= 31u ? 1u : ((1u << (32u - lb)) - 1u); /* epochs per table fill */
    const bool tables = MODE == AGNES_MODE_DEDUP || SKIP;

    auto off_at = [&](uint32_t k) -> uint64_t {
        const uint64_t o = vb.offsets[k];
        return o < NV ? o : NV;
    };
    const uint64_t v0 = rfl64(off_at(ia));
    uint64_t vend = rfl64(off_at(ib));
    vend = vend > v0 ? vend : v0;

    Window win;
    uint32_t vbase = ia;
    auto load_window = [&](uint32_t b) {
        vbase = b;
        const uint32_t k = b + lane;
        const bool in = k < ib;
        const uint64_t st = in ? off_at(k) : vend;
        const uint64_t en = in ? off_at(k + 1u) : vend;
        uint32_t set = 0;
        if (in) set = vb.instance_set ? vb.instance_set[k] : (a.n_sets ? k % a.n_sets : 0u);
        const bool sok = in && set < a.n_sets;
        agnes_set_info si;
        if (sok) {
            si = a.sets[set];
        } else {
            si.total = 0;
            si.q2 = si.q1 = si.maxpow = si.fast = 0;
        }
        const uint64_t len = en > st ? en - st : 0ull;
        const bool fast = sok && si.fast && vb.weight == nullptr && a.carry == nullptr &&
                          len < (1ull << 32) && len * (uint64_t)si.maxpow < (1ull << 31);
        win.end = en;
        win.tot = si.total;
        win.q2 = si.q2;
        win.q1 = si.q1;
        win.pb = set * nv;
        win.fl = (sok ? 1u : 0u) | (fast ? 2u : 0u);
    };
    auto endof = [&](uint32_t k) -> uint64_t { return rdl(win.end, k - vbase); };
    load_window(ia);

    uint64_t n_bad = 0;
    uint64_t c = v0;
    uint32_t cur = ia;
    bool open = false;
    uint64_t cur_start = v0;
    uint32_t ebase = ia;
    uint32_t pp = 0;
    Sm st, st_next;
    Fields f = load_fields(vb, c + lane, c + lane < vend);

    while (c < vend) {
        /* instance containing vote c */
        for (;;) {
            if (cur >= ib) break;
            if (cur - vbase >= 64u) load_window(cur);
            if (endof(cur) > c) break;
            ++cur;
            open = false;
        }
        if (cur >= ib) break; /* malformed offsets */
        if (cur - vbase >= 32u && vbase + 64u < ib) load_window(cur);

        if (!open) { /* RoundVotes::new for every round (round_votes.rs:83-90) + State */
            cur_start = c;
            if (tables && cur - ebase + 1u > emax) { /* epoch space used up: clear tables */
                if (MODE == AGNES_MODE_DEDUP) fill_u32(L.first_v, 2ull * R * nv, 0u, lane);
                if (SKIP) fill_u32(L.first_s, (uint64_t)R * nv, 0u, lane);
                ebase = cur;
            }
            if (a.carry) {
                const CarryBuf cb = carry_buf(L, pp);
                for (uint32_t k = lane; k < 2u * R; k += 64) {
                    const agnes_carry_rec cr = a.carry[(uint64_t)cur * 2u * R + k];
                    cb.vw[k] = (uint64_t)cr.value_w;
                    cb.vn[k] = (uint64_t)cr.nil_w;
                    cb.lv[k] = cr.value;
                }
                for (uint32_t k = lane; k < R; k += 64) cb.skw[k] = 0;
            } else {
                zero_carry(carry_buf(L, pp), R, lane);
            }
            if (SM) st = sm_load(&a.states[cur]);
            open = true;
            __builtin_amdgcn_wave_barrier();
        }

        /* chunk [c, cl): <= 64 votes, never past the window or the epoch budget */
        uint64_t cl = c + 64u < vend ? c + 64u : vend;
        if (vbase + 63u < ib) {
            const uint64_t e = endof(vbase + 63u);
            cl = e < cl ? e : cl;
        }
        if (tables) {
            const uint64_t kcut = (uint64_t)ebase + emax - 1u;
            if (kcut < ib && kcut <= (uint64_t)vbase + 63u) {
                const uint64_t e = endof((uint32_t)kcut);
                cl = e < cl ? e : cl;
            }
        }
        if (a.carry) {
            const uint64_t e = endof(cur);
            cl = e < cl ? e : cl;
        }

        /* next chunk's fields in flight while this one computes */
        const Fields fn = load_fields(vb, cl + lane, cl + lane < vend);

        /* lane -> instance map: walk the boundaries inside the chunk */
        const uint64_t j = c + lane;
        const uint32_t wl = cur - vbase;
        uint32_t myi = cur, head = 0;
        uint32_t q2l = rdl(win.q2, wl), q1l = rdl(win.q1, wl), pbl = rdl(win.pb, wl);
        int64_t totl = (int64_t)rdl((uint64_t)win.tot, wl);
        uint32_t fll = rdl(win.fl, wl);
        uint32_t fast_all = fll;
        uint32_t k = cur, m = 0, hl = 0;
        for (;;) {
            const uint64_t ek = endof(k);
            if (ek >= cl || k + 1u >= ib) break;
            ++k;
            ++m;
            const uint32_t h = (uint32_t)(ek > c ? ek - c : 0u);
            const uint32_t wk = k - vbase;
            const uint32_t kq2 = rdl(win.q2, wk), kq1 = rdl(win.q1, wk), kpb = rdl(win.pb, wk);
            const int64_t ktot = (int64_t)rdl((uint64_t)win.tot, wk);
            const uint32_t kfl = rdl(win.fl, wk);
            fast_all &= kfl;
            if (j >= ek) {
                myi = k;
                head = h;
                q2l = kq2;
                q1l = kq1;
                pbl = kpb;
                totl = ktot;
                fll = kfl;
            }
            hl = h;
        }
        Chunk chk;
        chk.c = c;
        chk.nvalid = (uint32_t)(cl - c);
        chk.cur = cur;
        chk.last = k;
        chk.m = m;
        chk.hl = hl;
        chk.cur_start = cur_start;
        chk.ebase = ebase;
        chk.last_continues = endof(k) > cl;
        if (SM && m != 0u) st_next = sm_load(&a.states[cur + 1u]);
        if (chk.last_continues && m != 0u) zero_carry(carry_buf(L, pp ^ 1u), R, lane);
        __builtin_amdgcn_wave_barrier();

        const bool setok = (fll & 1u) != 0u;
        if (fast_all & 2u)
            process_chunk<false, MODE, SKIP, SM>(a, L, pp, chk, f, myi, head, q2l, q1l, totl, pbl,
                                                 setok, st, st_next, lb, n_bad);
        else
            process_chunk<true, MODE, SKIP, SM>(a, L, pp, chk, f, myi, head, q2l, q1l, totl, pbl,
                                                setok, st, st_next, lb, n_bad);
        __builtin_amdgcn_wave_barrier();

        /* the instance open after this chunk */
        if (chk.last_continues) {
            if (m != 0u) {
                pp ^= 1u;
                cur_start = c + hl;
            }
            cur = k;
            open = true;
        } else {
            if (a.carry) { /* persist the finished executors */
                const CarryBuf cb = carry_buf(L, pp);
                for (uint32_t q = lane; q < 2u * R; q += 64) {
                    agnes_carry_rec cr;
                    cr.value_w = (int64_t)cb.vw[q];
                    cr.nil_w = (int64_t)cb.vn[q];
                    cr.value = cb.lv[q];
                    cr.pad = 0;
                    a.carry[(uint64_t)cur * 2u * R + q] = cr;
                }
            }
            cur = k + 1u;
            open = false;
        }
        c = cl;
        f = fn;
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
    const void* fn = reinterpret_cast<const void*>(&agnes::tally_kernel<MODE, SKIP, SM>);
    if (lds > 48u * 1024u) {
        hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    /* every wave owns an equal slice of the instances: launch exactly the
     * resident grid (blocks per CU from the occupancy query, cached per LDS size) */
    static thread_local uint64_t cached_lds = ~0ull;
    static thread_local int cached_per_cu = 0;
    if (cached_lds != lds) {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, (size_t)lds) !=
                hipSuccess || per_cu < 1)
            per_cu = 1;
        cached_lds = lds;
        cached_per_cu = per_cu;
    }
    const uint64_t cap = (uint64_t)(num_cus > 0 ? num_cus : 256) * (uint64_t)cached_per_cu;
    if (blocks > cap) blocks = cap;
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
