/*
 * agnes_apply.hip — batched State::apply over a tallied vote stream, one
 * instance per lane (K4 of the hot path; consensus_executor.rs:64-68 ->
 * state_machine.rs:196-211 for the events a vote can produce).
 *
 * The tally kernels leave one code byte per vote (event bits 0..2, RoundSkip bit
 * 3).  This pass walks each instance's codes in stream order and ORs the message
 * nibble (bits 4..7) into the votes that produce one, and leaves the final State.
 *
 * What makes it a light pass: the message of a vote depends only on (event,
 * vote round == State.round, step), never on the event's value.  Values matter
 * only for the State fields written at three places — the Prevote -> Precommit
 * PolkaValue (locked = valid = {round, v}, :198), the last set_valid_value
 * (:202: later writes overwrite earlier ones and emit nothing) and the commit
 * (:211).  The walk records those vote positions and resolves their values
 * afterwards (the vote's value, or for a nil vote the last value written into
 * its bucket before it: round_votes.rs:50-54), so the loop streams 2 B per vote
 * (code, round) and writes back only the bytes that gain a message.
 *
 * Instances the tally kernel deferred to the i64 LIST kernel (sums may reach
 * 2^31) are skipped here: that kernel applies their events itself.
 *
 * EDG (agnes_tally_edges, round 6): the same walk also writes the instance's
 * edge-triggered summary (agnes_edges.hip's walk, on the final codes of each window
 * while they are in registers) to its segment, and its count -- the separate edge
 * walk over the codes, rounds and types is gone.  It reads the type column too and
 * walks on past the commit (the codes after it still change their executors' levels).
 */
#include <hip/hip_runtime.h>

#include <cstdint>

#include "agnes_device.h"
#include "agnes_fast.h"
#include "agnes_internal.h"

namespace agnes {
namespace apply {

constexpr uint32_t NOPOS = 0xFFFFFFFFu;

/* Each lane walks its instance in 64-B blocks of the code and round columns,
 * fetched by LDS-DMA into lane-private slots (4 x 16 B per column, double
 * buffered): a block is one half of an L2 line, consumed before the next block
 * is needed, so a line is fetched once although the 64 lanes of a wave read 64
 * different lines.  LDS per wave: [stage 2][column 2][k 4][lane 64][16 B]. */
constexpr uint32_t BLK = 64u, LDS_PER_WAVE = 2u * 4u * 64u * 16u, WAVES = 4u;
/* (EDG) the type column too: [column 3][k 4][lane 64][16 B] */
constexpr uint32_t LDS_PER_WAVE_EDG = 3u * 4u * 64u * 16u;

/* the bytes of a 16-B window that runs past the batch end, into the lane's slot
 * (the batch's last instance only) */
__device__ __attribute__((noinline)) void tail_fill(const uint8_t* col, uint64_t w, uint64_t NV, unsigned char* slot) {
    uint32_t o[4] = {0, 0, 0, 0};
    for (uint32_t b = 0; b < 16u && w + b < NV; ++b) o[b >> 2] |= (uint32_t)col[w + b] << (8u * (b & 3u));
    *reinterpret_cast<uint4*>(slot) = make_uint4(o[0], o[1], o[2], o[3]);
}

/* 0xFF in byte i of the result for bit i of x (x < 16) */
__device__ __forceinline__ uint32_t bytes_of(uint32_t x) {
    const uint32_t b = (x * 0x00204081u) & 0x01010101u;
    return (b << 8) - b;
}
/* 0xFF in the bytes below byte i (i <= 4) */
__device__ __forceinline__ uint32_t below_bytes(uint32_t i) { return i >= 4u ? 0xFFFFFFFFu : (1u << (8u * i)) - 1u; }
/* 0xFF in the bytes of x that are zero (exact, no borrow) */
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    const uint32_t z = ~(t | x) & 0x80808080u;
    return z | (z - (z >> 7));
}
/* 0x01 in the bytes of x greater than k (-1 <= k <= 254) */
__device__ __forceinline__ uint32_t bytes_gt(uint32_t x, int32_t k) {
    const uint32_t c = (uint32_t)(255 - k) * 0x00010001u; /* byte + 255 - k carries into bit 8 iff byte > k */
    const uint32_t te = (x & 0x00FF00FFu) + c, to = ((x >> 8) & 0x00FF00FFu) + c;
    return ((te >> 8) & 0x00010001u) | (to & 0x01000100u);
}

/* Per-byte lookup tables over the event (bits 0..2 of a code), one per eqr:
 * bits 4..7 the message of a non-changing event, bit 0 CHG (the vote changes the
 * step: PolkaNil / PolkaValue at eqr in Prevote, PrecommitValue anywhere), bit 1
 * VUPD (PolkaValue at eqr in Precommit: set_valid_value, no message).  Table
 * bytes 0..3 in lo, 4..7 in hi (v_perm_b32 selectors 0..7). */
constexpr uint32_t CHG = 0x01u, VUPD = 0x02u;
constexpr uint32_t T0LO = 0u, T0HI = CHG << 8; /* not eqr: PrecommitValue commits (:211) */
constexpr uint32_t T1HI = (AGNES_VMSG_TIMEOUT_PRECOMMIT << 4) | (CHG << 8); /* PrecommitAny :208, PrecommitValue */
__device__ __forceinline__ uint32_t t1lo_of(uint32_t step) {
    return step == AGNES_STEP_PREVOTE ? ((AGNES_VMSG_TIMEOUT_PREVOTE << 4) << 8) | (CHG << 16) | ((CHG | VUPD) << 24)
         : step == AGNES_STEP_PRECOMMIT ? (VUPD << 24)
                                        : 0u;
}

/* the value a Value event at vote j carries: the vote's own, or (nil vote) the last
 * value counted into its (round, type) bucket before it, 0 if none (VoteCount::new
 * label; one value slot, last writer wins: round_votes.rs:36-54) */
__device__ uint32_t label_of(const agnes_tally_args& a, uint64_t lo, uint64_t j) {
    const uint32_t v = a.vb.value[j];
    if (v != AGNES_NIL) return v;
    const uint32_t r = a.vb.round[j], t = a.vb.type[j];
    /* 16 votes per round trip, newest window first (aligned 16-vote windows of the
     * columns; a window straddling lo is read byte-wise) */
    for (uint64_t w = j & ~15ull;; w -= 16u) {
        const uint64_t b = w > lo ? w : lo;
        const uint64_t e = w + 16u < j ? w + 16u : j;
        if (b < e) {
            uint32_t cand = 0, vals[16];
            if (b == w && e == w + 16u) {
                const uint4 rq = *reinterpret_cast<const uint4*>(a.vb.round + w);
                const uint4 tq = *reinterpret_cast<const uint4*>(a.vb.type + w);
                const uint4 cq = *reinterpret_cast<const uint4*>(a.codes + w);
                const uint4* vq = reinterpret_cast<const uint4*>(a.vb.value + w);
                const uint4 vv4[4] = {vq[0], vq[1], vq[2], vq[3]};
                const uint32_t rr[4] = {rq.x, rq.y, rq.z, rq.w}, tt[4] = {tq.x, tq.y, tq.z, tq.w};
                const uint32_t cc[4] = {cq.x, cq.y, cq.z, cq.w};
#pragma unroll
                for (uint32_t q = 0; q < 16u; ++q) {
                    const uint32_t sh = 8u * (q & 3u);
                    const uint32_t ev = (cc[q >> 2] >> sh) & AGNES_CODE_EVENT_MASK;
                    const uint4 vx = vv4[q >> 2];
                    vals[q] = (q & 3u) == 0u ? vx.x : (q & 3u) == 1u ? vx.y : (q & 3u) == 2u ? vx.z : vx.w;
                    cand |= (uint32_t)(((rr[q >> 2] >> sh) & 0xFFu) == r && ((tt[q >> 2] >> sh) & 0xFFu) == t &&
                                       ev != AGNES_CODE_INVALID && ev != AGNES_CODE_REJECTED && vals[q] != AGNES_NIL)
                            << q;
                }
            } else {
                for (uint32_t q = 0; q < 16u; ++q) {
                    const uint64_t k = w + q;
                    vals[q] = 0u;
                    if (k < b || k >= e) continue;
                    const uint32_t ev = a.codes[k] & AGNES_CODE_EVENT_MASK;
                    vals[q] = a.vb.value[k];
                    cand |= (uint32_t)(a.vb.round[k] == r && a.vb.type[k] == t && ev != AGNES_CODE_INVALID &&
                                       ev != AGNES_CODE_REJECTED && vals[q] != AGNES_NIL)
                            << q;
                }
            }
            if (cand) {
                const uint32_t q = 31u - (uint32_t)__builtin_clz(cand);
                uint32_t out = vals[0];
#pragma unroll
                for (uint32_t x = 1; x < 16u; ++x) out = x == q ? vals[x] : out;
                return out;
            }
        }
        if (w <= lo) break;
    }
    return 0u;
}

template <bool SKIP, bool EDG>
__global__ __launch_bounds__(256) void apply_codes(agnes_tally_args a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = a.vb.n_instances, ns = a.n_sets;
    if (i >= n) return;
    /* every per-instance input at once (one latency, not a chain) */
    uint4* const sp = reinterpret_cast<uint4*>(a.states + i);
    uint64_t lo = a.vb.offsets[i], hi = a.vb.offsets[i + 1u];
    const uint64_t seg0 = lo; /* (EDG) the instance's segment */
    const uint4 s0 = sp[0], s1 = sp[1], s2 = sp[2], s3 = sp[3];
    const uint64_t NV = a.vb.n_votes;
    lo = lo < NV ? lo : NV;
    hi = hi < NV ? hi : NV;
    if (hi <= lo) {
        if (EDG) a.edge_counts[i] = 0ull;
        return;
    }
    { /* the same domain test (u32, or u64 for a.w64) as the tally kernels: the rest is the LIST kernel's */
        const uint32_t set = a.vb.instance_set ? a.vb.instance_set[i] : (ns ? i % ns : 0u);
        if (set < ns) {
            const agnes_set_info si = a.sets[set];
            const uint64_t len = hi - lo;
            if (fast::defer_si(si, len, a.w64 != 0u)) return;
        }
    }

    const uint32_t step0 = s3.y & 0xFFu; /* dword 13: step | locked << 8 | valid << 16 | decided << 24 */
    if (!EDG && step0 == AGNES_STEP_COMMIT) return; /* :205 every later event: None */
    const int64_t round0 = (int64_t)(((uint64_t)s0.w << 32) | s0.z);
    uint32_t step = step0;
    uint32_t eq8 = (round0 >= 0 && round0 <= 255) ? (uint32_t)round0 : 0x100u; /* no u8 round equals 0x100 */
    int32_t rlt = round0 < -1 ? -1 : (round0 > 256 ? 256 : (int32_t)round0);
    bool skipped = false;
    /* the positions (relative to lo) whose values the State takes */
    uint32_t lock_at = NOPOS, valid_at = NOPOS, dec_at = NOPOS, dec_round = 0;

    /* Without RoundSkip, branch-free: a window holds at most one P1 (the first
     * PolkaNil / PolkaValue at eqr in Prevote, :197-198) and one commit (the first
     * PrecommitValue, :211), so two table lookups per dword — the start step's and
     * Precommit's — and byte masks decide every vote: start-table messages before
     * P1 (or the commit), Precommit-table messages between P1 and the commit, the
     * step messages at the two, nothing after the commit. */
    auto walk_ns = [&](uint64_t w, uint4 cq, uint4 rq, uint32_t (&ow)[4]) {
        const uint32_t c4[4] = {cq.x, cq.y, cq.z, cq.w}, r4[4] = {rq.x, rq.y, rq.z, rq.w};
        const int32_t rel = (int32_t)((int64_t)w - (int64_t)lo); /* > -16 */
        const uint32_t a0 = rel < 0 ? (uint32_t)(-rel) : 0u;
        const uint64_t rem = hi - w;
        const uint32_t a1 = rem < 16u ? (uint32_t)rem : 16u;
        const uint32_t allowed = ((1u << a1) - 1u) & ~((1u << a0) - 1u); /* this instance's bytes */
        const bool eqok = eq8 < 0x100u, pv0 = step == AGNES_STEP_PREVOTE;
        const uint32_t eqrep = (eq8 & 0xFFu) * 0x01010101u;
        const uint32_t tshi = eqok ? T1HI : T0HI;
        const uint32_t tslo = eqok ? t1lo_of(step) : T0LO, tplo = eqok ? t1lo_of(AGNES_STEP_PRECOMMIT) : T0LO;
        uint32_t os[4], op[4], cvb[4], p1b[4];
#pragma unroll
        for (uint32_t d = 0; d < 4u; ++d) {
            const uint32_t e = c4[d] & 0x07070707u;
            const uint32_t q = eqok ? zero_bytes(r4[d] ^ eqrep) : 0u;
            const uint32_t bm = bytes_of((allowed >> (4u * d)) & 0xFu);
            const uint32_t z = __builtin_amdgcn_perm(T0HI, T0LO, e) & ~q;
            os[d] = ((__builtin_amdgcn_perm(tshi, tslo, e) & q) | z) & bm;
            op[d] = ((__builtin_amdgcn_perm(tshi, tplo, e) & q) | z) & bm;
            cvb[d] = zero_bytes(e ^ 0x05050505u) & bm & 0x01010101u;   /* PrecommitValue, any round */
            p1b[d] = pv0 ? (os[d] & 0x01010101u & ~cvb[d]) : 0u;       /* PolkaNil / Value at eqr */
        }
        auto first = [](const uint32_t (&m)[4]) -> uint32_t {
            uint32_t f = 16u;
#pragma unroll
            for (int d = 3; d >= 0; --d)
                if (m[d]) f = 4u * (uint32_t)d + ((uint32_t)__builtin_ctz(m[d]) >> 3);
            return f;
        };
        /* 0xFF in the bytes of dword d whose window index lies in [b, e) */
        auto span = [](uint32_t d, uint32_t b, uint32_t e) -> uint32_t {
            const uint32_t lo4 = 4u * d;
            const uint32_t bb = b > lo4 ? (b - lo4 < 4u ? b - lo4 : 4u) : 0u;
            const uint32_t ee = e > lo4 ? (e - lo4 < 4u ? e - lo4 : 4u) : 0u;
            return below_bytes(ee) & ~below_bytes(bb);
        };
        const uint32_t fc = first(cvb), fp = first(p1b);
        const bool has_p1 = fp < fc;          /* P1 before the commit (a commit ends the walk) */
        const uint32_t pre = has_p1 ? fp : fc; /* start-table messages below this byte */
        uint32_t vup[4];
#pragma unroll
        for (uint32_t d = 0; d < 4u; ++d) {
            const uint32_t mid = has_p1 ? span(d, fp + 1u, fc) : 0u;
            ow[d] = c4[d] | (os[d] & 0xF0F0F0F0u & span(d, 0u, pre)) | (op[d] & 0xF0F0F0F0u & mid);
            /* set_valid_value (:202): Precommit-table PolkaValues at eqr before the commit */
            vup[d] = (has_p1 ? op[d] & mid : (step == AGNES_STEP_PRECOMMIT ? os[d] & span(d, 0u, fc) : 0u)) &
                     0x02020202u;
        }
        if (has_p1) {
            const uint32_t sh = 8u * (fp & 3u);
            const uint32_t ev = ((fp < 8u ? (fp < 4u ? c4[0] : c4[1]) : (fp < 12u ? c4[2] : c4[3])) >> sh) & 7u;
            const uint32_t m = ev == AGNES_CODE_POLKA_VALUE ? AGNES_VMSG_PRECOMMIT_VALUE : AGNES_VMSG_PRECOMMIT_NIL;
#pragma unroll
            for (uint32_t d = 0; d < 4u; ++d) ow[d] |= d == (fp >> 2) ? m << (sh + AGNES_CODE_MSG_SHIFT) : 0u;
            if (ev == AGNES_CODE_POLKA_VALUE) lock_at = valid_at = (uint32_t)(rel + (int32_t)fp); /* :198 */
            step = AGNES_STEP_PRECOMMIT;
        }
#pragma unroll
        for (int d = 3; d >= 0; --d) { /* the last set_valid_value of the window */
            if (vup[d]) {
                valid_at = (uint32_t)(rel + (int32_t)(4u * (uint32_t)d + ((31u - (uint32_t)__builtin_clz(vup[d])) >> 3)));
                break;
            }
        }
        if (fc < 16u) { /* :211 commit */
            const uint32_t sh = 8u * (fc & 3u);
#pragma unroll
            for (uint32_t d = 0; d < 4u; ++d)
                ow[d] |= d == (fc >> 2) ? AGNES_VMSG_DECISION << (sh + AGNES_CODE_MSG_SHIFT) : 0u;
            dec_at = (uint32_t)(rel + (int32_t)fc);
            dec_round = ((fc < 8u ? (fc < 4u ? r4[0] : r4[1]) : (fc < 12u ? r4[2] : r4[3])) >> sh) & 0xFFu;
            step = AGNES_STEP_COMMIT;
        }
        if (((ow[0] ^ c4[0]) | (ow[1] ^ c4[1]) | (ow[2] ^ c4[2]) | (ow[3] ^ c4[3])) ) {
            if (rel >= 0 && rem >= 16u) {
                *reinterpret_cast<uint4*>(a.codes + w) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
            } else {
                for (uint32_t b = 0; b < 16u; ++b) {
                    const uint32_t x = (ow[b >> 2] >> (8u * (b & 3u))) & 0xFFu;
                    if (x != ((c4[b >> 2] >> (8u * (b & 3u))) & 0xFFu)) a.codes[w + b] = (uint8_t)x;
                }
            }
        }
    };

    /* one 16-B window at w of this instance (cq, rq: its code and round bytes) */
    auto walk = [&](uint64_t w, uint4 cq, uint4 rq, uint32_t (&ow)[4]) {
        const uint32_t c4[4] = {cq.x, cq.y, cq.z, cq.w}, r4[4] = {rq.x, rq.y, rq.z, rq.w};
        const int32_t rel = (int32_t)((int64_t)w - (int64_t)lo); /* > -16 */
        const uint32_t a0 = rel < 0 ? (uint32_t)(-rel) : 0u;
        const uint64_t rem = hi - w;
        const uint32_t a1 = rem < 16u ? (uint32_t)rem : 16u;
        uint32_t allowed = ((1u << a1) - 1u) & ~((1u << a0) - 1u); /* bytes of this instance not yet walked */
        ow[0] = c4[0];
        ow[1] = c4[1];
        ow[2] = c4[2];
        ow[3] = c4[3];
        /* one pass per step change inside the window (at most a few per instance) */
        for (;;) {
            const uint32_t t1lo = eq8 < 0x100u ? t1lo_of(step) : T0LO;
            const uint32_t t1hi = eq8 < 0x100u ? T1HI : T0HI;
            const uint32_t eqrep = (eq8 & 0xFFu) * 0x01010101u;
            uint32_t o[4], any_c = 0, any_v = 0;
#pragma unroll
            for (uint32_t d = 0; d < 4u; ++d) {
                const uint32_t e = c4[d] & 0x07070707u;
                const uint32_t q = zero_bytes(r4[d] ^ eqrep);
                uint32_t od = (__builtin_amdgcn_perm(t1hi, t1lo, e) & q) | (__builtin_amdgcn_perm(T0HI, T0LO, e) & ~q);
                if (SKIP) od |= (c4[d] >> 3) & bytes_gt(r4[d], rlt); /* RoundSkip to a higher round: CHG */
                od &= bytes_of((allowed >> (4u * d)) & 0xFu);
                o[d] = od;
                any_c |= od & 0x01010101u;
                any_v |= od & 0x02020202u;
            }
            uint32_t fb = 16u; /* first changing byte */
            if (any_c) {
#pragma unroll
                for (int d = 3; d >= 0; --d) {
                    const uint32_t m = o[d] & 0x01010101u;
                    if (m) fb = 4u * (uint32_t)d + ((uint32_t)__builtin_ctz(m) >> 3);
                }
            }
            const uint32_t before = fb < 16u ? (1u << fb) - 1u : 0xFFFFu;
            /* messages of the bytes before it; the last set_valid_value among them */
#pragma unroll
            for (uint32_t d = 0; d < 4u; ++d) ow[d] |= o[d] & 0xF0F0F0F0u & bytes_of((before >> (4u * d)) & 0xFu);
            if (any_v) {
#pragma unroll
                for (uint32_t d = 0; d < 4u; ++d) {
                    const uint32_t m = o[d] & 0x02020202u & bytes_of((before >> (4u * d)) & 0xFu);
                    if (m) valid_at = (uint32_t)(rel + (int32_t)(4u * d + ((31u - (uint32_t)__builtin_clz(m)) >> 3)));
                }
            }
            if (fb >= 16u) break;
            /* the changing vote (state_machine.rs:196-211 via sm_vote's arms) */
            const uint32_t sh = 8u * (fb & 3u);
            const uint32_t cdw = fb < 8u ? (fb < 4u ? c4[0] : c4[1]) : (fb < 12u ? c4[2] : c4[3]);
            const uint32_t rdw = fb < 8u ? (fb < 4u ? r4[0] : r4[1]) : (fb < 12u ? r4[2] : r4[3]);
            const uint32_t c = (cdw >> sh) & 0xFFu, r = (rdw >> sh) & 0xFFu;
            const uint32_t jo = (uint32_t)(rel + (int32_t)fb);
            bool nr = false;
            if (SKIP && (c & AGNES_CODE_SKIP) && (int32_t)r > rlt) { /* :210 round_skip(s, r) */
                eq8 = r;
                rlt = (int32_t)r;
                step = AGNES_STEP_NEW_ROUND;
                skipped = true;
                nr = true;
            }
            const uint32_t ev = c & AGNES_CODE_EVENT_MASK;
            const bool eqr = r == eq8;
            uint32_t m = AGNES_VMSG_NONE;
            if (ev == AGNES_CODE_POLKA_ANY && eqr && step == AGNES_STEP_PREVOTE) {
                m = AGNES_VMSG_TIMEOUT_PREVOTE; /* :196 */
            } else if (ev == AGNES_CODE_POLKA_NIL && eqr && step == AGNES_STEP_PREVOTE) { /* :197 */
                m = AGNES_VMSG_PRECOMMIT_NIL;
                step = AGNES_STEP_PRECOMMIT;
            } else if (ev == AGNES_CODE_POLKA_VALUE && eqr && step == AGNES_STEP_PREVOTE) {
                m = AGNES_VMSG_PRECOMMIT_VALUE; /* :198 precommit: locked = valid = {round, v} */
                step = AGNES_STEP_PRECOMMIT;
                lock_at = valid_at = jo;
            } else if (ev == AGNES_CODE_POLKA_VALUE && eqr && step == AGNES_STEP_PRECOMMIT) {
                valid_at = jo; /* :202 */
            } else if (ev == AGNES_CODE_PRECOMMIT_ANY && eqr) {
                m = AGNES_VMSG_TIMEOUT_PRECOMMIT; /* :208 */
            } else if (ev == AGNES_CODE_PRECOMMIT_VALUE) {
                m = AGNES_VMSG_DECISION; /* :211 commit */
                step = AGNES_STEP_COMMIT;
                dec_at = jo;
                dec_round = r;
            }
            if (SKIP && nr)
                m = m == AGNES_VMSG_TIMEOUT_PRECOMMIT ? AGNES_VMSG_NEW_ROUND_TIMEOUT_PRECOMMIT
                  : m == AGNES_VMSG_DECISION           ? AGNES_VMSG_NEW_ROUND_DECISION
                                                       : AGNES_VMSG_NEW_ROUND;
#pragma unroll
            for (uint32_t d = 0; d < 4u; ++d) ow[d] |= (d == (fb >> 2)) ? (m << (sh + AGNES_CODE_MSG_SHIFT)) : 0u;
            allowed &= ~((2u << fb) - 1u);
            if (step == AGNES_STEP_COMMIT || !allowed) break;
        }
        if ((ow[0] ^ c4[0]) | (ow[1] ^ c4[1]) | (ow[2] ^ c4[2]) | (ow[3] ^ c4[3])) {
            /* whole window when it is all this instance's, else its changed bytes only */
            if (rel >= 0 && rem >= 16u) {
                *reinterpret_cast<uint4*>(a.codes + w) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
            } else {
                for (uint32_t b = 0; b < 16u; ++b) {
                    const uint32_t x = (ow[b >> 2] >> (8u * (b & 3u))) & 0xFFu;
                    if (x != ((c4[b >> 2] >> (8u * (b & 3u))) & 0xFFu)) a.codes[w + b] = (uint8_t)x;
                }
            }
        }
    };

    /* (EDG) the edges of one window from its final codes (agnes_edges.hip walk_one): an
     * executor's byte is its level (code bits 0..3) | last message << 4, key round * 2 +
     * type < 16 in byte key & 7 of est0 / est1; a vote whose byte changes is an edge */
    const uint32_t keys = 2u * a.max_rounds;
    uint64_t est0 = 0, est1 = 0, ecnt = 0;
    uint4* const eout = EDG ? reinterpret_cast<uint4*>(a.edge_out) + seg0 : nullptr;
    auto edges_win = [&](uint64_t w, const uint32_t (&o4)[4], uint4 rq, uint4 tq) {
        const uint32_t r4[4] = {rq.x, rq.y, rq.z, rq.w}, t4[4] = {tq.x, tq.y, tq.z, tq.w};
        const int32_t rel = (int32_t)((int64_t)w - (int64_t)lo); /* > -16 */
        const uint32_t a0 = rel < 0 ? (uint32_t)(-rel) : 0u;
        const uint64_t rem = hi - w;
        const uint32_t a1 = rem < 16u ? (uint32_t)rem : 16u;
#pragma unroll
        for (uint32_t b = 0; b < 16u; ++b) {
            if (b < a0 || b >= a1) continue;
            const uint32_t sh8 = 8u * (b & 3u);
            const uint32_t cb = (o4[b >> 2] >> sh8) & 0xFFu, rb = (r4[b >> 2] >> sh8) & 0xFFu,
                           tb = (t4[b >> 2] >> sh8) & 0xFFu;
            const uint32_t ev = cb & AGNES_CODE_EVENT_MASK;
            const uint32_t key = rb * 2u + tb;
            if (ev == AGNES_CODE_INVALID || ev == AGNES_CODE_REJECTED || tb > 1u || key >= keys) continue;
            const uint32_t sh = 8u * (key & 7u);
            const uint32_t old = (uint32_t)((key < 8u ? est0 : est1) >> sh) & 0xFFu;
            const uint32_t msg = cb >> AGNES_CODE_MSG_SHIFT;
            const uint32_t nb = (cb & 0xFu) | (msg ? msg << AGNES_CODE_MSG_SHIFT : old & 0xF0u);
            if (nb != old) {
                const uint64_t j = w + b;
                eout[ecnt] = make_uint4((uint32_t)j, (uint32_t)(j >> 32), i, rb | (tb << 8) | (cb << 16) | (old << 24));
                ++ecnt;
                const uint64_t x = (uint64_t)(old ^ nb) << sh;
                if (key < 8u) est0 ^= x;
                else est1 ^= x;
            }
        }
    };

    /* the lane's 64-B blocks by LDS-DMA; a window past the batch end is clamped to
     * an in-bounds one (16 <= NV: the launcher) and filled byte-wise after the wait */
    const uint32_t lane = threadIdx.x & 63u;
    unsigned char* const wbase = agnes_smem + rfl(threadIdx.x >> 6) * (EDG ? LDS_PER_WAVE_EDG : LDS_PER_WAVE); /* wave-uniform: m0 */
    const uint64_t wmax = (NV & ~15ull) - 16u; /* the last window fully inside [0, NV) */
    /* single-buffered: 8 KB per wave keeps 20 waves per CU resident to cover the latency */
    auto issue = [&](uint64_t blk) {
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) {
            const uint64_t w = blk + 16u * k;
            const uint64_t ws = w <= wmax ? w : wmax;
            fast::glds16(a.codes + ws, wbase + k * 1024u);
            fast::glds16(a.vb.round + ws, wbase + (4u + k) * 1024u);
            if (EDG) fast::glds16(a.vb.type + ws, wbase + (8u + k) * 1024u);
        }
    };
    uint64_t blk = lo & ~(uint64_t)(BLK - 1u);
    issue(blk);
    for (;;) {
        fast::dma_wait();
        /* the block's four windows out of LDS at once (one wait, not one per window) */
        uint4 cw[4], rw[4], tw[EDG ? 4 : 1];
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) {
            const uint64_t w = blk + 16u * k;
            unsigned char* const cs = wbase + k * 1024u + 16u * lane;
            unsigned char* const rs = wbase + (4u + k) * 1024u + 16u * lane;
            unsigned char* const ts = wbase + (8u + k) * 1024u + 16u * lane;
            if (w < hi && w + 16u > lo && w > wmax) { /* past the batch end: the real bytes */
                tail_fill(a.codes, w, NV, cs);
                tail_fill(a.vb.round, w, NV, rs);
                if (EDG) tail_fill(a.vb.type, w, NV, ts);
            }
            cw[k] = *reinterpret_cast<const uint4*>(cs);
            rw[k] = *reinterpret_cast<const uint4*>(rs);
            if constexpr (EDG) tw[k] = *reinterpret_cast<const uint4*>(ts);
        }
#pragma unroll
        for (uint32_t k = 0; k < 4u; ++k) {
            const uint64_t w = blk + 16u * k;
            if (w >= hi) break;
            if (w + 16u > lo) {
                uint32_t ow[4] = {cw[k].x, cw[k].y, cw[k].z, cw[k].w};
                if (step != AGNES_STEP_COMMIT) { /* (EDG: past the commit the codes stay as they are) */
                    if (SKIP) walk(w, cw[k], rw[k], ow);
                    else walk_ns(w, cw[k], rw[k], ow);
                }
                if constexpr (EDG) edges_win(w, ow, rw[k], tw[k]);
            }
            if (!EDG && step == AGNES_STEP_COMMIT) break;
        }
        const uint64_t nb = blk + BLK;
        if (nb >= hi || (!EDG && step == AGNES_STEP_COMMIT)) break;
        issue(nb); /* this block's LDS reads are consumed: the slot is free */
        blk = nb;
    }
    /* the wave's other lanes may still be streaming: nothing of this lane's in flight */
    fast::dma_wait();
    if (EDG) a.edge_counts[i] = ecnt;

    if (lock_at == NOPOS && valid_at == NOPOS && dec_at == NOPOS && !skipped && step == step0) return;
    /* the State back: round (RoundSkip), locked, valid, decision, step/flags.  Only
     * the starting round can see Polka events: a RoundSkip leaves NewRound, where
     * vote events change nothing but a commit (:196-211) */
    uint32_t d[16] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w, s2.x, s2.y, s2.z, s2.w, s3.x, s3.y, s3.z, s3.w};
    uint32_t flags = s3.y;
    if (skipped) {
        d[2] = eq8; /* the last RoundSkip's round */
        d[3] = 0u;
    }
    /* the three value sources: their votes' values in one round trip, the bucket
     * search only for a nil one */
    uint32_t lv = 0, vv = 0, dv = 0;
    if (lock_at != NOPOS) lv = a.vb.value[lo + lock_at];
    if (valid_at != NOPOS) vv = a.vb.value[lo + valid_at];
    if (dec_at != NOPOS) dv = a.vb.value[lo + dec_at];
    if (lock_at != NOPOS) {
        d[4] = s0.z;
        d[5] = s0.w;
        d[10] = lv != AGNES_NIL ? lv : label_of(a, lo, lo + lock_at);
        flags |= 1u << 8;
    }
    if (valid_at != NOPOS) {
        d[6] = s0.z;
        d[7] = s0.w;
        d[11] = valid_at == lock_at ? d[10] : (vv != AGNES_NIL ? vv : label_of(a, lo, lo + valid_at));
        flags |= 1u << 16;
    }
    if (dec_at != NOPOS) {
        d[8] = dec_round;
        d[9] = 0u;
        d[12] = dv != AGNES_NIL ? dv : label_of(a, lo, lo + dec_at);
        flags |= 1u << 24;
    }
    d[13] = (flags & ~0xFFu) | step;
    sp[0] = make_uint4(d[0], d[1], d[2], d[3]);
    sp[1] = make_uint4(d[4], d[5], d[6], d[7]);
    sp[2] = make_uint4(d[8], d[9], d[10], d[11]);
    sp[3] = make_uint4(d[12], d[13], d[14], d[15]);
}

} // namespace apply
} // namespace agnes

/* ------------------------------------------------------------------ */

bool agnes_apply_codes_supported(const agnes_tally_args* a) {
    /* 16-B windows of the u8 columns */
    return ((reinterpret_cast<uintptr_t>(a->codes) | reinterpret_cast<uintptr_t>(a->vb.round) |
             reinterpret_cast<uintptr_t>(a->vb.type)) & 15u) == 0u &&
           a->vb.n_votes >= 32u && a->states != nullptr && (a->flags & AGNES_FLAG_STATE_MACHINE) != 0;
}

bool agnes_apply_edges_supported(uint32_t max_rounds) { return max_rounds >= 1u && max_rounds <= 8u; }

template <bool SKIP, bool EDG>
static hipError_t launch_apply(const agnes_tally_args* a, uint32_t blocks, hipStream_t st) {
    const size_t lds = (size_t)(EDG ? agnes::apply::LDS_PER_WAVE_EDG : agnes::apply::LDS_PER_WAVE) * agnes::apply::WAVES;
    static thread_local bool attr = false;
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&agnes::apply::apply_codes<SKIP, EDG>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = true;
    }
    hipLaunchKernelGGL((agnes::apply::apply_codes<SKIP, EDG>), dim3(blocks), dim3(256), lds, st, *a);
    return hipGetLastError();
}

hipError_t agnes_launch_apply_codes(const agnes_tally_args* a, hipStream_t st) {
    const uint32_t n = a->vb.n_instances;
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (n + 255u) / 256u;
    const bool skip = (a->flags & AGNES_FLAG_ROUND_SKIP) != 0;
    if (a->edge_counts) {
        if (!a->edge_out || !agnes_apply_edges_supported(a->max_rounds)) return hipErrorInvalidValue;
        return skip ? launch_apply<true, true>(a, blocks, st) : launch_apply<false, true>(a, blocks, st);
    }
    return skip ? launch_apply<true, false>(a, blocks, st) : launch_apply<false, false>(a, blocks, st);
}
