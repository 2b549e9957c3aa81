/*
 * agnes_gen.h — counter-based synthetic vote streams (splitmix64), identical on
 * the host (gcc, oracle tests) and on the device (hipcc, agnes_gen_votes_device).
 *
 * Every field of every vote is a pure function of (params, instance, position),
 * so a stream never has to be stored to be reproduced, shards generate the same
 * votes as one big batch would (global ids come from instance_base), and the CPU
 * checker can rebuild any vote without a device round trip.
 *
 * Shape of instance i (global id gi = instance_base + i):
 *   R_i rounds ~ U[rounds_min, rounds_max]; round r holds M = 2n + D + E + H votes:
 *     [0, 2n)        base votes: vote b -> type b / n, validator b % n,
 *                    nil with probability nil_permille, else the round's proposal
 *     [2n, 2n+D)     exact duplicates of a hashed base vote        (C4: duplicates)
 *     [.., +E)       equivocations: same (type, validator), other value (C4)
 *     [.., +H)       early votes tagged round r+1                     (C4: RoundSkip)
 *   positions inside the round permuted by a keyed Feistel bijection (order SHUFFLED),
 *   or prevotes-then-precommits (PHASED), or identity (SORTED).
 *   Abstention (absent_permille > 0): round r of instance gi keeps only its first M_r =
 *   M - A_r positions, A_r ~ U[0, 2 M absent / 1000] hashed from (gi, r) -- with the
 *   SHUFFLED order a uniformly random subset of its votes is absent -- so instance
 *   lengths (and the offsets of a batch) take any value, not multiples of the round.
 * Not part of the tally hot path.
 */
#ifndef AGNES_GEN_H
#define AGNES_GEN_H

#include <stdint.h>

#if defined(__HIPCC__)
#define AGNES_HD __host__ __device__
#else
#define AGNES_HD
#endif

#ifndef AGNES_NIL
#define AGNES_NIL 0xFFFFFFFFu
#endif

typedef struct agnes_gen_shape {
    uint32_t n;   /* validators                  */
    uint32_t n2;  /* base votes per round = 2n    */
    uint32_t D;   /* duplicates per round         */
    uint32_t E;   /* equivocations per round      */
    uint32_t H;   /* higher-round votes per round */
    uint32_t M;   /* votes per round              */
} agnes_gen_shape;

AGNES_HD static inline uint64_t agnes_mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

AGNES_HD static inline uint64_t agnes_hash4(uint64_t seed, uint64_t a, uint64_t b, uint64_t c) {
    uint64_t h = agnes_mix64(seed ^ 0xA6E5A6E5A6E5A6E5ull);
    h = agnes_mix64(h ^ a);
    h = agnes_mix64(h ^ (b + 0x632BE59BD9B4E019ull));
    return agnes_mix64(h ^ (c + 0x8CB92BA72F3D8DD7ull));
}

AGNES_HD static inline agnes_gen_shape agnes_gen_shape_of(uint32_t n_vals, uint32_t dup_pm,
                                                         uint32_t equiv_pm, uint32_t higher_pm) {
    agnes_gen_shape s;
    s.n = n_vals;
    s.n2 = 2u * n_vals;
    s.D = (uint32_t)(((uint64_t)s.n2 * dup_pm) / 1000u);
    s.E = (uint32_t)(((uint64_t)s.n2 * equiv_pm) / 1000u);
    s.H = (uint32_t)(((uint64_t)s.n2 * higher_pm) / 1000u);
    s.M = s.n2 + s.D + s.E + s.H;
    return s;
}

AGNES_HD static inline uint32_t agnes_gen_rounds(uint64_t seed, uint32_t gi, uint32_t rmin,
                                                 uint32_t rmax) {
    uint32_t span = rmax - rmin + 1u;
    return rmin + (uint32_t)(agnes_hash4(seed, 0x524F554E44ull, gi, 0) % span);
}

/* proposal value of (instance, round): never AGNES_NIL, bit 0 free for equivocation */
AGNES_HD static inline uint32_t agnes_gen_proposal(uint64_t seed, uint32_t gi, uint32_t r) {
    return (uint32_t)(agnes_hash4(seed, 0x50524F50ull, gi, r) & 0x7FFFFFFEull);
}

/* keyed Feistel bijection on [0, dom) by cycle walking over [0, 2^k) */
AGNES_HD static inline uint32_t agnes_permute(uint32_t x, uint32_t dom, uint64_t key) {
    if (dom <= 1u) return 0u;
    uint32_t k = 0;
    while ((1u << k) < dom) ++k;
    if (k & 1u) ++k;
    if (k < 2u) k = 2u;
    const uint32_t half = k >> 1;
    const uint32_t mask = (1u << half) - 1u;
    do {
        uint32_t L = x >> half, R = x & mask;
        for (uint32_t rnd = 0; rnd < 4u; ++rnd) {
            uint32_t nl = R;
            R = L ^ (uint32_t)(agnes_mix64(key ^ ((uint64_t)rnd << 32) ^ R) & mask);
            L = nl;
        }
        x = (L << half) | R;
    } while (x >= dom);
    return x;
}

typedef struct agnes_gen_vote {
    uint32_t round;
    uint32_t type;
    uint32_t value;
    uint32_t validator;
} agnes_gen_vote;

/* base vote b of (gi, r) */
AGNES_HD static inline agnes_gen_vote agnes_gen_base(uint64_t seed, uint32_t gi, uint32_t r,
                                                     uint32_t b, uint32_t n, uint32_t nil_pm) {
    agnes_gen_vote v;
    v.round = r;
    v.type = b / n;
    v.validator = b % n;
    int nil = (agnes_hash4(seed, 0x4E494Cull ^ ((uint64_t)r << 40), gi, b) % 1000u) < nil_pm;
    v.value = nil ? AGNES_NIL : agnes_gen_proposal(seed, gi, r);
    return v;
}

/* votes of round r of instance gi: M less its absent ones (see the header) */
AGNES_HD static inline uint32_t agnes_gen_round_votes(uint64_t seed, uint32_t gi, uint32_t r, agnes_gen_shape s,
                                                      uint32_t absent_pm) {
    if (!absent_pm) return s.M;
    const uint64_t span = ((uint64_t)s.M * absent_pm * 2u) / 1000u;
    const uint64_t A = agnes_hash4(seed, 0x414253454E54ull, gi, r) % (span + 1u);
    return A < s.M ? s.M - (uint32_t)A : 0u;
}

/* vote at position t (0-based) of instance gi */
AGNES_HD static inline agnes_gen_vote agnes_gen_vote_at(uint64_t seed, uint32_t gi, uint64_t t,
                                                        agnes_gen_shape s, uint32_t nil_pm,
                                                        uint32_t order, uint32_t absent_pm) {
    uint32_t r, pos;
    if (!absent_pm) {
        r = (uint32_t)(t / s.M);
        pos = (uint32_t)(t % s.M);
    } else { /* the round holding position t (the instance's rounds are few) */
        r = 0;
        for (uint32_t mr = agnes_gen_round_votes(seed, gi, 0u, s, absent_pm); t >= mr;
             mr = agnes_gen_round_votes(seed, gi, ++r, s, absent_pm))
            t -= mr;
        pos = (uint32_t)t;
    }
    const uint64_t key = agnes_hash4(seed, 0x5045524Dull, gi, r);
    uint32_t q;
    if (order == 2u) {
        q = pos;
    } else if (order == 1u) {
        if (pos < s.n) q = agnes_permute(pos, s.n, key);
        else if (pos < s.n2) q = s.n + agnes_permute(pos - s.n, s.n, key ^ 0x1111ull);
        else q = s.n2 + agnes_permute(pos - s.n2, s.M - s.n2, key ^ 0x2222ull);
    } else {
        q = agnes_permute(pos, s.M, key);
    }
    if (q < s.n2) return agnes_gen_base(seed, gi, r, q, s.n, nil_pm);
    const uint64_t h = agnes_hash4(seed, 0x455854ull ^ ((uint64_t)r << 40), gi, q);
    if (q < s.n2 + s.D) { /* exact duplicate */
        return agnes_gen_base(seed, gi, r, (uint32_t)(h % s.n2), s.n, nil_pm);
    }
    if (q < s.n2 + s.D + s.E) { /* equivocation: same (type, validator), another value */
        agnes_gen_vote v = agnes_gen_base(seed, gi, r, (uint32_t)(h % s.n2), s.n, nil_pm);
        const uint32_t prop = agnes_gen_proposal(seed, gi, r);
        if (v.value == AGNES_NIL) v.value = prop;
        else v.value = ((h >> 32) & 1u) ? AGNES_NIL : (prop ^ 1u);
        return v;
    }
    /* early vote from round r+1 */
    agnes_gen_vote v;
    v.round = r + 1u;
    v.type = (uint32_t)((h >> 32) & 1u);
    v.validator = (uint32_t)(h % s.n);
    v.value = agnes_gen_proposal(seed, gi, r + 1u);
    return v;
}

#endif /* AGNES_GEN_H */
