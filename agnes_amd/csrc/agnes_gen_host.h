/*
 * agnes_gen_host.h — host-side helpers over agnes_gen.h (offsets, full host
 * streams, power tables).  Header-only static functions so the engine library
 * and the CPU checker each compile their own copy of the same arithmetic.
 */
#ifndef AGNES_GEN_HOST_H
#define AGNES_GEN_HOST_H

#include <math.h>
#include <stdint.h>

#include "../../include/agnes.h"
#include "agnes_gen.h"

static inline int agnes_gen_params_ok(const agnes_gen_params* p) {
    if (!p || p->n_vals == 0 || p->rounds_min > p->rounds_max || p->rounds_max > 255u) return 0;
    if (p->nil_permille > 1000u || p->absent_permille > 500u) return 0;
    if (p->higher_permille && p->rounds_max + 1u > 255u) return 0;
    if ((uint64_t)p->n_vals * 2u > 0x40000000ull) return 0;
    return 1;
}

static inline agnes_gen_shape agnes_gen_shape_p(const agnes_gen_params* p) {
    return agnes_gen_shape_of(p->n_vals, p->dup_permille, p->equiv_permille, p->higher_permille);
}

static inline uint64_t agnes_gen_host_instance_votes(const agnes_gen_params* p, uint32_t i) {
    agnes_gen_shape s = agnes_gen_shape_p(p);
    const uint32_t gi = p->instance_base + i;
    const uint32_t R = agnes_gen_rounds(p->seed, gi, p->rounds_min, p->rounds_max);
    if (!p->absent_permille) return (uint64_t)R * s.M;
    uint64_t n = 0;
    for (uint32_t r = 0; r < R; ++r) n += agnes_gen_round_votes(p->seed, gi, r, s, p->absent_permille);
    return n;
}

static inline int agnes_gen_host_offsets(const agnes_gen_params* p, uint64_t* offsets) {
    if (!agnes_gen_params_ok(p) || !offsets) return AGNES_E_INVALID;
    uint64_t acc = 0;
    offsets[0] = 0;
    for (uint32_t i = 0; i < p->n_instances; ++i) {
        acc += agnes_gen_host_instance_votes(p, i);
        offsets[i + 1] = acc;
    }
    return AGNES_OK;
}

static inline int agnes_gen_host_votes(const agnes_gen_params* p, const uint64_t* offsets,
                                       uint32_t* instance, uint8_t* round, uint8_t* type,
                                       uint32_t* value, uint32_t* validator) {
    if (!agnes_gen_params_ok(p) || !offsets) return AGNES_E_INVALID;
    agnes_gen_shape s = agnes_gen_shape_p(p);
    for (uint32_t i = 0; i < p->n_instances; ++i) {
        const uint32_t gi = p->instance_base + i;
        for (uint64_t j = offsets[i]; j < offsets[i + 1]; ++j) {
            agnes_gen_vote v =
                agnes_gen_vote_at(p->seed, gi, j - offsets[i], s, p->nil_permille, p->order, p->absent_permille);
            instance[j] = i;
            round[j] = (uint8_t)v.round;
            type[j] = (uint8_t)v.type;
            value[j] = v.value;
            validator[j] = v.validator;
        }
    }
    return AGNES_OK;
}

static inline int agnes_gen_host_power(uint64_t seed, uint32_t n_sets, uint32_t n_vals,
                                       uint32_t kind, int64_t lo, int64_t hi, int64_t* power) {
    if (!power || n_vals == 0 || n_sets == 0) return AGNES_E_INVALID;
    for (uint32_t s = 0; s < n_sets; ++s) {
        const uint64_t key = agnes_hash4(seed, 0x504F574552ull, s, 0);
        for (uint32_t v = 0; v < n_vals; ++v) {
            int64_t w;
            if (kind == AGNES_POWER_EQUAL) {
                w = lo;
            } else if (kind == AGNES_POWER_ZIPF) {
                uint32_t rank = agnes_permute(v, n_vals, key);
                double x = (double)hi / pow((double)rank + 1.0, 1.1);
                w = (int64_t)floor(x);
                if (w < lo) w = lo;
            } else {
                if (hi < lo) return AGNES_E_INVALID;
                uint64_t span = (uint64_t)(hi - lo) + 1u;
                w = lo + (int64_t)(agnes_hash4(seed, 0x554E49ull, s, v) % span);
            }
            power[(uint64_t)s * n_vals + v] = w;
        }
    }
    return AGNES_OK;
}

#endif
