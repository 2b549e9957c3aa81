#define _GNU_SOURCE
/*
 * agnes_oracle.c — scalar CPU restatement of Liamsi/agnes (clean-room, plain C).
 * TEST INFRASTRUCTURE ONLY (see agnes_oracle.h): the checker of the HIP engine
 * and the cpu_baseline of bench.py.  Never linked into the product.
 *
 * i64 arithmetic follows Rust's release build: two's-complement wrapping, done
 * here in uint64_t (signed overflow is undefined in C) and compared signed.
 */
#include "agnes_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "../agnes_amd/csrc/agnes_gen_host.h"

static inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t wmul(int64_t a, int64_t k) { return (int64_t)((uint64_t)a * (uint64_t)k); }

/* is_quorum: `3 * value > 2 * total`, round_votes.rs:31-33 */
int orc_is_quorum(int64_t value, int64_t total) { return wmul(value, 3) > wmul(total, 2); }

/* +1/3 for RoundSkip (state_machine.rs:106 "+1/3 votes from a higher round";
 * no producer in the reference — extension) */
int orc_is_one_third(int64_t value, int64_t total) { return wmul(value, 3) > total; }

/* VoteCount::new, round_votes.rs:36-45 (Value{} label = 0) */
void orc_vc_new(orc_vote_count* c, int64_t total) {
    c->nil = 0;
    c->value_w = 0;
    c->total = total;
    c->value = 0;
    c->pad = 0;
}

/* VoteCount::add_vote, round_votes.rs:48-67 */
uint32_t orc_vc_add(orc_vote_count* c, uint32_t value, int64_t weight, uint32_t* tvalue) {
    if (value != AGNES_NIL) { /* Some(v): :50-54, one value slot, last writer wins */
        c->value_w = wadd(c->value_w, weight);
        c->value = value;
    } else { /* None: :55 */
        c->nil = wadd(c->nil, weight);
    }
    if (orc_is_quorum(c->value_w, c->total)) { /* :58-59 */
        if (tvalue) *tvalue = c->value;
        return AGNES_THRESH_VALUE;
    }
    if (orc_is_quorum(c->nil, c->total)) return AGNES_THRESH_NIL;                /* :60-61 */
    if (orc_is_quorum(wadd(c->value_w, c->nil), c->total)) return AGNES_THRESH_ANY; /* :62-63 */
    return AGNES_THRESH_INIT;                                                     /* :64-65 */
}

/* RoundVotes::new, round_votes.rs:83-90 */
void orc_rv_new(orc_round_votes* rv, int64_t height, int64_t round, int64_t total) {
    rv->height = height;
    rv->round = round;
    orc_vc_new(&rv->prevotes, total);
    orc_vc_new(&rv->precommits, total);
}

/* RoundVotes::add_vote, round_votes.rs:92-97 */
uint32_t orc_rv_add(orc_round_votes* rv, uint32_t typ, uint32_t value, int64_t weight,
                    uint32_t* tvalue) {
    return typ == AGNES_PREVOTE ? orc_vc_add(&rv->prevotes, value, weight, tvalue)
                                : orc_vc_add(&rv->precommits, value, weight, tvalue);
}

/* VoteExecutor::to_event, vote_executor.rs:26-36 */
uint32_t orc_to_event(uint32_t typ, uint32_t thresh) {
    if (thresh == AGNES_THRESH_INIT) return AGNES_EV_NONE; /* :28 */
    if (typ == AGNES_PREVOTE) {
        if (thresh == AGNES_THRESH_ANY) return AGNES_EV_POLKA_ANY; /* :29 */
        if (thresh == AGNES_THRESH_NIL) return AGNES_EV_POLKA_NIL; /* :30 */
        return AGNES_EV_POLKA_VALUE;                               /* :31 */
    }
    if (thresh == AGNES_THRESH_ANY) return AGNES_EV_PRECOMMIT_ANY; /* :32 */
    if (thresh == AGNES_THRESH_NIL) return AGNES_EV_NONE;          /* :33 */
    return AGNES_EV_PRECOMMIT_VALUE;                               /* :34 */
}

/* VoteExecutor::apply, vote_executor.rs:20-23 */
uint32_t orc_ve_apply(orc_round_votes* rv, const agnes_vote* v, int64_t weight, uint32_t* evalue) {
    uint32_t tv = 0;
    uint32_t th = orc_rv_add(rv, v->typ, v->value, weight, &tv);
    if (evalue) *evalue = tv;
    return orc_to_event(v->typ, th);
}

/* ------------------------------------------------------------------------ */
/* State machine, state_machine.rs                                          */

/* State::new, :35-43 */
void orc_state_new(int64_t height, agnes_state* s) {
    memset(s, 0, sizeof(*s));
    s->height = height;
    s->round = 0;
    s->step = AGNES_STEP_NEW_ROUND;
}

/* next_step, :58-66 */
static void next_step(agnes_state* s) {
    if (s->step == AGNES_STEP_NEW_ROUND) s->step = AGNES_STEP_PROPOSE;
    else if (s->step == AGNES_STEP_PROPOSE) s->step = AGNES_STEP_PREVOTE;
    else if (s->step == AGNES_STEP_PREVOTE) s->step = AGNES_STEP_PRECOMMIT;
}

static void set_locked(agnes_state* s, uint32_t v) { /* :78-82 */
    s->locked_present = 1;
    s->locked_round = s->round;
    s->locked_value = v;
}

static void set_valid(agnes_state* s, uint32_t v) { /* :85-89 */
    s->valid_present = 1;
    s->valid_round = s->round;
    s->valid_value = v;
}

static void m_vote(agnes_message* m, uint32_t typ, int64_t round, uint32_t value) {
    m->kind = AGNES_MSG_VOTE;
    m->vote_type = (uint8_t)typ;
    m->round = round;
    m->value = value;
}

static void m_timeout(agnes_message* m, int64_t round, uint32_t step) {
    m->kind = AGNES_MSG_TIMEOUT;
    m->round = round;
    m->timeout_step = (uint8_t)step;
}

/* fn apply, :183-214 — arms tried in order, first match wins */
int orc_state_apply(agnes_state* s, int64_t round, const agnes_event* ev, uint32_t flags,
                    agnes_message* msg) {
    memset(msg, 0, sizeof(*msg));
    const int eqr = s->round == round; /* :184 */
    const uint32_t k = ev->kind;
    const uint32_t v = ev->value;
    switch (s->step) {
    case AGNES_STEP_NEW_ROUND:
        if (k == AGNES_EV_NEW_ROUND_PROPOSER && eqr) { /* :187 propose, :222-229 */
            next_step(s);
            msg->kind = AGNES_MSG_PROPOSAL;
            msg->round = s->round;
            if (s->valid_present) {
                msg->value = s->valid_value;
                msg->pol_round = s->valid_round;
            } else {
                msg->value = v;
                msg->pol_round = -1;
            }
            return 1;
        }
        if (k == AGNES_EV_NEW_ROUND && eqr) { /* :188, :278-281 */
            next_step(s);
            m_timeout(msg, s->round, AGNES_TIMEOUT_PROPOSE);
            return 1;
        }
        break;
    case AGNES_STEP_PROPOSE:
        /* :191 guard eqr && valid_vr (:170-172) */
        if (k == AGNES_EV_PROPOSAL && eqr && ev->pol_round >= -1 && ev->pol_round < s->round) {
            next_step(s); /* prevote, :237-246 */
            uint32_t out;
            if (s->locked_present) {
                int same = (flags & AGNES_FLAG_DISTINCT_VALUES) ? (s->locked_value == v) : 1;
                if (s->locked_round <= ev->pol_round) out = v; /* :240 */
                else if (same) out = v;                        /* :241 (ZST: always) */
                else out = AGNES_NIL;                          /* :242 */
            } else {
                out = v; /* :243 */
            }
            m_vote(msg, AGNES_PREVOTE, s->round, out);
            return 1;
        }
        if ((k == AGNES_EV_PROPOSAL_INVALID || k == AGNES_EV_TIMEOUT_PROPOSE) && eqr) {
            next_step(s); /* :192-193 prevote_nil, :250-253 */
            m_vote(msg, AGNES_PREVOTE, s->round, AGNES_NIL);
            return 1;
        }
        break;
    case AGNES_STEP_PREVOTE:
        if (k == AGNES_EV_POLKA_ANY && eqr) { /* :196, :287-289 */
            m_timeout(msg, s->round, AGNES_TIMEOUT_PREVOTE);
            return 1;
        }
        if ((k == AGNES_EV_POLKA_NIL || k == AGNES_EV_TIMEOUT_PREVOTE) && eqr) {
            next_step(s); /* :197,:199 precommit_nil, :268-271 */
            m_vote(msg, AGNES_PRECOMMIT, s->round, AGNES_NIL);
            return 1;
        }
        if (k == AGNES_EV_POLKA_VALUE && eqr) { /* :198 precommit, :261-264 */
            set_locked(s, v);
            set_valid(s, v);
            next_step(s);
            m_vote(msg, AGNES_PRECOMMIT, s->round, v);
            return 1;
        }
        break;
    case AGNES_STEP_PRECOMMIT:
        if (k == AGNES_EV_POLKA_VALUE && eqr) { /* :202 set_valid_value, :304-306 */
            set_valid(s, v);
            return 0;
        }
        break;
    case AGNES_STEP_COMMIT:
        return 0; /* :205 */
    default:
        return 0;
    }
    /* :208-211, from every step except Commit */
    if (k == AGNES_EV_PRECOMMIT_ANY && eqr) { /* :208, :293-295 */
        m_timeout(msg, s->round, AGNES_TIMEOUT_PRECOMMIT);
        return 1;
    }
    if (k == AGNES_EV_TIMEOUT_PRECOMMIT && eqr) { /* :209 round_skip(s, round + 1) */
        int64_t r = wadd(round, 1);
        s->round = r; /* set_round, :46-52 */
        s->step = AGNES_STEP_NEW_ROUND;
        msg->kind = AGNES_MSG_NEW_ROUND;
        msg->round = r;
        return 1;
    }
    if (k == AGNES_EV_ROUND_SKIP && s->round < round) { /* :210 */
        s->round = round;
        s->step = AGNES_STEP_NEW_ROUND;
        msg->kind = AGNES_MSG_NEW_ROUND;
        msg->round = round;
        return 1;
    }
    if (k == AGNES_EV_PRECOMMIT_VALUE) { /* :211 commit, :320-322 (no round guard) */
        s->step = AGNES_STEP_COMMIT;
        s->decided = 1; /* extension: record the Decision */
        s->decision_round = round;
        s->decision_value = v;
        msg->kind = AGNES_MSG_DECISION;
        msg->round = round;
        msg->value = v;
        return 1;
    }
    return 0; /* :212 */
}

/* ------------------------------------------------------------------------ */
/* batch contract                                                           */

static uint8_t ev_to_code(uint32_t ev) {
    switch (ev) {
    case AGNES_EV_POLKA_ANY: return AGNES_CODE_POLKA_ANY;
    case AGNES_EV_POLKA_NIL: return AGNES_CODE_POLKA_NIL;
    case AGNES_EV_POLKA_VALUE: return AGNES_CODE_POLKA_VALUE;
    case AGNES_EV_PRECOMMIT_ANY: return AGNES_CODE_PRECOMMIT_ANY;
    case AGNES_EV_PRECOMMIT_VALUE: return AGNES_CODE_PRECOMMIT_VALUE;
    default: return AGNES_CODE_NONE;
    }
}

/* message nibble for (RoundSkip message, tally-event message) */
static int vmsg_of(int has1, const agnes_message* m1, int has2, const agnes_message* m2) {
    int b = AGNES_VMSG_NONE;
    if (has2) {
        if (m2->kind == AGNES_MSG_TIMEOUT && m2->timeout_step == AGNES_TIMEOUT_PREVOTE)
            b = AGNES_VMSG_TIMEOUT_PREVOTE;
        else if (m2->kind == AGNES_MSG_TIMEOUT && m2->timeout_step == AGNES_TIMEOUT_PRECOMMIT)
            b = AGNES_VMSG_TIMEOUT_PRECOMMIT;
        else if (m2->kind == AGNES_MSG_VOTE && m2->vote_type == AGNES_PRECOMMIT)
            b = m2->value == AGNES_NIL ? AGNES_VMSG_PRECOMMIT_NIL : AGNES_VMSG_PRECOMMIT_VALUE;
        else if (m2->kind == AGNES_MSG_DECISION)
            b = AGNES_VMSG_DECISION;
        else
            return -1;
    }
    if (has1) {
        if (m1->kind != AGNES_MSG_NEW_ROUND) return -1;
        if (b == AGNES_VMSG_NONE) return AGNES_VMSG_NEW_ROUND;
        if (b == AGNES_VMSG_TIMEOUT_PRECOMMIT) return AGNES_VMSG_NEW_ROUND_TIMEOUT_PRECOMMIT;
        if (b == AGNES_VMSG_DECISION) return AGNES_VMSG_NEW_ROUND_DECISION;
        return -1;
    }
    return b;
}

typedef struct tally_scratch {
    orc_vote_count* cnt;  /* [max_rounds][2] */
    uint32_t* seen_rtv;   /* [max_rounds][2][n_vals] stamp = instance + 1 */
    uint32_t* seen_rv;    /* [max_rounds][n_vals]                          */
    int64_t* skip_w;      /* [max_rounds]                                  */
} tally_scratch;

static int needs_validator(const agnes_config* cfg, const agnes_vote_batch* b) {
    return b->weight == NULL || cfg->mode == AGNES_MODE_DEDUP || (cfg->flags & AGNES_FLAG_ROUND_SKIP);
}

static int tally_range(const agnes_config* cfg, const agnes_vote_batch* b, const orc_power* pw,
                       uint8_t* codes, agnes_state* states, uint32_t i0, uint32_t i1,
                       tally_scratch* sc, uint64_t* n_invalid, uint32_t* labels) {
    const uint32_t R = cfg->max_rounds;
    const uint32_t nv = pw ? pw->n_vals : 0;
    const int dedup = cfg->mode == AGNES_MODE_DEDUP;
    const int skip_on = (cfg->flags & AGNES_FLAG_ROUND_SKIP) != 0;
    const int sm = (cfg->flags & AGNES_FLAG_STATE_MACHINE) != 0;
    const int need_val = needs_validator(cfg, b);
    uint64_t bad = 0;
    for (uint32_t i = i0; i < i1; ++i) {
        const uint32_t set = b->instance_set ? b->instance_set[i] : (pw && pw->n_sets ? i % pw->n_sets : 0);
        const int set_ok = pw && set < pw->n_sets;
        const int64_t total = set_ok ? pw->totals[set] : 0;
        for (uint32_t r = 0; r < 2 * R; ++r) orc_vc_new(&sc->cnt[r], total);
        for (uint32_t r = 0; r < R; ++r) sc->skip_w[r] = 0;
        const uint32_t stamp = i + 1u;
        agnes_state* st = (sm && states) ? &states[i] : NULL;
        for (uint64_t j = b->offsets[i]; j < b->offsets[i + 1]; ++j) {
            const uint32_t r = b->round[j], t = b->type[j], val = b->validator[j];
            const uint32_t value = b->value[j];
            if (labels) labels[j] = AGNES_NIL;
            if (b->instance[j] != i || r >= R || t > 1u || (need_val && (!set_ok || val >= nv)) ||
                (!b->weight && !set_ok)) {
                codes[j] = AGNES_CODE_INVALID;
                ++bad;
                continue;
            }
            const int64_t w = b->weight ? b->weight[j] : pw->power[(uint64_t)set * nv + val];
            if (skip_on) {
                uint32_t* s = &sc->seen_rv[(uint64_t)r * nv + val];
                if (*s != stamp) { /* first vote of (round, validator): counts once */
                    *s = stamp;
                    sc->skip_w[r] = wadd(sc->skip_w[r], w);
                }
            }
            if (dedup) {
                uint32_t* s = &sc->seen_rtv[((uint64_t)r * 2u + t) * nv + val];
                if (*s == stamp) {
                    codes[j] = AGNES_CODE_REJECTED;
                    continue;
                }
                *s = stamp;
            }
            uint32_t tv = 0;
            const uint32_t th = orc_vc_add(&sc->cnt[r * 2u + t], value, w, &tv);
            const uint32_t ev = orc_to_event(t, th);
            if (labels && (ev == AGNES_EV_POLKA_VALUE || ev == AGNES_EV_PRECOMMIT_VALUE)) labels[j] = tv;
            const int skip = skip_on && orc_is_one_third(sc->skip_w[r], total);
            uint8_t code = (uint8_t)(ev_to_code(ev) | (skip ? AGNES_CODE_SKIP : 0u));
            if (st) {
                agnes_message m1, m2;
                int h1 = 0, h2 = 0;
                if (skip) {
                    agnes_event e = {0};
                    e.kind = AGNES_EV_ROUND_SKIP;
                    e.round = r;
                    h1 = orc_state_apply(st, r, &e, cfg->flags, &m1);
                }
                if (ev != AGNES_EV_NONE) {
                    agnes_event e = {0};
                    e.kind = (uint8_t)ev;
                    e.round = r;
                    e.value = tv;
                    h2 = orc_state_apply(st, r, &e, cfg->flags, &m2); /* consensus_executor.rs:68 */
                }
                int vm = vmsg_of(h1, &m1, h2, &m2);
                if (vm < 0) return AGNES_E_INVALID;
                code = (uint8_t)(code | (vm << AGNES_CODE_MSG_SHIFT));
            }
            codes[j] = code;
        }
    }
    *n_invalid += bad;
    return AGNES_OK;
}

static int scratch_alloc(tally_scratch* sc, uint32_t R, uint32_t nv) {
    sc->cnt = (orc_vote_count*)calloc((size_t)R * 2u, sizeof(orc_vote_count));
    sc->seen_rtv = (uint32_t*)calloc((size_t)R * 2u * (nv ? nv : 1), sizeof(uint32_t));
    sc->seen_rv = (uint32_t*)calloc((size_t)R * (nv ? nv : 1), sizeof(uint32_t));
    sc->skip_w = (int64_t*)calloc(R, sizeof(int64_t));
    return sc->cnt && sc->seen_rtv && sc->seen_rv && sc->skip_w;
}

static void scratch_free(tally_scratch* sc) {
    free(sc->cnt);
    free(sc->seen_rtv);
    free(sc->seen_rv);
    free(sc->skip_w);
}

static int check_args(const agnes_config* cfg, const agnes_vote_batch* b, const uint8_t* codes) {
    if (!cfg || !b || !codes || !b->offsets) return 0;
    if (cfg->max_rounds == 0 || cfg->max_rounds > 256u) return 0;
    if (cfg->mode > AGNES_MODE_DEDUP) return 0;
    if (b->n_votes && (!b->instance || !b->round || !b->type || !b->value || !b->validator)) return 0;
    return 1;
}

int orc_tally(const agnes_config* cfg, const agnes_vote_batch* b, const orc_power* pw,
              uint8_t* codes, agnes_state* states, uint64_t* n_invalid) {
    if (!check_args(cfg, b, codes)) return AGNES_E_INVALID;
    tally_scratch sc;
    if (!scratch_alloc(&sc, cfg->max_rounds, pw ? pw->n_vals : 0)) {
        scratch_free(&sc);
        return AGNES_E_NOMEM;
    }
    uint64_t bad = 0;
    int rc = tally_range(cfg, b, pw, codes, states, 0, b->n_instances, &sc, &bad, NULL);
    scratch_free(&sc);
    if (n_invalid) *n_invalid = bad;
    return rc;
}

typedef struct mt_job {
    const agnes_config* cfg;
    const agnes_vote_batch* b;
    const orc_power* pw;
    uint8_t* codes;
    agnes_state* states;
    uint32_t* labels;
    uint32_t i0, i1;
    uint64_t bad;
    int rc;
} mt_job;

static void* mt_run(void* arg) {
    mt_job* j = (mt_job*)arg;
    tally_scratch sc;
    j->bad = 0;
    if (!scratch_alloc(&sc, j->cfg->max_rounds, j->pw ? j->pw->n_vals : 0)) {
        j->rc = AGNES_E_NOMEM;
    } else {
        j->rc = tally_range(j->cfg, j->b, j->pw, j->codes, j->states, j->i0, j->i1, &sc, &j->bad, j->labels);
    }
    scratch_free(&sc);
    return NULL;
}

int orc_tally_mt(const agnes_config* cfg, const agnes_vote_batch* b, const orc_power* pw,
                 uint8_t* codes, agnes_state* states, uint64_t* n_invalid, int threads) {
    return orc_tally_labels(cfg, b, pw, codes, states, n_invalid, NULL, threads);
}

int orc_tally_labels(const agnes_config* cfg, const agnes_vote_batch* b, const orc_power* pw,
                     uint8_t* codes, agnes_state* states, uint64_t* n_invalid, uint32_t* labels,
                     int threads) {
    if (!check_args(cfg, b, codes)) return AGNES_E_INVALID;
    if (threads < 1) threads = 1;
    if ((uint32_t)threads > b->n_instances) threads = b->n_instances ? (int)b->n_instances : 1;
    mt_job* jobs = (mt_job*)calloc((size_t)threads, sizeof(mt_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !th) {
        free(jobs);
        free(th);
        return AGNES_E_NOMEM;
    }
    /* contiguous instance ranges with ~equal vote counts (rayon-style split) */
    const uint64_t nvotes = b->offsets[b->n_instances];
    uint32_t cur = 0;
    for (int t = 0; t < threads; ++t) {
        uint64_t target = nvotes * (uint64_t)(t + 1) / (uint64_t)threads;
        uint32_t end = cur;
        while (end < b->n_instances && b->offsets[end] < target) ++end;
        if (t == threads - 1) end = b->n_instances;
        jobs[t] = (mt_job){cfg, b, pw, codes, states, labels, cur, end, 0, AGNES_OK};
        cur = end;
    }
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, mt_run, &jobs[t]);
    uint64_t bad = 0;
    int rc = AGNES_OK;
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        bad += jobs[t].bad;
        if (jobs[t].rc != AGNES_OK) rc = jobs[t].rc;
    }
    free(jobs);
    free(th);
    if (n_invalid) *n_invalid = bad;
    return rc;
}

int orc_apply_events(agnes_state* states, uint32_t n, const uint64_t* off, const agnes_event* ev,
                     agnes_message* msgs, uint32_t flags) {
    if (!states || !off || (off[n] && (!ev || !msgs))) return AGNES_E_INVALID;
    for (uint32_t i = 0; i < n; ++i)
        for (uint64_t k = off[i]; k < off[i + 1]; ++k)
            orc_state_apply(&states[i], ev[k].round, &ev[k], flags, &msgs[k]);
    return AGNES_OK;
}

/* ConsensusExecutor::apply_msg over per-instance message streams
 * (consensus_executor.rs:54-86; include/agnes.h agnes_apply_msgs).  One
 * ConsensusExecutor per instance: a VoteCount per (round, type) (the HeightVotes
 * the reference leaves as a stub, :5) and the State.  Message kinds:
 *   VOTE      :61-69  VoteExecutor::apply (the batch validation and weight of
 *                     orc_tally), then apply_event(v.round, event)
 *   PROPOSAL  :56-60  Event::Proposal(pol_round, value) at p.round
 *   TIMEOUT   :70-77  TimeoutPropose / Prevote / Precommit at t.round
 *   NEW_ROUND         Event::NewRound / NewRoundProposer(value) at round (the
 *                     executor's own NewRound, execute :31-33) */
int orc_apply_msgs(const agnes_config* cfg, const agnes_vote_batch* b, const orc_power* pw, const uint8_t* kinds,
                   const int32_t* pol, uint8_t* codes, agnes_state* states, agnes_message* msgs,
                   uint64_t* n_invalid) {
    if (!cfg || !b || !states || !b->offsets || cfg->max_rounds == 0 || cfg->max_rounds > 256u) return AGNES_E_INVALID;
    if (b->n_votes && (!kinds || !codes || !msgs || !b->instance || !b->round || !b->type || !b->value ||
                       (!b->weight && !b->validator)))
        return AGNES_E_INVALID;
    const uint32_t R = cfg->max_rounds, nv = pw ? pw->n_vals : 0;
    orc_vote_count* cnt = (orc_vote_count*)calloc((size_t)2u * R, sizeof(orc_vote_count));
    if (!cnt) return AGNES_E_NOMEM;
    uint64_t bad = 0;
    for (uint32_t i = 0; i < b->n_instances; ++i) {
        const uint32_t set = b->instance_set ? b->instance_set[i] : (pw && pw->n_sets ? i % pw->n_sets : 0);
        const int set_ok = pw && set < pw->n_sets;
        const int64_t total = set_ok ? pw->totals[set] : 0;
        for (uint32_t k = 0; k < 2u * R; ++k) orc_vc_new(&cnt[k], total);
        for (uint64_t j = b->offsets[i]; j < b->offsets[i + 1]; ++j) {
            const uint32_t r = b->round[j], t = b->type[j], v = b->value[j];
            agnes_event e;
            memset(&e, 0, sizeof(e));
            e.kind = AGNES_EV_NONE;
            e.round = r;
            codes[j] = AGNES_CODE_NONE;
            if (kinds[j] == AGNES_IN_VOTE) {
                if (b->instance[j] != i || r >= R || t > 1u || (!b->weight && (!set_ok || b->validator[j] >= nv))) {
                    codes[j] = AGNES_CODE_INVALID;
                    ++bad;
                } else {
                    const int64_t w = b->weight ? b->weight[j] : pw->power[(uint64_t)set * nv + b->validator[j]];
                    uint32_t tv = 0;
                    const uint32_t ev = orc_to_event(t, orc_vc_add(&cnt[r * 2u + t], v, w, &tv));
                    codes[j] = ev_to_code(ev);
                    e.kind = (uint8_t)ev;
                    e.value = tv;
                }
            } else if (kinds[j] == AGNES_IN_PROPOSAL) {
                e.kind = AGNES_EV_PROPOSAL;
                e.value = v;
                e.pol_round = pol ? pol[j] : -1;
            } else if (kinds[j] == AGNES_IN_TIMEOUT && t <= AGNES_TIMEOUT_PRECOMMIT) {
                e.kind = (uint8_t)(t == AGNES_TIMEOUT_PROPOSE   ? AGNES_EV_TIMEOUT_PROPOSE
                                   : t == AGNES_TIMEOUT_PREVOTE ? AGNES_EV_TIMEOUT_PREVOTE
                                                                : AGNES_EV_TIMEOUT_PRECOMMIT);
            } else if (kinds[j] == AGNES_IN_NEW_ROUND) {
                e.kind = (uint8_t)(v != AGNES_NIL ? AGNES_EV_NEW_ROUND_PROPOSER : AGNES_EV_NEW_ROUND);
                e.value = v;
            } else {
                codes[j] = AGNES_CODE_INVALID;
                ++bad;
            }
            if (e.kind != AGNES_EV_NONE) orc_state_apply(&states[i], r, &e, cfg->flags, &msgs[j]);
            else memset(&msgs[j], 0, sizeof(msgs[j]));
        }
    }
    free(cnt);
    if (n_invalid) *n_invalid = bad;
    return AGNES_OK;
}

/* ValidatorSet::new (validators.rs:28-31) with sort + dedup (:49-55), the
 * intended behaviour (the file does not compile): per set, validators sorted by
 * address (Validator::address = public key, :15-17), equal addresses by power then
 * input index (one of the orders sort_unstable_by allows, made deterministic),
 * exact duplicates (address and power, a derived PartialEq) dropped keeping the
 * first; totals = the wrapping sum (vote_executor.rs:13's total_weight).  Same
 * contract as agnes_valset_build (include/agnes.h), host pointers. */
typedef struct vs_ctx {
    const uint8_t* addr;
    const int64_t* power;
    const uint32_t* set_of;
    uint32_t addr_len;
} vs_ctx;

static int vs_cmp3(const vs_ctx* k, uint32_t i, uint32_t j) {
    const uint32_t si = k->set_of ? k->set_of[i] : 0u, sj = k->set_of ? k->set_of[j] : 0u;
    if (si != sj) return si < sj ? -1 : 1;
    const int c = memcmp(k->addr + (size_t)i * k->addr_len, k->addr + (size_t)j * k->addr_len, k->addr_len);
    if (c) return c < 0 ? -1 : 1;
    if (k->power[i] != k->power[j]) return k->power[i] < k->power[j] ? -1 : 1;
    return 0;
}

static int vs_qcmp(const void* a, const void* b, void* arg) {
    const uint32_t i = *(const uint32_t*)a, j = *(const uint32_t*)b;
    const int c = vs_cmp3((const vs_ctx*)arg, i, j);
    return c ? c : (i < j ? -1 : (i > j ? 1 : 0));
}

int orc_valset_build(const uint8_t* addr, uint32_t addr_len, const int64_t* power, const uint32_t* set_of,
                     uint64_t n, uint32_t n_sets, uint32_t* order, uint64_t* set_offsets, int64_t* power_out,
                     int64_t* totals, uint64_t* n_out) {
    if (!n_out || !set_offsets || !totals || n_sets == 0 || addr_len == 0 || (n && (!addr || !power || !order)))
        return AGNES_E_INVALID;
    uint32_t* idx = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    if (!idx) return AGNES_E_NOMEM;
    for (uint64_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
    vs_ctx k = {addr, power, set_of, addr_len};
    qsort_r(idx, n, sizeof(uint32_t), vs_qcmp, &k);
    uint64_t m = 0;
    for (uint64_t t = 0; t < n; ++t) {
        const uint32_t a = idx[t];
        if ((set_of ? set_of[a] : 0u) >= n_sets) continue;
        if (t > 0 && vs_cmp3(&k, idx[t - 1], a) == 0) continue; /* Vec::dedup */
        order[m] = a;
        if (power_out) power_out[m] = power[a];
        ++m;
    }
    uint64_t o = 0;
    for (uint32_t s = 0; s <= n_sets; ++s) {
        while (o < m && (set_of ? set_of[order[o]] : 0u) < s) ++o;
        set_offsets[s] = s == n_sets ? m : o;
    }
    for (uint32_t s = 0; s < n_sets; ++s) {
        int64_t t = 0;
        for (uint64_t q = set_offsets[s]; q < set_offsets[s + 1]; ++q) t = wadd(t, power[order[q]]);
        totals[s] = t;
    }
    free(idx);
    *n_out = m;
    return AGNES_OK;
}

/* Edge-triggered summary (include/agnes.h agnes_edge).  The
 * per-vote codes are VoteExecutor::apply's level-triggered Option<Event>
 * (vote_executor.rs:20-36) for the vote's (round, type) executor — the
 * reference's HeightVotes stub (consensus_executor.rs:5, vote_executor.rs:9,14) —
 * and the message State::apply produced for it (state_machine.rs:196-211, whose
 * Timeout arms repeat too).  An executor starts at level 0 with no message
 * (VoteCount::new, round_votes.rs:36-45); a valid vote is an edge when its level
 * (code bits 0..3) differs from the level its executor's previous valid vote
 * left, or when it carries a message (bits 4..7) other than the executor's last.
 * offsets[n+1] always written; out (NULL: count only) gets the records. */
int orc_edges(const agnes_config* cfg, const agnes_vote_batch* b, const uint8_t* codes,
              uint64_t* offsets, agnes_edge* out) {
    if (!cfg || !b || !offsets || cfg->max_rounds < 1 || cfg->max_rounds > 256) return AGNES_E_INVALID;
    const uint32_t keys = 2u * cfg->max_rounds;
    uint8_t level[512];
    uint64_t k = 0;
    offsets[0] = 0;
    for (uint32_t i = 0; i < b->n_instances; ++i) {
        memset(level, 0, sizeof level);
        uint64_t lo = b->offsets[i], hi = b->offsets[i + 1];
        if (lo > b->n_votes) lo = b->n_votes;
        if (hi > b->n_votes) hi = b->n_votes;
        for (uint64_t j = lo; j < hi; ++j) {
            const uint32_t c = codes[j], ev = c & AGNES_CODE_EVENT_MASK;
            const uint32_t r = b->round[j], t = b->type[j], key = r * 2u + t;
            if (ev == AGNES_CODE_INVALID || ev == AGNES_CODE_REJECTED || t > 1u || key >= keys) continue;
            const uint32_t prev = level[key], msg = c >> AGNES_CODE_MSG_SHIFT;
            const uint32_t nl = (c & 0xFu) | (msg ? (msg << AGNES_CODE_MSG_SHIFT) : (prev & 0xF0u));
            if (prev != nl) {
                if (out) {
                    agnes_edge* e = &out[k];
                    e->vote = j;
                    e->instance = i;
                    e->round = (uint8_t)r;
                    e->type = (uint8_t)t;
                    e->code = (uint8_t)c;
                    e->prev = (uint8_t)prev;
                }
                ++k;
            }
            level[key] = (uint8_t)nl;
        }
        offsets[i + 1] = k;
    }
    return AGNES_OK;
}

/* The event stream (include/agnes.h agnes_vote_event): per instance, in vote
 * order, the Some(Event)s of ConsensusExecutor::apply_vote (consensus_executor.rs:
 * 61-69): a RoundSkip first when the vote completed +1/3 of a higher round (the
 * extension's event, code bit AGNES_CODE_SKIP), then the VoteExecutor event
 * (vote_executor.rs:20-36, code bits 0..2), whose Value is the one the tally's
 * VoteCount gave it (labels, orc_tally_labels).  offsets[n+1] always written; out
 * (NULL: count only) gets the records. */
int orc_events(const agnes_config* cfg, const agnes_vote_batch* b, const uint8_t* codes,
               const uint32_t* labels, uint64_t* offsets, agnes_vote_event* out) {
    static const uint8_t kind_of[8] = {AGNES_EV_NONE, AGNES_EV_POLKA_ANY, AGNES_EV_POLKA_NIL,
                                       AGNES_EV_POLKA_VALUE, AGNES_EV_PRECOMMIT_ANY,
                                       AGNES_EV_PRECOMMIT_VALUE, AGNES_EV_NONE, AGNES_EV_NONE};
    if (!cfg || !b || !offsets || (out && !labels)) return AGNES_E_INVALID;
    uint64_t k = 0;
    offsets[0] = 0;
    for (uint32_t i = 0; i < b->n_instances; ++i) {
        uint64_t lo = b->offsets[i], hi = b->offsets[i + 1];
        if (lo > b->n_votes) lo = b->n_votes;
        if (hi > b->n_votes) hi = b->n_votes;
        for (uint64_t j = lo; j < hi; ++j) {
            const uint32_t c = codes[j], ev = c & AGNES_CODE_EVENT_MASK;
            if (ev == AGNES_CODE_INVALID || ev == AGNES_CODE_REJECTED) continue;
            for (int pass = 0; pass < 2; ++pass) {
                const uint32_t kind = pass == 0 ? ((c & AGNES_CODE_SKIP) ? AGNES_EV_ROUND_SKIP : AGNES_EV_NONE)
                                                : kind_of[ev];
                if (kind == AGNES_EV_NONE) continue;
                if (out) {
                    agnes_vote_event* e = &out[k];
                    memset(e, 0, sizeof(*e));
                    e->vote = j;
                    e->instance = i;
                    e->value = (kind == AGNES_EV_POLKA_VALUE || kind == AGNES_EV_PRECOMMIT_VALUE) ? labels[j]
                                                                                              : AGNES_NIL;
                    e->round = b->round[j];
                    e->kind = (uint8_t)kind;
                    e->message = (uint8_t)(c >> AGNES_CODE_MSG_SHIFT);
                }
                ++k;
            }
        }
        offsets[i + 1] = k;
    }
    return AGNES_OK;
}

void orc_set_totals(const int64_t* power, uint32_t n_sets, uint32_t n_vals, int64_t* totals) {
    for (uint32_t s = 0; s < n_sets; ++s) {
        int64_t t = 0;
        for (uint32_t v = 0; v < n_vals; ++v) t = wadd(t, power[(uint64_t)s * n_vals + v]);
        totals[s] = t;
    }
}

uint64_t orc_gen_instance_votes(const agnes_gen_params* p, uint32_t i) {
    return agnes_gen_host_instance_votes(p, i);
}
int orc_gen_offsets(const agnes_gen_params* p, uint64_t* offsets) {
    return agnes_gen_host_offsets(p, offsets);
}
int orc_gen_votes(const agnes_gen_params* p, const uint64_t* offsets, uint32_t* instance,
                  uint8_t* round, uint8_t* type, uint32_t* value, uint32_t* validator) {
    return agnes_gen_host_votes(p, offsets, instance, round, type, value, validator);
}
int orc_gen_power(uint64_t seed, uint32_t n_sets, uint32_t n_vals, uint32_t kind, int64_t lo,
                  int64_t hi, int64_t* power) {
    return agnes_gen_host_power(seed, n_sets, n_vals, kind, lo, hi, power);
}
