/*
 * agnes_api.cpp — host side of the C ABI declared in include/agnes.h.
 *
 * Owns device residency (power tables, per-set quorum constants, error
 * counters) and enqueues the gfx950 kernels of agnes_kernels.hip.  Every
 * compute entry point — including the scalar mirrors of VoteExecutor::apply
 * and State::apply — runs on the GPU; without a visible device they return
 * AGNES_E_NODEVICE.  Nothing here throws across the boundary.
 */
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/agnes.h"
#include "agnes_gen_host.h"
#include "agnes_internal.h"

struct agnes_ctx {
    int device = 0;
    int num_cus = 256;
    int64_t* d_power = nullptr;
    uint32_t* d_power32 = nullptr;
    agnes_set_info* d_sets = nullptr;
    uint32_t n_sets = 0;
    uint32_t n_vals = 0;
    unsigned long long* d_err = nullptr; /* the invalid-vote count's stripes, then AGNES_QUEUE_WORDS
                                            work-queue counters (agnes_internal.h): one memset per call */
    hipStream_t last_stream = nullptr;
    bool used = false;               /* a call has enqueued work on last_stream */
    hipEvent_t order_ev = nullptr;   /* orders a call on another stream after it */
    uint32_t sets_dom = 0;     /* 2: every set inside the u32 fast domain, 1: inside the u64 one, 0: neither */
    uint32_t* d_list = nullptr; /* [list_cap] deferred instances, [list_cap] walk list */
    uint32_t list_cap = 0;
    uint64_t* d_scan = nullptr; /* edge-offset scan: block totals */
    uint64_t scan_cap = 0;
    void* d_dd = nullptr;       /* agnes_dedup_first: bucket counts, scan scratch, (key, index) pairs */
    uint64_t dd_cap = 0;
    int32_t* d_edtab = nullptr; /* Ed25519 fixed-base table (agnes_wire_ingest), built on first use */
    unsigned long long* d_ovf = nullptr; /* records the dense writers dropped since agnes_records_overflow */
};

namespace {

int status_of(hipError_t e) {
    if (e == hipSuccess) return AGNES_OK;
    if (e == hipErrorOutOfMemory) return AGNES_E_NOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return AGNES_E_NODEVICE;
    return AGNES_E_DEVICE;
}

#define AGNES_TRY(expr)                              \
    do {                                             \
        hipError_t e_ = (expr);                      \
        if (e_ != hipSuccess) return status_of(e_);  \
    } while (0)

/* The ctx scratch (queue counters, deferred / walk lists, the invalid counter, the
 * edge-scan scratch) is shared by every call: a call on a different stream than
 * the previous one waits for that stream's work first (one event), so calls on
 * one ctx never overlap (include/agnes.h, agnes_ctx). */
int order_stream(agnes_ctx* c, hipStream_t st) {
    if (c->used && c->last_stream != st) {
        if (!c->order_ev) AGNES_TRY(hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming));
        AGNES_TRY(hipEventRecord(c->order_ev, c->last_stream));
        AGNES_TRY(hipStreamWaitEvent(st, c->order_ev, 0));
    }
    c->last_stream = st;
    c->used = true;
    return AGNES_OK;
}

#define AGNES_ORDER(c, st)                          \
    do {                                            \
        const int o_ = order_stream((c), (st));     \
        if (o_ != AGNES_OK) return o_;              \
    } while (0)

void free_power(agnes_ctx* c) {
    if (c->d_power) (void)hipFree(c->d_power);
    if (c->d_power32) (void)hipFree(c->d_power32);
    if (c->d_sets) (void)hipFree(c->d_sets);
    c->d_power = nullptr;
    c->d_power32 = nullptr;
    c->d_sets = nullptr;
    c->n_sets = c->n_vals = 0;
}

int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

/* quorum constants of one set (see agnes_internal.h) */
agnes_set_info set_info(const int64_t* pw, uint32_t n_vals, int64_t total) {
    agnes_set_info si{};
    si.total = total;
    int64_t mn = 0, mx = 0;
    for (uint32_t v = 0; v < n_vals; ++v) {
        mn = v == 0 || pw[v] < mn ? pw[v] : mn;
        mx = v == 0 || pw[v] > mx ? pw[v] : mx;
    }
    const bool fast = mn >= 0 && mx < (1ll << 31) && total >= 0 && total <= INT64_MAX / 2;
    si.fast = fast ? 1u : 0u;
    if (fast) {
        const uint64_t t2 = (uint64_t)(2 * total) / 3u, t1 = (uint64_t)total / 3u;
        si.q2 = t2 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)t2;
        si.q1 = t1 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)t1;
        si.maxpow = (uint32_t)mx;
    }
    const bool w64 = mn >= 0 && total >= 0 && total < (1ll << 61);
    si.w64 = w64 ? 1u : 0u;
    if (w64) {
        si.q2w = (uint64_t)(2 * total) / 3u;
        si.q1w = (uint64_t)total / 3u;
        si.maxw = (uint64_t)mx;
    }
    return si;
}

bool cfg_ok(const agnes_config* cfg) {
    return cfg && cfg->max_rounds >= 1 && cfg->max_rounds <= 256 && cfg->mode <= AGNES_MODE_DEDUP &&
           (cfg->flags & ~(AGNES_FLAG_ROUND_SKIP | AGNES_FLAG_STATE_MACHINE | AGNES_FLAG_DISTINCT_VALUES |
                           AGNES_FLAG_ONE_INSTANCE | AGNES_FLAG_WEIGHTS_CACHED | AGNES_FLAG_MASKED_REJECTED |
                           (AGNES_ROUTE_MASK << AGNES_ROUTE_SHIFT) |
                           AGNES_FLAG_EPOCH_BITS(0x1F))) == 0;
}

/* ---- scalar mirror: one process-wide context ---- */
std::mutex g_mu;
agnes_ctx* g_ctx = nullptr;

int scalar_ctx(agnes_ctx** out) {
    if (!g_ctx) {
        const char* d = std::getenv("AGNES_DEVICE");
        int rc = agnes_ctx_create(d ? std::atoi(d) : 0, &g_ctx);
        if (rc != AGNES_OK) {
            g_ctx = nullptr;
            return rc;
        }
    }
    *out = g_ctx;
    return AGNES_OK;
}

} // namespace

extern "C" {

namespace {
struct KtRec {
    const char* name;
    hipEvent_t b, e;
};
bool kt_on = false;
std::vector<KtRec> kt_recs;
size_t kt_used = 0;
std::mutex kt_mu;
} // namespace

void agnes_kt_mark(const char* name, hipStream_t st, bool begin) {
    if (!kt_on) return;
    std::lock_guard<std::mutex> g(kt_mu);
    if (begin) {
        if (kt_used == kt_recs.size()) {
            KtRec r{name, nullptr, nullptr};
            if (hipEventCreate(&r.b) != hipSuccess || hipEventCreate(&r.e) != hipSuccess) return;
            kt_recs.push_back(r);
        }
        kt_recs[kt_used].name = name;
        (void)hipEventRecord(kt_recs[kt_used].b, st);
    } else if (kt_used < kt_recs.size()) {
        (void)hipEventRecord(kt_recs[kt_used].e, st);
        ++kt_used;
    }
}

int agnes_kernel_timing(int enable) {
    std::lock_guard<std::mutex> g(kt_mu);
    kt_on = enable != 0;
    kt_used = 0;
    return AGNES_OK;
}

int agnes_kernel_times(agnes_kernel_time* out, uint32_t cap, uint32_t* n) {
    if (!n || (cap && !out)) return AGNES_E_INVALID;
    std::lock_guard<std::mutex> g(kt_mu);
    uint32_t k = 0;
    for (size_t i = 0; i < kt_used; ++i) {
        const KtRec& r = kt_recs[i];
        AGNES_TRY(hipEventSynchronize(r.e));
        float ms = 0.f;
        AGNES_TRY(hipEventElapsedTime(&ms, r.b, r.e));
        uint32_t j = 0;
        while (j < k && j < cap && std::strncmp(out[j].name, r.name, sizeof(out[j].name) - 1) != 0) ++j;
        if (j == k) {
            if (k < cap) {
                std::memset(&out[k], 0, sizeof(out[k]));
                std::strncpy(out[k].name, r.name, sizeof(out[k].name) - 1);
            }
            ++k;
        }
        if (j < cap) {
            out[j].launches += 1;
            out[j].total_ms += ms;
        }
    }
    *n = k;
    return AGNES_OK;
}

uint32_t agnes_abi_version(void) { return AGNES_ABI_VERSION; }

int agnes_ctx_create(int device, agnes_ctx** out) {
    if (!out) return AGNES_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return AGNES_E_NODEVICE;
    if (device < 0 || device >= n) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(device));
    agnes_ctx* c = new (std::nothrow) agnes_ctx();
    if (!c) return AGNES_E_NOMEM;
    c->device = device;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        cus > 0)
        c->num_cus = cus;
    hipError_t e = hipMalloc(&c->d_err, AGNES_COUNTER_BYTES);
    if (e != hipSuccess) {
        delete c;
        return status_of(e);
    }
    (void)hipMemset(c->d_err, 0, AGNES_COUNTER_BYTES);
    e = hipMalloc(&c->d_ovf, sizeof(unsigned long long));
    if (e != hipSuccess) {
        (void)hipFree(c->d_err);
        delete c;
        return status_of(e);
    }
    (void)hipMemset(c->d_ovf, 0, sizeof(unsigned long long));
    *out = c;
    return AGNES_OK;
}

void agnes_ctx_destroy(agnes_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    free_power(c);
    if (c->d_err) (void)hipFree(c->d_err);
    if (c->d_list) (void)hipFree(c->d_list);
    if (c->d_scan) (void)hipFree(c->d_scan);
    if (c->d_dd) (void)hipFree(c->d_dd);
    if (c->d_edtab) (void)hipFree(c->d_edtab);
    if (c->d_ovf) (void)hipFree(c->d_ovf);
    if (c->order_ev) (void)hipEventDestroy(c->order_ev);
    delete c;
}

int agnes_ctx_device(const agnes_ctx* c) { return c ? c->device : AGNES_E_INVALID; }

int agnes_upload_power(agnes_ctx* c, const int64_t* power, uint32_t n_sets, uint32_t n_vals,
                       const int64_t* totals) {
    if (!c || n_sets == 0 || (n_vals && !power) || (n_vals == 0 && !totals)) return AGNES_E_INVALID;
    if ((uint64_t)n_sets * n_vals >= (1ull << 32)) return AGNES_E_UNSUPPORTED; /* 32-bit row bases */
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_TRY(hipDeviceSynchronize());
    free_power(c);
    const uint64_t n = (uint64_t)n_sets * n_vals;
    std::vector<agnes_set_info> sets(n_sets);
    std::vector<uint32_t> p32(n);
    bool all_fast = true, all_w64 = true;
    for (uint32_t s = 0; s < n_sets; ++s) {
        const int64_t* row = power + (uint64_t)s * n_vals;
        int64_t t = 0;
        if (totals) t = totals[s];
        else
            for (uint32_t v = 0; v < n_vals; ++v) t = wadd(t, row[v]);
        sets[s] = set_info(row, n_vals, t);
        all_fast = all_fast && sets[s].fast;
        all_w64 = all_w64 && sets[s].w64;
        for (uint32_t v = 0; v < n_vals; ++v) p32[(uint64_t)s * n_vals + v] = (uint32_t)row[v];
    }
    const size_t pb = (size_t)(n ? n : 1);
    AGNES_TRY(hipMalloc(&c->d_power, pb * sizeof(int64_t)));
    AGNES_TRY(hipMalloc(&c->d_power32, pb * sizeof(uint32_t)));
    AGNES_TRY(hipMalloc(&c->d_sets, n_sets * sizeof(agnes_set_info)));
    if (n) {
        AGNES_TRY(hipMemcpy(c->d_power, power, n * sizeof(int64_t), hipMemcpyHostToDevice));
        AGNES_TRY(hipMemcpy(c->d_power32, p32.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    AGNES_TRY(hipMemcpy(c->d_sets, sets.data(), n_sets * sizeof(agnes_set_info),
                        hipMemcpyHostToDevice));
    c->n_sets = n_sets;
    c->n_vals = n_vals;
    c->sets_dom = all_fast ? 2u : (all_w64 ? 1u : 0u);
    return AGNES_OK;
}

int64_t agnes_lds_bytes_per_wave(const agnes_config* cfg, uint32_t n_vals) {
    if (!cfg_ok(cfg)) return AGNES_E_INVALID;
    const int64_t b = agnes_lds_per_wave(cfg->mode, cfg->flags, cfg->max_rounds, n_vals);
    return b > AGNES_MAX_LDS_PER_WAVE ? AGNES_E_UNSUPPORTED : b;
}

static int tally_impl(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b,
                      uint8_t* codes, const agnes_state* states_in, agnes_state* states,
                      agnes_carry_rec* carry, const agnes_set_info* sets, uint32_t n_sets, uint32_t sets_dom,
                      hipStream_t st, uint64_t* ev_counts = nullptr, bool* counted = nullptr,
                      void* rec_out = nullptr, bool edges = false, bool* fast_counted = nullptr) {
    if (!c || !cfg_ok(cfg) || !b || !b->offsets) return AGNES_E_INVALID;
    if (b->n_votes && (!codes || !b->instance || !b->round || !b->type || !b->value ||
                       !b->validator))
        return AGNES_E_INVALID;
    if ((cfg->flags & AGNES_FLAG_STATE_MACHINE) && !states) return AGNES_E_INVALID;
    /* the kernel reads 4 consecutive votes per lane: u32 columns 16-B aligned,
     * u8 columns and the codes 4-B aligned, weights naturally aligned */
    if (((uintptr_t)b->instance | (uintptr_t)b->value | (uintptr_t)b->validator) & 15u) return AGNES_E_INVALID;
    if (((uintptr_t)b->round | (uintptr_t)b->type | (uintptr_t)codes) & 3u) return AGNES_E_INVALID;
    if ((uintptr_t)b->weight & 7u) return AGNES_E_INVALID;
    const int64_t lpw = agnes_lds_bytes_per_wave(cfg, c->n_vals);
    if (lpw < 0) return (int)lpw;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, st);
    /* i64 for every instance with caller weights, carried executors or a power set in
     * neither fast domain; u64 sums (tally_fast<W64>) when a set is outside the u32 one */
    const bool wide_all = b->weight != nullptr || carry != nullptr || sets_dom == 0u;
    const bool w64 = !wide_all && sets_dom == 1u;
    if (!wide_all && (!c->d_list || c->list_cap < b->n_instances)) {
        /* [list_cap] deferred instances | [list_cap] walk list */
        AGNES_TRY(hipStreamSynchronize(st));
        if (c->d_list) (void)hipFree(c->d_list);
        c->d_list = nullptr;
        c->list_cap = 0;
        AGNES_TRY(hipMalloc(&c->d_list, (2 * (size_t)b->n_instances + 1) * sizeof(uint32_t)));
        c->list_cap = b->n_instances;
    }
    /* the invalid count and the work-queue counters: one memset -- or, on the flow route
     * with the unaligned-stream kernel, zeroed by its gate pass (flow_prep: one launch
     * fewer in the step) */
    const uint32_t route0 = (cfg->flags >> AGNES_ROUTE_SHIFT) & AGNES_ROUTE_MASK;
    const bool prep = !wide_all && route0 == AGNES_ROUTE_AUTO && cfg->mode == AGNES_MODE_REFERENCE &&
                      !(cfg->flags & AGNES_FLAG_ROUND_SKIP) && cfg->max_rounds <= 15u && agnes_flow_rg_build();
    if (!prep) AGNES_TRY(hipMemsetAsync(c->d_err, 0, wide_all ? AGNES_ERR_BYTES : AGNES_COUNTER_BYTES, st));
    agnes_tally_args a;
    std::memset(&a, 0, sizeof(a));
    a.prep_zero = prep ? 1u : 0u;
    a.vb = *b;
    a.power = c->d_power;
    a.power32 = c->d_power32;
    a.sets = sets;
    a.n_sets = n_sets;
    a.n_vals = c->n_vals;
    a.max_rounds = cfg->max_rounds;
    a.flags = cfg->flags;
    a.one_inst = (cfg->flags & AGNES_FLAG_ONE_INSTANCE) ? 1u : 0u;
    a.one_id = cfg->reserved;
    a.codes = codes;
    a.w64 = w64 ? 1u : 0u;
    a.states = (cfg->flags & AGNES_FLAG_STATE_MACHINE) ? states : nullptr;
    a.states_in = nullptr;
    if (a.states && states_in && states_in != states) {
        /* the sweep route reads the input States itself; the other routes work in place */
        const uint32_t route = (cfg->flags >> AGNES_ROUTE_SHIFT) & AGNES_ROUTE_MASK;
        const bool sweep = !wide_all && route == AGNES_ROUTE_AUTO &&
                           cfg->mode == AGNES_MODE_REFERENCE &&
                           !(cfg->flags & AGNES_FLAG_ROUND_SKIP) && cfg->max_rounds <= 15u;
        if (sweep) {
            a.states_in = states_in;
        } else if (b->n_instances) {
            AGNES_TRY(hipMemcpyAsync(states, states_in, (size_t)b->n_instances * sizeof(agnes_state),
                                     hipMemcpyDeviceToDevice, st));
        }
    }
    a.carry = carry;
    a.n_invalid = c->d_err;
    a.list = c->d_list;
    a.walk = c->d_list ? c->d_list + (size_t)c->list_cap : nullptr;
    a.list_count = c->d_list ? reinterpret_cast<uint32_t*>(c->d_err + AGNES_ERR_BYTES / 8) : nullptr;
    /* DEDUP / RoundSkip tables tag entries with (instance epoch, local vote index):
     * the local index of any vote is < n_votes, so it needs bit_length(n_votes - 1) bits */
    if (cfg->mode == AGNES_MODE_DEDUP || (cfg->flags & AGNES_FLAG_ROUND_SKIP)) {
        if (b->n_votes > (1ull << 31)) return AGNES_E_UNSUPPORTED;
        uint32_t lb = 1;
        while (lb < 31 && (1ull << lb) < b->n_votes) ++lb;
        /* AGNES_FLAG_EPOCH_BITS: spend more bits on the index (fewer epochs per fill) */
        const uint32_t want = (cfg->flags >> AGNES_EPOCH_BITS_SHIFT) & 0x1Fu;
        if (want > lb && want <= 31u) lb = want;
        a.epoch_shift = lb;
    } else {
        a.epoch_shift = 31;
    }
    /* agnes_tally_events: the flow route counts each instance's event records as it goes */
    if (ev_counts) {
        const uint32_t route = (cfg->flags >> AGNES_ROUTE_SHIFT) & AGNES_ROUTE_MASK;
        bool flow = !wide_all && !w64 && route == AGNES_ROUTE_AUTO && cfg->mode == AGNES_MODE_REFERENCE &&
                    !(cfg->flags & AGNES_FLAG_ROUND_SKIP) &&
                    agnes_flow_counts_events(cfg->flags, cfg->max_rounds, edges, rec_out != nullptr);
        if (flow) a.ev_counts = ev_counts;
        if (flow && rec_out) a.rec_out = rec_out; /* agnes_tally_records / _edges: the flow kernel writes them too */
        if (flow && edges) a.edges = 1u;
        if (counted) *counted = flow;
        /* the per-instance route (DEDUP, RoundSkip, or forced) counts them in tally_fast:
         * every instance it runs; the ones it defers to the i64 LIST kernel are the
         * caller's to count (agnes_tally_events: a list pass) */
        const bool fast = !flow && !wide_all && !rec_out && route != AGNES_ROUTE_WIDE &&
                          (cfg->mode == AGNES_MODE_DEDUP || (cfg->flags & AGNES_FLAG_ROUND_SKIP) ||
                           route == AGNES_ROUTE_INSTANCE || route == AGNES_ROUTE_SPLIT);
        if (fast) a.ev_counts = ev_counts;
        /* agnes_tally_edges on the split per-instance route (C4): apply_codes writes the
         * edges of every instance it walks (the LIST kernel's are the caller's to walk) */
        const bool sm = (cfg->flags & AGNES_FLAG_STATE_MACHINE) != 0;
        const bool apply_edges = !flow && edges && rec_out && !wide_all && sm &&
                                 (route == AGNES_ROUTE_AUTO || route == AGNES_ROUTE_SPLIT) &&
                                 (cfg->mode == AGNES_MODE_DEDUP || (cfg->flags & AGNES_FLAG_ROUND_SKIP) ||
                                  route == AGNES_ROUTE_SPLIT) &&
                                 agnes_apply_codes_supported(&a) && agnes_apply_edges_supported(cfg->max_rounds);
        if (apply_edges) {
            a.edge_counts = ev_counts;
            a.edge_out = rec_out;
        }
        if (fast_counted) *fast_counted = fast || apply_edges;
    }
    return status_of(agnes_launch_tally(&a, cfg->mode, c->num_cus, wide_all, st));
}

int agnes_tally(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint8_t* codes,
                agnes_state* states, void* stream) {
    if (!c || !cfg || (cfg->flags & (AGNES_FLAG_ONE_INSTANCE | AGNES_FLAG_WEIGHTS_CACHED | AGNES_FLAG_MASKED_REJECTED)))
        return AGNES_E_INVALID; /* agnes_tally_carried only */
    return tally_impl(c, cfg, b, codes, nullptr, states, nullptr, c->d_sets, c->n_sets, c->sets_dom,
                      (hipStream_t)stream);
}

int agnes_tally_states(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint8_t* codes,
                       const agnes_state* states_in, agnes_state* states_out, void* stream) {
    if (!c || !cfg || (cfg->flags & (AGNES_FLAG_ONE_INSTANCE | AGNES_FLAG_WEIGHTS_CACHED | AGNES_FLAG_MASKED_REJECTED)))
        return AGNES_E_INVALID;
    return tally_impl(c, cfg, b, codes, states_in, states_out, nullptr, c->d_sets, c->n_sets, c->sets_dom,
                      (hipStream_t)stream);
}

static_assert(sizeof(agnes_vote_count) == sizeof(agnes_carry_rec), "agnes_vote_count is the carried executor");
static_assert(sizeof(agnes_edge) == 16, "agnes_edge is one 16-B record");

int agnes_tally_carried(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint8_t* codes,
                        agnes_vote_count* counts, void* stream) {
    if (!c || !cfg || !b || (b->n_instances && !counts)) return AGNES_E_INVALID;
    if (cfg->mode != AGNES_MODE_REFERENCE || (cfg->flags & (AGNES_FLAG_ROUND_SKIP | AGNES_FLAG_STATE_MACHINE)))
        return AGNES_E_UNSUPPORTED;
    return tally_impl(c, cfg, b, codes, nullptr, nullptr, reinterpret_cast<agnes_carry_rec*>(counts), c->d_sets,
                      c->n_sets, c->sets_dom, (hipStream_t)stream);
}

int agnes_tally_partials(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, agnes_vote_count* counts,
                         int64_t* weights, void* stream) {
    if (!c || !cfg_ok(cfg) || !b || !b->offsets || (b->n_instances && !counts)) return AGNES_E_INVALID;
    if (b->n_votes && (!b->instance || !b->round || !b->type || !b->value || !b->validator))
        return AGNES_E_INVALID;
    if (cfg->mode != AGNES_MODE_REFERENCE || (cfg->flags & (AGNES_FLAG_ROUND_SKIP | AGNES_FLAG_STATE_MACHINE)))
        return AGNES_E_UNSUPPORTED;
    /* the partials gather the power table; caller weights (carried's has_w validity
     * rules: no valid validator or set needed) are not what pass A computes */
    if (b->weight) return AGNES_E_UNSUPPORTED;
    if (b->n_votes >= 0xFFFFFFFFull || cfg->max_rounds > 1024u) /* LDS: 48 B per round */
        return AGNES_E_UNSUPPORTED;
    if ((uintptr_t)weights & 7u) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    const hipStream_t st = (hipStream_t)stream;
    AGNES_ORDER(c, st);
    return status_of(agnes_launch_partials(b, c->d_power, c->d_power32, c->d_sets, c->n_sets, c->n_vals, cfg->max_rounds,
                                           (cfg->flags & AGNES_FLAG_ONE_INSTANCE) ? 1u : 0u, cfg->reserved,
                                           reinterpret_cast<agnes_carry_rec*>(counts), weights, st));
}

int agnes_last_error_count(agnes_ctx* c, uint64_t* out) {
    if (!c || !out) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_TRY(hipStreamSynchronize(c->last_stream));
    unsigned long long v[AGNES_ERR_BYTES / 8];
    AGNES_TRY(hipMemcpy(v, c->d_err, sizeof(v), hipMemcpyDeviceToHost));
    uint64_t sum = 0;
    for (uint32_t k = 0; k < AGNES_ERR_STRIPES; ++k) sum += v[k * (AGNES_ERR_STRIDE / 8u)];
    *out = sum;
    return AGNES_OK;
}

int agnes_apply_events(agnes_ctx* c, agnes_state* states, uint32_t n, const uint64_t* off,
                       const agnes_event* ev, agnes_message* msgs, uint32_t flags, void* stream) {
    if (!c || (n && (!states || !off))) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    return status_of(agnes_launch_apply_events(states, n, off, ev, msgs, flags, (hipStream_t)stream));
}

int agnes_apply_msgs(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, const uint8_t* kinds,
                     const int32_t* pol, uint8_t* codes, agnes_state* states, agnes_message* msgs, void* stream) {
    if (!c || !cfg || !b || cfg->max_rounds < 1u) return AGNES_E_INVALID;
    if (cfg->mode != AGNES_MODE_REFERENCE || (cfg->flags & (AGNES_FLAG_ROUND_SKIP | AGNES_FLAG_ONE_INSTANCE)) ||
        cfg->max_rounds > 16u)
        return AGNES_E_UNSUPPORTED;
    if (b->n_instances && (!b->offsets || !states)) return AGNES_E_INVALID;
    if (b->n_votes && (!kinds || !codes || !msgs || !b->instance || !b->round || !b->type || !b->value ||
                       (!b->weight && !b->validator)))
        return AGNES_E_INVALID;
    if (!b->weight && !c->d_sets) return AGNES_E_INVALID; /* the power table weighs the votes */
    AGNES_TRY(hipSetDevice(c->device));
    const hipStream_t st = (hipStream_t)stream;
    AGNES_ORDER(c, st);
    AGNES_TRY(hipMemsetAsync(c->d_err, 0, AGNES_ERR_BYTES, st));
    return status_of(agnes_launch_apply_msgs(b, kinds, pol, c->d_power, c->d_sets, c->n_sets, c->n_vals,
                                             cfg->max_rounds, cfg->flags, states, msgs, codes, c->d_err, st));
}

/* ---------------- C5: the State machine of a split instance ---------------- */

static int one_sm_args(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint64_t base,
                       const uint8_t* codes, const agnes_state* state, const int64_t* marks) {
    if (!c || !cfg || !b || !state || !marks) return AGNES_E_INVALID;
    if (cfg->mode > AGNES_MODE_DEDUP || (cfg->flags & AGNES_FLAG_ROUND_SKIP)) return AGNES_E_UNSUPPORTED;
    if (b->n_votes && (!codes || !b->round || !b->value)) return AGNES_E_INVALID;
    if (base + b->n_votes > (1ull << 31) || base + b->n_votes < base) return AGNES_E_UNSUPPORTED;
    return AGNES_OK;
}

int agnes_one_sm_scan(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint64_t base,
                      const uint8_t* codes, const agnes_state* state, int64_t* marks, void* stream) {
    const int rc = one_sm_args(c, cfg, b, base, codes, state, marks);
    if (rc != AGNES_OK) return rc;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    return status_of(agnes_launch_one_sm(0, codes, b->round, b->value, b->n_votes, base,
                                         const_cast<agnes_state*>(state), marks, c->num_cus, (hipStream_t)stream));
}

int agnes_one_sm_apply(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint64_t base,
                       uint8_t* codes, const agnes_state* state, int64_t* marks, void* stream) {
    const int rc = one_sm_args(c, cfg, b, base, codes, state, marks);
    if (rc != AGNES_OK) return rc;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    return status_of(agnes_launch_one_sm(1, codes, b->round, b->value, b->n_votes, base,
                                         const_cast<agnes_state*>(state), marks, c->num_cus, (hipStream_t)stream));
}

int agnes_one_sm_finish(agnes_ctx* c, const int64_t* marks, agnes_state* state, void* stream) {
    if (!c || !marks || !state) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    return status_of(agnes_launch_one_sm(2, nullptr, nullptr, nullptr, 0, 0, state, const_cast<int64_t*>(marks),
                                         c->num_cus, (hipStream_t)stream));
}

/* ---------------- wire format + Ed25519 ---------------- */

int agnes_wire_ingest(agnes_ctx* c, const agnes_wire_vote* records, uint64_t n, const uint8_t* pubkeys,
                      uint32_t n_sets, uint32_t n_vals, const uint32_t* instance_set, uint32_t n_instances,
                      int64_t height, uint32_t max_rounds, uint32_t* instance, uint8_t* round, uint8_t* type,
                      uint32_t* value, uint32_t* validator, uint8_t* verdict, void* stream) {
    if (!c || max_rounds == 0u || max_rounds > 256u) return AGNES_E_INVALID;
    if (n && (!records || !instance || !round || !type || !value || !validator || !verdict)) return AGNES_E_INVALID;
    if (n && n_sets && n_vals && !pubkeys) return AGNES_E_INVALID;
    if (((uintptr_t)records & 7u) || ((uintptr_t)pubkeys & 15u)) return AGNES_E_INVALID;
    if (n > (1ull << 36)) return AGNES_E_UNSUPPORTED; /* (n + 255) / 256 blocks fit the grid */
    AGNES_TRY(hipSetDevice(c->device));
    const hipStream_t st = (hipStream_t)stream;
    AGNES_ORDER(c, st);
    if (!c->d_edtab) { /* the fixed-base table: once per context, on the caller's stream */
        AGNES_TRY(hipMalloc(&c->d_edtab, agnes_wire_table_bytes()));
        AGNES_TRY(agnes_launch_wire_table(c->d_edtab, st));
    }
    agnes_wire_args a{records, n, pubkeys, n_sets, n_vals, instance_set, n_instances, max_rounds, height,
                      instance, value, validator, round, type, verdict, c->d_edtab};
    AgnesKt kt("wire_ingest", st);
    return status_of(agnes_launch_wire_ingest(&a, st));
}

/* ---------------- validator sets ---------------- */

int agnes_valset_build(agnes_ctx* c, const uint8_t* addr, uint32_t addr_len, const int64_t* power,
                       const uint32_t* set_of, uint64_t n, uint32_t n_sets, uint32_t* order, uint64_t* set_offsets,
                       int64_t* power_out, int64_t* totals, uint8_t* addr_out, uint64_t* n_out, void* stream) {
    if (!c || !n_out || n_sets == 0 || addr_len == 0 || addr_len > 64u || !set_offsets || !totals) return AGNES_E_INVALID;
    if (n && (!addr || !power || !order || !power_out)) return AGNES_E_INVALID;
    if (n > (1ull << 30)) return AGNES_E_UNSUPPORTED;
    AGNES_TRY(hipSetDevice(c->device));
    const hipStream_t st = (hipStream_t)stream;
    AGNES_ORDER(c, st);
    uint32_t N = 2048u; /* the sort's power of two (>= one LDS tile) */
    while (N < n) N <<= 1;
    uint32_t* idx = nullptr;
    uint64_t* pos = nullptr;
    uint64_t* scr = nullptr;
    uint32_t* set_out = nullptr;
    hipError_t e = hipMalloc(&idx, 4ull * N);
    if (e == hipSuccess) e = hipMalloc(&pos, 8ull * (N + 1ull));
    if (e == hipSuccess) e = hipMalloc(&scr, 8ull * (agnes_edges_scratch_words(N) + 1u));
    if (e == hipSuccess) e = hipMalloc(&set_out, 4ull * (n ? n : 1u));
    if (e == hipSuccess)
        e = agnes_launch_valset_build(addr, addr_len, power, set_of, (uint32_t)n, n_sets, idx, N, pos, scr, set_out,
                                      order, power_out, addr_out, set_offsets, totals, st);
    uint64_t m = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&m, pos + N, sizeof(m), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(idx);
    (void)hipFree(pos);
    (void)hipFree(scr);
    (void)hipFree(set_out);
    if (e != hipSuccess) return status_of(e);
    *n_out = m;
    return AGNES_OK;
}

int agnes_valset_find(agnes_ctx* c, const uint8_t* sorted_addr, uint32_t addr_len, const uint64_t* set_offsets,
                      uint32_t n_sets, const uint8_t* q_addr, const uint32_t* q_set, uint64_t n_q, uint64_t* out,
                      void* stream) {
    if (!c || !set_offsets || addr_len == 0 || addr_len > 64u || (n_q && (!q_addr || !out || !sorted_addr)))
        return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    return status_of(agnes_launch_valset_find(sorted_addr, addr_len, set_offsets, n_sets, q_addr, q_set, n_q, out,
                                              (hipStream_t)stream));
}

/* ---------------- edge-triggered summary ---------------- */

static bool edges_args_ok(const agnes_config* cfg, const agnes_vote_batch* b, const uint8_t* codes) {
    /* the walks read codes, round and type 4 bytes at a time */
    return cfg && b && cfg->max_rounds >= 1u && cfg->max_rounds <= 256u &&
           !(((uintptr_t)codes | (uintptr_t)b->round | (uintptr_t)b->type) & 3u) &&
           (b->n_instances == 0 || (b->offsets && (b->n_votes == 0 || (codes && b->round && b->type))));
}

int agnes_edge_offsets(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, const uint8_t* codes,
                       uint64_t* offsets, void* stream) {
    if (!c || !offsets || !edges_args_ok(cfg, b, codes)) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    const uint64_t words = agnes_edges_scratch_words(b->n_instances);
    if (words > c->scan_cap) {
        if (c->d_scan) AGNES_TRY(hipFree(c->d_scan));
        c->d_scan = nullptr;
        c->scan_cap = 0;
        AGNES_TRY(hipMalloc(&c->d_scan, words * sizeof(uint64_t)));
        c->scan_cap = words;
    }
    return status_of(agnes_launch_edges(b, codes, cfg->max_rounds, offsets, nullptr, c->d_scan,
                                        (hipStream_t)stream));
}

int agnes_edges(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, const uint8_t* codes,
                const uint64_t* offsets, agnes_edge* out, uint64_t out_cap, void* stream) {
    if (!c || !offsets || !out || !edges_args_ok(cfg, b, codes) || ((uintptr_t)out & 15u)) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    return status_of(agnes_launch_edges(b, codes, cfg->max_rounds, const_cast<uint64_t*>(offsets), out,
                                        nullptr, (hipStream_t)stream, out_cap, c->d_ovf));
}

int agnes_records_overflow(agnes_ctx* c, uint64_t* dropped) {
    if (!c || !dropped) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_TRY(hipStreamSynchronize(c->last_stream));
    unsigned long long v = 0;
    AGNES_TRY(hipMemcpy(&v, c->d_ovf, sizeof(v), hipMemcpyDeviceToHost));
    if (v) AGNES_TRY(hipMemset(c->d_ovf, 0, sizeof(v)));
    *dropped = v;
    return v ? AGNES_E_OVERFLOW : AGNES_OK;
}

/* ---------------- C5: the fold of one instance's slices ---------------- */

int agnes_fold_counts(agnes_ctx* c, agnes_vote_count* counts, uint32_t n_slices, uint32_t keys,
                      const agnes_vote_count* carry, agnes_vote_count* totals, uint32_t flags, void* stream) {
    if (!c || (n_slices && keys && !counts) || keys > 512u || (flags & ~0x1Fu)) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    return status_of(agnes_launch_fold(counts, n_slices, keys, carry, totals, flags, (hipStream_t)stream));
}

/* ---------------- event stream ---------------- */

int agnes_event_offsets(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, const uint8_t* codes,
                        uint64_t* offsets, void* stream) {
    if (!c || !offsets || !edges_args_ok(cfg, b, codes)) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    const uint64_t words = agnes_edges_scratch_words(b->n_instances);
    if (words > c->scan_cap) {
        if (c->d_scan) AGNES_TRY(hipFree(c->d_scan));
        c->d_scan = nullptr;
        c->scan_cap = 0;
        AGNES_TRY(hipMalloc(&c->d_scan, words * sizeof(uint64_t)));
        c->scan_cap = words;
    }
    return status_of(agnes_launch_events(b, codes, cfg->max_rounds, offsets, nullptr, c->d_scan,
                                         (hipStream_t)stream));
}

uint64_t agnes_events_capacity(const agnes_config* cfg, const agnes_vote_batch* b) {
    if (!cfg || !b) return 0;
    return b->n_votes * ((cfg->flags & AGNES_FLAG_ROUND_SKIP) ? 2u : 1u);
}

int agnes_tally_events(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint8_t* codes,
                       const agnes_state* states_in, agnes_state* states_out, uint64_t* offsets,
                       agnes_vote_event* out, void* stream) {
    if (!c || !cfg || !b || (cfg->flags & (AGNES_FLAG_ONE_INSTANCE | AGNES_FLAG_WEIGHTS_CACHED | AGNES_FLAG_MASKED_REJECTED))) return AGNES_E_INVALID;
    if (!offsets || !out || ((uintptr_t)out & 7u)) return AGNES_E_INVALID;
    if (b->n_votes && (!b->value || ((uintptr_t)b->value & 3u))) return AGNES_E_INVALID;
    if (cfg_ok(cfg) && cfg->max_rounds > 64u) return AGNES_E_UNSUPPORTED; /* the emit's value slots in LDS */
    const hipStream_t st = (hipStream_t)stream;
    bool counted = false, fast_counted = false;
    const int rc = tally_impl(c, cfg, b, codes, states_in, states_out, nullptr, c->d_sets, c->n_sets, c->sets_dom, st,
                              offsets + 1, &counted, nullptr, false, &fast_counted);
    if (rc != AGNES_OK) return rc;
    const uint64_t words = agnes_edges_scratch_words(b->n_instances);
    if (words > c->scan_cap) {
        AGNES_TRY(hipStreamSynchronize(st));
        if (c->d_scan) AGNES_TRY(hipFree(c->d_scan));
        c->d_scan = nullptr;
        c->scan_cap = 0;
        AGNES_TRY(hipMalloc(&c->d_scan, words * sizeof(uint64_t)));
        c->scan_cap = words;
    }
    if (counted || fast_counted) {
        /* the tally counted its instances' records; the flow kernel's walk list, or the
         * instances tally_fast deferred to the LIST kernel, here */
        AGNES_TRY(hipMemsetAsync(offsets, 0, sizeof(uint64_t), st));
        const uint32_t* const lc = reinterpret_cast<const uint32_t*>(c->d_err + AGNES_ERR_BYTES / 8);
        if (counted)
            AGNES_TRY(agnes_launch_event_count_list(b, codes, c->d_list + (size_t)c->list_cap, lc + AGNES_WALK_COUNT,
                                                    offsets, c->num_cus, st));
        else
            AGNES_TRY(agnes_launch_event_count_list(b, codes, c->d_list, lc, offsets, c->num_cus, st));
        AgnesKt kt("event_scan", st);
        AGNES_TRY(agnes_launch_offsets_scan(offsets, b->n_instances, c->d_scan, st));
    } else {
        AGNES_TRY(agnes_launch_events(b, codes, cfg->max_rounds, offsets, nullptr, c->d_scan, st));
    }
    /* out holds agnes_events_capacity() records (the contract): the emit never writes past it */
    return status_of(agnes_launch_events(b, codes, cfg->max_rounds, offsets, out, nullptr, st,
                                         agnes_events_capacity(cfg, b), c->d_ovf));
}

static_assert(sizeof(agnes_seg_event) == 16, "agnes_seg_event is one 16-B record");

int agnes_tally_records(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint8_t* codes,
                        const agnes_state* states_in, agnes_state* states_out, uint64_t* counts, agnes_seg_event* out,
                        void* stream) {
    if (!c || !cfg || !b || (cfg->flags & (AGNES_FLAG_ONE_INSTANCE | AGNES_FLAG_WEIGHTS_CACHED | AGNES_FLAG_MASKED_REJECTED)))
        return AGNES_E_INVALID;
    if ((b->n_instances && !counts) || (b->n_votes && !out) || ((uintptr_t)out & 15u)) return AGNES_E_INVALID;
    if (b->n_votes && (!b->value || ((uintptr_t)b->value & 3u))) return AGNES_E_INVALID;
    if (cfg_ok(cfg) && cfg->max_rounds > 64u) return AGNES_E_UNSUPPORTED; /* the walk's value slots in LDS */
    const hipStream_t st = (hipStream_t)stream;
    bool counted = false;
    const int rc = tally_impl(c, cfg, b, codes, states_in, states_out, nullptr, c->d_sets, c->n_sets, c->sets_dom, st,
                              counts, &counted, out);
    if (rc != AGNES_OK) return rc;
    const uint32_t mult = (cfg->flags & AGNES_FLAG_ROUND_SKIP) ? 2u : 1u;
    if (counted) /* the flow kernel wrote its batches' records; the walk list's instances here */
        return status_of(agnes_launch_seg_walk(b, codes, cfg->max_rounds, mult, c->d_list + (size_t)c->list_cap,
                                               reinterpret_cast<const uint32_t*>(c->d_err + AGNES_ERR_BYTES / 8) +
                                                   AGNES_WALK_COUNT,
                                               counts, out, st));
    /* the emit pass keeps record positions inside a batch as u32: a batch that could
     * hold 2^32 records or more (n_votes x mult) goes to the walk, whose positions are u64 */
    if (b->n_instances && (uint64_t)b->n_votes * mult < (1ull << 32) && agnes_seg_emit_ok(b, codes, cfg->max_rounds))
        /* the event stream's emit pass writing each record to its instance's segment
         * (and the counts): no count pass before it */
        return status_of(agnes_launch_seg_emit(b, codes, cfg->max_rounds, mult, counts, out, st));
    return status_of(agnes_launch_seg_walk(b, codes, cfg->max_rounds, mult, nullptr, nullptr, counts, out, st));
}

int agnes_tally_edges(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint8_t* codes,
                      const agnes_state* states_in, agnes_state* states_out, uint64_t* counts, agnes_edge* out,
                      void* stream) {
    if (!c || !cfg || !b || (cfg->flags & (AGNES_FLAG_ONE_INSTANCE | AGNES_FLAG_WEIGHTS_CACHED | AGNES_FLAG_MASKED_REJECTED)))
        return AGNES_E_INVALID;
    if ((b->n_instances && !counts) || (b->n_votes && !out) || ((uintptr_t)out & 15u)) return AGNES_E_INVALID;
    if (cfg_ok(cfg) && cfg->max_rounds > 128u) return AGNES_E_UNSUPPORTED; /* the walk's executor bytes in LDS */
    const hipStream_t st = (hipStream_t)stream;
    bool counted = false, applied = false;
    const int rc = tally_impl(c, cfg, b, codes, states_in, states_out, nullptr, c->d_sets, c->n_sets, c->sets_dom, st,
                              counts, &counted, out, true, &applied);
    if (rc != AGNES_OK) return rc;
    if (applied) /* apply_codes wrote the edges; the instances deferred to the LIST kernel here */
        return status_of(agnes_launch_edge_seg_walk(b, codes, cfg->max_rounds, c->d_list,
                                                    reinterpret_cast<const uint32_t*>(c->d_err + AGNES_ERR_BYTES / 8),
                                                    counts, out, st));
    if (counted) /* the flow kernel wrote its batches' edges; the walk list's instances here */
        return status_of(agnes_launch_edge_seg_walk(b, codes, cfg->max_rounds, c->d_list + (size_t)c->list_cap,
                                                    reinterpret_cast<const uint32_t*>(c->d_err + AGNES_ERR_BYTES / 8) +
                                                        AGNES_WALK_COUNT,
                                                    counts, out, st));
    return status_of(agnes_launch_edge_seg_walk(b, codes, cfg->max_rounds, nullptr, nullptr, counts, out, st));
}

int agnes_edges_compact(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, const uint64_t* counts,
                        const agnes_edge* seg, uint64_t* offsets, agnes_edge* out, uint64_t out_cap, void* stream) {
    if (!c || !cfg_ok(cfg) || !b || !b->offsets || !offsets || (b->n_instances && (!counts || !seg)) ||
        ((uintptr_t)out & 15u) || ((uintptr_t)seg & 15u))
        return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    const hipStream_t st = (hipStream_t)stream;
    AGNES_ORDER(c, st);
    AGNES_TRY(hipMemsetAsync(offsets, 0, sizeof(uint64_t), st));
    if (b->n_instances == 0) return AGNES_OK;
    const uint64_t words = agnes_edges_scratch_words(b->n_instances);
    if (words > c->scan_cap) {
        AGNES_TRY(hipStreamSynchronize(st));
        if (c->d_scan) AGNES_TRY(hipFree(c->d_scan));
        c->d_scan = nullptr;
        c->scan_cap = 0;
        AGNES_TRY(hipMalloc(&c->d_scan, words * sizeof(uint64_t)));
        c->scan_cap = words;
    }
    AGNES_TRY(hipMemcpyAsync(offsets + 1, counts, sizeof(uint64_t) * b->n_instances, hipMemcpyDeviceToDevice, st));
    {
        AgnesKt kt("edge_scan", st);
        AGNES_TRY(agnes_launch_offsets_scan(offsets, b->n_instances, c->d_scan, st));
    }
    if (!out) return AGNES_OK;
    return status_of(agnes_launch_edge_compact(b, seg, offsets, out, st, out_cap, c->d_ovf));
}

int agnes_records_compact(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, const uint64_t* counts,
                          const agnes_seg_event* seg, uint64_t* offsets, agnes_vote_event* out, uint64_t out_cap,
                          void* stream) {
    if (!c || !cfg_ok(cfg) || !b || !b->offsets || !offsets || (b->n_instances && (!counts || !seg)) ||
        ((uintptr_t)out & 7u) || ((uintptr_t)seg & 15u))
        return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    const hipStream_t st = (hipStream_t)stream;
    AGNES_ORDER(c, st);
    AGNES_TRY(hipMemsetAsync(offsets, 0, sizeof(uint64_t), st));
    if (b->n_instances == 0) return AGNES_OK;
    const uint64_t words = agnes_edges_scratch_words(b->n_instances);
    if (words > c->scan_cap) {
        AGNES_TRY(hipStreamSynchronize(st));
        if (c->d_scan) AGNES_TRY(hipFree(c->d_scan));
        c->d_scan = nullptr;
        c->scan_cap = 0;
        AGNES_TRY(hipMalloc(&c->d_scan, words * sizeof(uint64_t)));
        c->scan_cap = words;
    }
    AGNES_TRY(hipMemcpyAsync(offsets + 1, counts, sizeof(uint64_t) * b->n_instances, hipMemcpyDeviceToDevice, st));
    {
        AgnesKt kt("event_scan", st);
        AGNES_TRY(agnes_launch_offsets_scan(offsets, b->n_instances, c->d_scan, st));
    }
    if (!out) return AGNES_OK; /* the offsets only (the caller sizes out from offsets[n]) */
    const uint32_t mult = (cfg->flags & AGNES_FLAG_ROUND_SKIP) ? 2u : 1u;
    return status_of(agnes_launch_seg_compact(b, mult, seg, offsets, out, st, out_cap, c->d_ovf));
}

int agnes_events(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, const uint8_t* codes,
                 const uint64_t* offsets, agnes_vote_event* out, uint64_t out_cap, void* stream) {
    if (!c || !offsets || !out || !edges_args_ok(cfg, b, codes) || ((uintptr_t)out & 7u)) return AGNES_E_INVALID;
    if (cfg->max_rounds > 64u) return AGNES_E_UNSUPPORTED; /* the value slots of a lane's executors in LDS */
    if (b->n_votes && (!b->value || ((uintptr_t)b->value & 3u))) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    return status_of(agnes_launch_events(b, codes, cfg->max_rounds, const_cast<uint64_t*>(offsets), out,
                                         nullptr, (hipStream_t)stream, out_cap, c->d_ovf));
}

/* ---------------- DEDUP for a split instance ---------------- */

/* fused: agnes_dedup_first_mask (first and type_out from one counting sort) */
static int dedup_impl(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint64_t base,
                      uint64_t* first, uint8_t* type_out, void* stream, bool fused = false) {
    if (!c || !cfg_ok(cfg) || !b || !first) return AGNES_E_INVALID;
    if (b->n_votes && (!b->instance || !b->round || !b->type || !b->validator)) return AGNES_E_INVALID;
    if (c->n_vals == 0) return AGNES_E_INVALID; /* no power table: no validator range */
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    if (b->instance_set) return AGNES_E_UNSUPPORTED; /* one instance: its set is reserved % n_sets */
    const uint32_t set = cfg->reserved % (c->n_sets ? c->n_sets : 1u);
    if ((!type_out || fused) && b->n_votes && agnes_dedup_bucketed(b->n_votes, cfg->max_rounds, c->n_vals)) {
        /* the first-index table by a counting sort over key buckets: no global atomics */
        const uint64_t need = agnes_dedup_scratch_bytes(b->n_votes, cfg->max_rounds, c->n_vals);
        if (need > c->dd_cap) {
            if (c->d_dd) AGNES_TRY(hipFree(c->d_dd));
            c->d_dd = nullptr;
            c->dd_cap = 0;
            AGNES_TRY(hipMalloc(&c->d_dd, need));
            c->dd_cap = need;
        }
        return status_of(agnes_launch_dedup_first_bucketed(b, cfg->reserved, cfg->max_rounds, c->n_vals,
                                                           set < c->n_sets, base, first, fused ? type_out : nullptr,
                                                           c->d_dd, (hipStream_t)stream));
    }
    if (fused) { /* outside the bucketed domain: the two passes over a filled table */
        AGNES_TRY(agnes_launch_dedup_fill(first, 2ull * cfg->max_rounds * c->n_vals, (hipStream_t)stream));
        const int rc = status_of(agnes_launch_dedup(b, cfg->reserved, cfg->max_rounds, c->n_vals, set < c->n_sets,
                                                    base, first, nullptr, (hipStream_t)stream));
        if (rc != AGNES_OK) return rc;
    }
    return status_of(agnes_launch_dedup(b, cfg->reserved, cfg->max_rounds, c->n_vals, set < c->n_sets, base,
                                        first, type_out, (hipStream_t)stream));
}

int agnes_dedup_first(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint64_t base,
                      uint64_t* first, void* stream) {
    return dedup_impl(c, cfg, b, base, first, nullptr, stream);
}

int agnes_dedup_mask(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint64_t base,
                     const uint64_t* first, uint8_t* type_out, void* stream) {
    if (!type_out && b && b->n_votes) return AGNES_E_INVALID;
    if (b && b->n_votes == 0) return AGNES_OK;
    return dedup_impl(c, cfg, b, base, const_cast<uint64_t*>(first), type_out, stream);
}

int agnes_dedup_first_mask(agnes_ctx* c, const agnes_config* cfg, const agnes_vote_batch* b, uint64_t base,
                           uint64_t* first, uint8_t* type_out, void* stream) {
    if (!c || !cfg_ok(cfg) || !b || !first) return AGNES_E_INVALID;
    if (!type_out && b->n_votes) return AGNES_E_INVALID;
    if (b->n_votes == 0) { /* no vote: the table is still written whole (INT64_MAX everywhere) */
        if (c->n_vals == 0) return AGNES_E_INVALID;
        AGNES_TRY(hipSetDevice(c->device));
        AGNES_ORDER(c, (hipStream_t)stream);
        AGNES_TRY(agnes_launch_dedup_fill(first, 2ull * cfg->max_rounds * c->n_vals, (hipStream_t)stream));
        return AGNES_OK;
    }
    return dedup_impl(c, cfg, b, base, first, type_out, stream, true);
}

int agnes_dedup_reject(agnes_ctx* c, const uint8_t* type_masked, uint64_t n, uint8_t* codes, void* stream) {
    if (!c || (n && (!type_masked || !codes))) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    return status_of(agnes_launch_dedup_reject(type_masked, n, codes, (hipStream_t)stream));
}

/* ---------------- generator ---------------- */

uint64_t agnes_gen_instance_votes(const agnes_gen_params* p, uint32_t i) {
    if (!agnes_gen_params_ok(p)) return 0;
    return agnes_gen_host_instance_votes(p, i);
}

int agnes_gen_offsets(const agnes_gen_params* p, uint64_t* offsets) {
    return agnes_gen_host_offsets(p, offsets);
}

int agnes_gen_power(uint64_t seed, uint32_t n_sets, uint32_t n_vals, uint32_t kind, int64_t lo,
                    int64_t hi, int64_t* power) {
    return agnes_gen_host_power(seed, n_sets, n_vals, kind, lo, hi, power);
}

int agnes_gen_votes_device(agnes_ctx* c, const agnes_gen_params* p, const uint64_t* d_offsets,
                           uint64_t n_votes, uint32_t* instance, uint8_t* round, uint8_t* type,
                           uint32_t* value, uint32_t* validator, void* stream) {
    if (!c || !agnes_gen_params_ok(p) || !d_offsets) return AGNES_E_INVALID;
    if (n_votes && (!instance || !round || !type || !value || !validator)) return AGNES_E_INVALID;
    AGNES_TRY(hipSetDevice(c->device));
    AGNES_ORDER(c, (hipStream_t)stream);
    return status_of(agnes_launch_gen(p, d_offsets, n_votes, instance, round, type, value,
                                      validator, (hipStream_t)stream));
}

/* ---------------- scalar mirror ---------------- */

/* One GPU-resident executor pair (prevotes, precommits) + a 1-vote batch.
 * device block: [set_info 56][pad][carry 3x24][offsets 16][weight 8][pad][instance 16]
 *               [value 16][validator 16][round 4][type 4][code 4]
 * (vote columns 16-byte aligned: the kernel reads 4 votes per lane) */
namespace {
constexpr size_t SX_SET = 0, SX_CARRY = 64, SX_OFF = 144, SX_W = 160, SX_INST = 176, SX_VAL = 192,
                 SX_VIDX = 208, SX_ROUND = 224, SX_TYPE = 228, SX_CODE = 232, SX_BYTES = 240;
static_assert(sizeof(agnes_set_info) <= SX_CARRY, "scalar block layout");

struct ScalarExec {
    unsigned char* dev = nullptr;
};

bool sx_init(ScalarExec* x, int64_t total) {
    agnes_ctx* c = nullptr;
    if (scalar_ctx(&c) != AGNES_OK) return false;
    if (hipSetDevice(c->device) != hipSuccess) return false;
    if (hipMalloc(&x->dev, SX_BYTES) != hipSuccess) return false;
    unsigned char host[SX_BYTES];
    std::memset(host, 0, sizeof(host));
    agnes_set_info si = set_info(nullptr, 0, total);
    si.fast = 0; /* caller weights: always the wrapping i64 path */
    si.w64 = 0;
    std::memcpy(host + SX_SET, &si, sizeof(si));
    const uint64_t off[2] = {0, 1};
    std::memcpy(host + SX_OFF, off, sizeof(off));
    if (hipMemcpy(x->dev, host, SX_BYTES, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(x->dev);
        x->dev = nullptr;
        return false;
    }
    return true;
}

/* Tally one vote on the GPU against executor record `slot` (0 prevotes,
 * 1 precommits) as vote type `as_type`; returns the vote's code byte and the
 * executor's last value label. */
int sx_add(ScalarExec* x, uint32_t slot, uint32_t as_type, uint32_t value, int64_t weight,
           uint32_t* code, uint32_t* label) {
    agnes_ctx* c = nullptr;
    int rc = scalar_ctx(&c);
    if (rc != AGNES_OK) return rc;
    AGNES_TRY(hipSetDevice(c->device));
    unsigned char stage[SX_CODE - SX_W];
    std::memset(stage, 0, sizeof(stage));
    std::memcpy(stage + (SX_W - SX_W), &weight, 8);
    std::memcpy(stage + (SX_VAL - SX_W), &value, 4);
    stage[SX_TYPE - SX_W] = (uint8_t)as_type;
    AGNES_TRY(hipMemcpy(x->dev + SX_W, stage, sizeof(stage), hipMemcpyHostToDevice));
    agnes_vote_batch b;
    std::memset(&b, 0, sizeof(b));
    b.instance = (const uint32_t*)(x->dev + SX_INST);
    b.round = x->dev + SX_ROUND;
    b.type = x->dev + SX_TYPE;
    b.value = (const uint32_t*)(x->dev + SX_VAL);
    b.validator = (const uint32_t*)(x->dev + SX_VIDX);
    b.offsets = (const uint64_t*)(x->dev + SX_OFF);
    b.weight = (const int64_t*)(x->dev + SX_W);
    b.n_votes = 1;
    b.n_instances = 1;
    agnes_config cfg = {AGNES_MODE_REFERENCE, 0u, 1u, 0u};
    const uint32_t saved_nv = c->n_vals;
    c->n_vals = 0; /* no power table: the validator index is unused */
    agnes_carry_rec* carry = (agnes_carry_rec*)(x->dev + SX_CARRY) + slot;
    rc = tally_impl(c, &cfg, &b, x->dev + SX_CODE, nullptr, nullptr, carry,
                    (const agnes_set_info*)(x->dev + SX_SET), 1u, false, nullptr);
    c->n_vals = saved_nv;
    if (rc != AGNES_OK) return rc;
    unsigned char back[SX_BYTES];
    AGNES_TRY(hipMemcpy(back, x->dev, SX_BYTES, hipMemcpyDeviceToHost));
    agnes_carry_rec cr;
    std::memcpy(&cr, back + SX_CARRY + (slot + as_type) * sizeof(agnes_carry_rec), sizeof(cr));
    *code = back[SX_CODE];
    *label = cr.value;
    return AGNES_OK;
}
} // namespace

struct agnes_ve {
    ScalarExec x;
};

struct agnes_rv {
    ScalarExec x;
};

agnes_ve* agnes_ve_new(int64_t height, int64_t total_weight) {
    (void)height; /* stored but never read by the reference either (round_votes.rs:75) */
    std::lock_guard<std::mutex> g(g_mu);
    agnes_ve* ve = new (std::nothrow) agnes_ve();
    if (!ve) return nullptr;
    if (!sx_init(&ve->x, total_weight)) {
        delete ve;
        return nullptr;
    }
    return ve;
}

int agnes_ve_apply(agnes_ve* ve, const agnes_vote* vote, int64_t weight, agnes_event* out) {
    if (!ve || !vote || vote->typ > 1) return AGNES_E_INVALID;
    std::lock_guard<std::mutex> g(g_mu);
    /* the reference executor ignores vote.round: one RoundVotes at round 0
     * (vote_executor.rs:9,14); the engine tallies the vote in that executor */
    uint32_t code = 0, label = 0;
    const int rc = sx_add(&ve->x, 0u, vote->typ, vote->value, weight, &code, &label);
    if (rc != AGNES_OK) return rc;
    code &= AGNES_CODE_EVENT_MASK;
    if (code == AGNES_CODE_NONE) return 0;
    if (code > AGNES_CODE_PRECOMMIT_VALUE) return AGNES_E_DEVICE;
    if (out) {
        std::memset(out, 0, sizeof(*out));
        out->kind = (uint8_t)(code + 3u); /* CODE_POLKA_ANY(1).. -> EV_POLKA_ANY(4).. */
        out->round = vote->round;         /* apply_event(v.round, ..), consensus_executor.rs:68 */
        out->value = (code == AGNES_CODE_POLKA_VALUE || code == AGNES_CODE_PRECOMMIT_VALUE) ? label : 0u;
    }
    return 1;
}

void agnes_ve_free(agnes_ve* ve) {
    if (!ve) return;
    std::lock_guard<std::mutex> g(g_mu);
    if (g_ctx) (void)hipSetDevice(g_ctx->device);
    if (ve->x.dev) (void)hipFree(ve->x.dev);
    delete ve;
}

agnes_rv* agnes_rv_new(int64_t height, int64_t round, int64_t total) {
    (void)height;
    (void)round; /* RoundVotes.height/.round are never read (round_votes.rs:75-76) */
    std::lock_guard<std::mutex> g(g_mu);
    agnes_rv* rv = new (std::nothrow) agnes_rv();
    if (!rv) return nullptr;
    if (!sx_init(&rv->x, total)) {
        delete rv;
        return nullptr;
    }
    return rv;
}

int agnes_rv_add_vote(agnes_rv* rv, const agnes_vote* vote, int64_t weight, uint32_t* value) {
    if (!rv || !vote || vote->typ > 1) return AGNES_E_INVALID;
    std::lock_guard<std::mutex> g(g_mu);
    /* tallied as a prevote against the vote type's own executor record: the
     * prevote event codes are in bijection with Thresh (vote_executor.rs:29-31) */
    uint32_t code = 0, label = 0;
    const int rc = sx_add(&rv->x, vote->typ, 0u, vote->value, weight, &code, &label);
    if (rc != AGNES_OK) return rc;
    switch (code & AGNES_CODE_EVENT_MASK) {
    case AGNES_CODE_NONE: return (int)AGNES_THRESH_INIT;
    case AGNES_CODE_POLKA_ANY: return (int)AGNES_THRESH_ANY;
    case AGNES_CODE_POLKA_NIL: return (int)AGNES_THRESH_NIL;
    case AGNES_CODE_POLKA_VALUE:
        if (value) *value = label;
        return (int)AGNES_THRESH_VALUE;
    default: return AGNES_E_DEVICE;
    }
}

void agnes_rv_free(agnes_rv* rv) {
    if (!rv) return;
    std::lock_guard<std::mutex> g(g_mu);
    if (g_ctx) (void)hipSetDevice(g_ctx->device);
    if (rv->x.dev) (void)hipFree(rv->x.dev);
    delete rv;
}

void agnes_state_init(int64_t height, agnes_state* out) {
    if (!out) return;
    std::memset(out, 0, sizeof(*out)); /* State::new, state_machine.rs:35-43 */
    out->height = height;
    out->round = 0;
    out->step = AGNES_STEP_NEW_ROUND;
}

int agnes_state_apply(const agnes_state* in, int64_t round, const agnes_event* ev, uint32_t flags,
                      agnes_state* out, agnes_message* msg) {
    if (!in || !ev || !out) return AGNES_E_INVALID;
    std::lock_guard<std::mutex> g(g_mu);
    agnes_ctx* c = nullptr;
    int rc = scalar_ctx(&c);
    if (rc != AGNES_OK) return rc;
    AGNES_TRY(hipSetDevice(c->device));
    struct Blk {
        agnes_state s;
        agnes_event e;
        uint64_t off[2];
        agnes_message m;
    } h;
    std::memset(&h, 0, sizeof(h));
    h.s = *in;
    h.e = *ev;
    h.e.round = round;
    h.off[0] = 0;
    h.off[1] = 1;
    Blk* d = nullptr;
    AGNES_TRY(hipMalloc(&d, sizeof(Blk)));
    hipError_t e = hipMemcpy(d, &h, sizeof(Blk), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = agnes_launch_apply_events(&d->s, 1u, d->off, &d->e, &d->m, flags, nullptr);
    if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof(Blk), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return status_of(e);
    *out = h.s;
    if (msg) *msg = h.m;
    return h.m.kind != AGNES_MSG_NONE ? 1 : 0;
}

} // extern "C"
