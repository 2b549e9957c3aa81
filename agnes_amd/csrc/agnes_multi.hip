/*
 * agnes_multi.hip — the native multi-GPU driver (include/agnes.h agnes_multi_*):
 * one agnes_ctx, one HIP stream and one host thread per device; a host batch is
 * cut into contiguous instance ranges balanced by votes (the
 * instances are independent, so there is no collective on the data path), each
 * range is copied to its device, tallied by agnes_tally and copied back.  This is
 * the entry a consumer without torch.distributed binds (a Rust node, a C++
 * service); agnes_amd/dist.py is the Python one-process-per-GPU equivalent.
 *
 * The device side of a range: the vote columns of votes [off[i0], off[i1]), its
 * offsets rebased to 0, and its instance column rebased to the range
 * (instance - i0: the engine's batch contract numbers a batch's instances from 0),
 * by one small kernel after the copy.
 */
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "agnes_internal.h"

namespace agnes {
namespace multi {

__global__ __launch_bounds__(256) void rebase_kernel(uint32_t* inst, uint64_t n, uint32_t base) {
    for (uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x; j < n; j += (uint64_t)gridDim.x * 256u)
        inst[j] -= base; /* (wraps for a vote naming an instance outside the range: still INVALID) */
}

/* device buffers of one range, grown as needed */
struct Bufs {
    uint32_t *inst = nullptr, *value = nullptr, *val = nullptr, *iset = nullptr;
    uint8_t *round = nullptr, *type = nullptr, *codes = nullptr;
    uint64_t* off = nullptr;
    int64_t* weight = nullptr;
    agnes_state* states = nullptr;
    uint64_t votes = 0, insts = 0;
};

struct Dev {
    int device = 0;
    agnes_ctx* ctx = nullptr;
    hipStream_t st = nullptr;
    Bufs b;
};

} // namespace multi
} // namespace agnes

struct agnes_multi {
    std::vector<agnes::multi::Dev> dev;
    uint32_t n_sets = 0; /* of the uploaded power table */
};

namespace {

using agnes::multi::Bufs;
using agnes::multi::Dev;

void free_bufs(Bufs& b) {
    void* ps[] = {b.inst, b.value, b.val, b.iset, b.round, b.type, b.codes, b.off, b.weight, b.states};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    b = Bufs{};
}

int status(hipError_t e) {
    if (e == hipSuccess) return AGNES_OK;
    if (e == hipErrorOutOfMemory) return AGNES_E_NOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return AGNES_E_NODEVICE;
    return AGNES_E_DEVICE;
}

#define MTRY(expr)                                   \
    do {                                             \
        const hipError_t e_ = (expr);                \
        if (e_ != hipSuccess) return status(e_);     \
    } while (0)

int grow(Bufs& b, uint64_t votes, uint64_t insts) {
    if (votes <= b.votes && insts <= b.insts && b.inst) return AGNES_OK;
    free_bufs(b);
    const uint64_t v = votes ? votes : 1, m = insts ? insts : 1;
    MTRY(hipMalloc(&b.inst, 4 * v));
    MTRY(hipMalloc(&b.value, 4 * v));
    MTRY(hipMalloc(&b.val, 4 * v));
    MTRY(hipMalloc(&b.round, v));
    MTRY(hipMalloc(&b.type, v));
    MTRY(hipMalloc(&b.codes, v));
    MTRY(hipMalloc(&b.weight, 8 * v));
    MTRY(hipMalloc(&b.off, 8 * (m + 1)));
    MTRY(hipMalloc(&b.iset, 4 * m));
    MTRY(hipMalloc(&b.states, sizeof(agnes_state) * m));
    b.votes = v;
    b.insts = m;
    return AGNES_OK;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

/* one device's range [i0, i1) of the host batch */
int run_range(Dev& d, uint32_t n_sets, const agnes_config* cfg, const agnes_vote_batch* hb, uint32_t i0, uint32_t i1,
              uint8_t* codes, agnes_state* states, agnes_multi_stats* out) {
    MTRY(hipSetDevice(d.device));
    const uint32_t m = i1 - i0;
    const uint64_t v0 = hb->offsets[i0], v1 = hb->offsets[i1], nv = v1 - v0;
    const bool sm = (cfg->flags & AGNES_FLAG_STATE_MACHINE) && states;
    int rc = grow(d.b, nv, m);
    if (rc != AGNES_OK) return rc;
    std::vector<uint64_t> off(m + 1);
    for (uint32_t k = 0; k <= m; ++k) off[k] = hb->offsets[i0 + k] - v0;
    const auto t0 = std::chrono::steady_clock::now();
    if (nv) {
        MTRY(hipMemcpyAsync(d.b.inst, hb->instance + v0, 4 * nv, hipMemcpyHostToDevice, d.st));
        MTRY(hipMemcpyAsync(d.b.round, hb->round + v0, nv, hipMemcpyHostToDevice, d.st));
        MTRY(hipMemcpyAsync(d.b.type, hb->type + v0, nv, hipMemcpyHostToDevice, d.st));
        MTRY(hipMemcpyAsync(d.b.value, hb->value + v0, 4 * nv, hipMemcpyHostToDevice, d.st));
        if (hb->validator) MTRY(hipMemcpyAsync(d.b.val, hb->validator + v0, 4 * nv, hipMemcpyHostToDevice, d.st));
        if (hb->weight) MTRY(hipMemcpyAsync(d.b.weight, hb->weight + v0, 8 * nv, hipMemcpyHostToDevice, d.st));
    }
    MTRY(hipMemcpyAsync(d.b.off, off.data(), 8 * (m + 1), hipMemcpyHostToDevice, d.st));
    if (hb->instance_set) MTRY(hipMemcpyAsync(d.b.iset, hb->instance_set + i0, 4 * m, hipMemcpyHostToDevice, d.st));
    if (sm) MTRY(hipMemcpyAsync(d.b.states, states + i0, sizeof(agnes_state) * m, hipMemcpyHostToDevice, d.st));
    if (nv && i0) {
        const uint64_t blocks = (nv + 255u) / 256u;
        hipLaunchKernelGGL(agnes::multi::rebase_kernel, dim3((uint32_t)(blocks < 2048u ? blocks : 2048u)), dim3(256),
                           0, d.st, d.b.inst, nv, i0);
        MTRY(hipGetLastError());
    }
    MTRY(hipStreamSynchronize(d.st));
    const double h2d = ms_since(t0);
    agnes_vote_batch db{};
    db.instance = d.b.inst;
    db.round = d.b.round;
    db.type = d.b.type;
    db.value = d.b.value;
    db.validator = hb->validator ? d.b.val : nullptr;
    db.offsets = d.b.off;
    db.instance_set = hb->instance_set ? d.b.iset : nullptr;
    db.weight = hb->weight ? d.b.weight : nullptr;
    db.n_votes = nv;
    db.n_instances = m;
    /* the range's instance sets: the default (instance % n_sets) counts from the
     * batch's instance 0, so a rebased range passes its sets explicitly */
    std::vector<uint32_t> sets;
    if (!hb->instance_set && i0 && n_sets > 1 && m) {
        sets.resize(m);
        for (uint32_t k = 0; k < m; ++k) sets[k] = (i0 + k) % n_sets;
        MTRY(hipMemcpyAsync(d.b.iset, sets.data(), 4 * m, hipMemcpyHostToDevice, d.st));
        db.instance_set = d.b.iset;
    }
    const auto t1 = std::chrono::steady_clock::now();
    rc = agnes_tally(d.ctx, cfg, &db, d.b.codes, sm ? d.b.states : nullptr, d.st);
    if (rc != AGNES_OK) return rc;
    uint64_t bad = 0;
    rc = agnes_last_error_count(d.ctx, &bad); /* synchronises the stream */
    if (rc != AGNES_OK) return rc;
    const double tally = ms_since(t1);
    const auto t2 = std::chrono::steady_clock::now();
    if (nv) MTRY(hipMemcpyAsync(codes + v0, d.b.codes, nv, hipMemcpyDeviceToHost, d.st));
    if (sm) MTRY(hipMemcpyAsync(states + i0, d.b.states, sizeof(agnes_state) * m, hipMemcpyDeviceToHost, d.st));
    MTRY(hipStreamSynchronize(d.st));
    if (out) {
        out->i0 = i0;
        out->i1 = i1;
        out->device = d.device;
        out->n_votes = nv;
        out->n_invalid = bad;
        out->h2d_ms = h2d;
        out->tally_ms = tally;
        out->d2h_ms = ms_since(t2);
    }
    return AGNES_OK;
}

} // namespace

extern "C" {

int agnes_multi_create(const int* devices, uint32_t n_devices, agnes_multi** out) {
    if (!devices || !n_devices || !out) return AGNES_E_INVALID;
    *out = nullptr;
    agnes_multi* m = new (std::nothrow) agnes_multi();
    if (!m) return AGNES_E_NOMEM;
    m->dev.resize(n_devices);
    for (uint32_t k = 0; k < n_devices; ++k) {
        Dev& d = m->dev[k];
        d.device = devices[k];
        int rc = agnes_ctx_create(d.device, &d.ctx);
        if (rc == AGNES_OK && hipSetDevice(d.device) != hipSuccess) rc = AGNES_E_NODEVICE;
        if (rc == AGNES_OK && hipStreamCreateWithFlags(&d.st, hipStreamNonBlocking) != hipSuccess) rc = AGNES_E_DEVICE;
        if (rc != AGNES_OK) {
            agnes_multi_destroy(m);
            return rc;
        }
    }
    *out = m;
    return AGNES_OK;
}

void agnes_multi_destroy(agnes_multi* m) {
    if (!m) return;
    for (Dev& d : m->dev) {
        if (hipSetDevice(d.device) == hipSuccess) {
            if (d.st) (void)hipStreamSynchronize(d.st);
            free_bufs(d.b);
            if (d.st) (void)hipStreamDestroy(d.st);
        }
        if (d.ctx) agnes_ctx_destroy(d.ctx);
    }
    delete m;
}

int agnes_multi_upload_power(agnes_multi* m, const int64_t* power, uint32_t n_sets, uint32_t n_vals,
                             const int64_t* totals) {
    if (!m) return AGNES_E_INVALID;
    for (Dev& d : m->dev) {
        const int rc = agnes_upload_power(d.ctx, power, n_sets, n_vals, totals);
        if (rc != AGNES_OK) return rc;
    }
    m->n_sets = n_sets;
    return AGNES_OK;
}

int agnes_multi_tally(agnes_multi* m, const agnes_config* cfg, const agnes_vote_batch* hb, uint8_t* codes,
                      agnes_state* states, agnes_multi_stats* stats) {
    if (!m || !cfg || !hb || !hb->offsets) return AGNES_E_INVALID;
    if (hb->n_votes && (!codes || !hb->instance || !hb->round || !hb->type || !hb->value ||
                        (!hb->validator && !hb->weight)))
        return AGNES_E_INVALID;
    const uint32_t n = hb->n_instances, D = (uint32_t)m->dev.size();
    if (hb->offsets[n] > hb->n_votes) return AGNES_E_INVALID;
    for (uint32_t i = 0; i < n; ++i)
        if (hb->offsets[i + 1] < hb->offsets[i]) return AGNES_E_INVALID;
    /* contiguous ranges with ~equal votes */
    std::vector<uint32_t> cut(D + 1, n);
    cut[0] = 0;
    const uint64_t total = hb->offsets[n] - hb->offsets[0];
    uint32_t cur = 0;
    for (uint32_t k = 1; k < D; ++k) {
        const uint64_t target = hb->offsets[0] + total * k / D;
        while (cur < n && hb->offsets[cur] < target) ++cur;
        cut[k] = cur;
    }
    std::vector<int> rc(D, AGNES_OK);
    std::vector<std::thread> th;
    th.reserve(D);
    for (uint32_t k = 0; k < D; ++k)
        th.emplace_back([&, k]() {
            rc[k] = run_range(m->dev[k], m->n_sets, cfg, hb, cut[k], cut[k + 1], codes, states,
                              stats ? stats + k : nullptr);
        });
    for (auto& t : th) t.join();
    for (int r : rc)
        if (r != AGNES_OK) return r;
    return AGNES_OK;
}

} // extern "C"
