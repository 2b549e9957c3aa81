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
 *
 * C5 (agnes_multi_tally_one): ONE instance's stream cut into consecutive slices, one
 * per device in device order -- the path's one real exchange step (SURVEY.md
 * §8(e)).  A vote's event needs the exact running sums before it (round_votes.rs:
 * 48-67, driven per vote by vote_executor.rs:20-23), so every device tallies its
 * slice twice around an exchange of the slice totals (the agnes_amd/dist.py
 * tally_one_instance protocol, natively): pass A partials -> ALL-GATHER of the
 * slice totals -> the fold of the slices before each device -> pass B.  DEDUP adds an
 * ALL-REDUCE(MIN) of the first-vote table before the tally, the State machine an
 * ALL-REDUCE(MIN) of the P1 / C positions and an ALL-REDUCE(MAX) of the valid
 * candidate / decision round.  The exchanges run over RCCL (ncclCommInitAll over
 * the devices, one communicator rank per device: xGMI between MI355X GPUs) when
 * the devices are distinct, else through pinned host memory (several contexts on
 * one GPU, the single-GPU tests).
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
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
    uint64_t* eoff = nullptr; /* the range's edge offsets (agnes_multi_edge_offsets) */
    uint64_t etotal = 0;
    uint64_t v0 = 0; /* the range's first vote in the last agnes_multi_tally's batch */
};

/* a reusable barrier of the driver's host threads (one per device) */
struct Barrier {
    std::mutex mu;
    std::condition_variable cv;
    uint32_t n = 0, arrived = 0;
    uint64_t gen = 0;
    void wait() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};

} // namespace multi
} // namespace agnes

struct agnes_multi {
    std::vector<agnes::multi::Dev> dev;
    uint32_t n_sets = 0; /* of the uploaded power table */
    uint32_t n_vals = 0;
    uint32_t xmode = AGNES_MULTI_EXCHANGE_AUTO;
    std::vector<ncclComm_t> comms; /* one rank per device (RCCL exchanges), created on first use */
    std::atomic<bool> comms_dead{false}; /* a collective failed on some rank: aborted (handles null), rebuilt next call */
    std::atomic<uint32_t> rccl_checked{0u}; /* bit op: the first RCCL collective of that kind was checked */
    std::atomic<bool> rccl_bad{false};      /* ... and differed: the host exchange from then on */
    std::atomic<bool> used_rccl{false};     /* the last call's exchanges went through RCCL */
    uint32_t test_corrupt = 0;              /* test hook (agnes_multi_test_corrupt): bit op flips a result */
    std::vector<int> xerr;         /* per device: its status entering an RCCL exchange (host agreement) */
    agnes::multi::Barrier bar;
    std::vector<unsigned char*> stage; /* pinned host staging of the host exchange, per device */
    std::vector<uint64_t> stage_cap;
    /* the last agnes_multi_tally's ranges (for agnes_multi_edge_offsets / _edges) */
    std::vector<uint32_t> cut;
    bool have_ranges = false;
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
    d.v0 = v0;
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

/* ---- the exchanges of a split instance (C5) ---------------------------------------
 * One call per device thread, every thread the same call in the same order.  RCCL:
 * one collective on the device's communicator rank (stream-ordered, xGMI between
 * distinct MI355X).  Host: each thread stages its buffer in pinned memory, a barrier,
 * the reduction (each thread combines a contiguous part of the elements), a barrier,
 * each thread copies the result back. */
enum XOp { X_MIN_U64, X_MIN_I64, X_MAX_I64, X_GATHER };

int stage_grow(agnes_multi* m, uint32_t d, uint64_t bytes) {
    if (m->stage_cap[d] >= bytes) return AGNES_OK;
    if (m->stage[d]) (void)hipHostFree(m->stage[d]);
    m->stage[d] = nullptr;
    m->stage_cap[d] = 0;
    MTRY(hipHostMalloc(reinterpret_cast<void**>(&m->stage[d]), bytes, hipHostMallocDefault));
    m->stage_cap[d] = bytes;
    return AGNES_OK;
}

/* in place on the device (count int64 / u64 elements); X_GATHER: count elements per
 * device from send into recv (D * count, device order).  Every thread reaches every
 * barrier, also after an error (it then reports the error). */
/* RCCL: the device threads agree on every status before and after a collective is
 * enqueued.  A thread that has already failed (a hipMalloc, a launch) never issues a
 * collective on its unfilled buffers, and nor does any other thread -- their matching
 * collectives would wait forever; a collective one rank could not enqueue aborts every
 * communicator (the others' enqueued halves are cancelled), and the next call rebuilds
 * them.  `mine` is the calling thread's status so far. */
bool agree_ok(agnes_multi* m, uint32_t d, int mine) {
    m->xerr[d] = mine;
    m->bar.wait();
    bool ok = true;
    for (int e : m->xerr) ok = ok && e == AGNES_OK;
    m->bar.wait(); /* every thread has read xerr before it is written again */
    return ok;
}

/* The host exchange's result for op over every device's staged send buffer (8-B
 * elements; X_GATHER: the D buffers in device order). */
void host_result(const agnes_multi* m, XOp op, uint64_t count, uint64_t* out) {
    const uint32_t D = (uint32_t)m->dev.size();
    if (op == X_GATHER) {
        for (uint32_t k = 0; k < D; ++k) std::memcpy(out + (size_t)k * count, m->stage[k], 8u * count);
        return;
    }
    for (uint64_t e = 0; e < count; ++e) {
        uint64_t acc = reinterpret_cast<const uint64_t*>(m->stage[0])[e];
        for (uint32_t k = 1; k < D; ++k) {
            const uint64_t x = reinterpret_cast<const uint64_t*>(m->stage[k])[e];
            if (op == X_MIN_U64) acc = x < acc ? x : acc;
            else if (op == X_MIN_I64) acc = (int64_t)x < (int64_t)acc ? x : acc;
            else acc = (int64_t)x > (int64_t)acc ? x : acc;
        }
        out[e] = acc;
    }
}

/* The first RCCL collective of each kind (the all-gather, the MIN all-reduces on u64
 * and i64, the MAX one) of a handle is checked against the host exchange of the same
 * data: the multi-device RCCL path has not run on hardware in this repository's tests,
 * which share one device.  Before the collective every thread stages its send buffer
 * in pinned memory (the all-reduces run in place); after it every thread compares its
 * received elements with the host result.  A mismatch anywhere makes every thread take
 * the host result, and the handle use the host exchange from then on; the fallback is
 * reported in agnes_multi_stats.exchange (AGNES_MULTI_X_FALLBACK). */
int stage_send(agnes_multi* m, uint32_t d, const int64_t* send, uint64_t count) {
    Dev& dv = m->dev[d];
    int rc = stage_grow(m, d, 8u * count);
    if (rc == AGNES_OK && hipMemcpyAsync(m->stage[d], send, 8u * count, hipMemcpyDeviceToHost, dv.st) != hipSuccess)
        rc = AGNES_E_DEVICE;
    if (rc == AGNES_OK && hipStreamSynchronize(dv.st) != hipSuccess) rc = AGNES_E_DEVICE;
    return rc;
}

int check_collective(agnes_multi* m, uint32_t d, XOp op, int64_t* recv, uint64_t count) {
    Dev& dv = m->dev[d];
    const uint32_t D = (uint32_t)m->dev.size();
    const uint64_t n = op == X_GATHER ? (uint64_t)D * count : count;
    std::vector<uint64_t> want((size_t)n), got((size_t)n);
    int rc = AGNES_OK;
    if (m->test_corrupt & (0x11u << op)) { /* test hook: one received element flipped */
        if (hipMemsetAsync(recv, 0x5A, 1, dv.st) != hipSuccess) rc = AGNES_E_DEVICE;
    }
    if (rc == AGNES_OK && hipMemcpyAsync(got.data(), recv, 8u * n, hipMemcpyDeviceToHost, dv.st) != hipSuccess)
        rc = AGNES_E_DEVICE;
    if (rc == AGNES_OK && hipStreamSynchronize(dv.st) != hipSuccess) rc = AGNES_E_DEVICE;
    host_result(m, op, count, want.data());
    const bool same = rc == AGNES_OK && std::memcmp(want.data(), got.data(), 8u * n) == 0;
    const bool all_same = agree_ok(m, d, same ? AGNES_OK : AGNES_E_DEVICE);
    if (!all_same && rc == AGNES_OK) {
        if (hipMemcpyAsync(recv, want.data(), 8u * n, hipMemcpyHostToDevice, dv.st) != hipSuccess) rc = AGNES_E_DEVICE;
        if (rc == AGNES_OK && hipStreamSynchronize(dv.st) != hipSuccess) rc = AGNES_E_DEVICE;
    }
    m->bar.wait(); /* every thread has compared: the stages are free again */
    if (d == 0u) {
        if (!all_same) m->rccl_bad = true;
        m->rccl_checked |= 1u << op;
    }
    m->bar.wait(); /* every thread sees the same flags from here on */
    return rc;
}

int exchange(agnes_multi* m, uint32_t d, XOp op, const int64_t* send, int64_t* recv, uint64_t count, int mine) {
    Dev& dv = m->dev[d];
    const uint32_t D = (uint32_t)m->dev.size();
    /* once a self-check has failed (rccl_bad, published between two barriers, so every
     * thread sees the same value) the call's later collectives take the host exchange too */
    if (!m->comms.empty() && !m->rccl_bad) {
        const bool check = !(m->rccl_checked & (1u << op));
        if (check && mine == AGNES_OK) mine = stage_send(m, d, send, count);
        if (!agree_ok(m, d, mine)) return mine != AGNES_OK ? mine : AGNES_E_DEVICE;
        ncclResult_t r;
        if (op == X_GATHER)
            r = ncclAllGather(send, recv, count, ncclInt64, m->comms[d], dv.st);
        else
            r = ncclAllReduce(send, recv, count, op == X_MIN_U64 ? ncclUint64 : ncclInt64,
                              op == X_MAX_I64 ? ncclMax : ncclMin, m->comms[d], dv.st);
        const int rc = r == ncclSuccess ? AGNES_OK : AGNES_E_DEVICE;
        if (!agree_ok(m, d, rc)) {
            /* every rank aborts its own communicator; the handles are dropped (the next
             * call rebuilds them) so that nothing destroys an aborted one again */
            (void)ncclCommAbort(m->comms[d]);
            m->comms[d] = nullptr;
            if (d == 0u) m->comms_dead = true;
            return AGNES_E_DEVICE;
        }
        m->used_rccl = true;
        if (check) return check_collective(m, d, op, recv, count);
        if (m->test_corrupt & (0x10u << op)) { /* test hook: an RCCL that is really broken */
            if (hipMemsetAsync(recv, 0x5A, 1, dv.st) != hipSuccess || hipStreamSynchronize(dv.st) != hipSuccess)
                return AGNES_E_DEVICE;
        }
        return AGNES_OK;
    }
    const uint64_t bytes = 8u * count;
    int rc = mine != AGNES_OK ? mine : stage_grow(m, d, bytes);
    if (rc == AGNES_OK && hipMemcpyAsync(m->stage[d], send, bytes, hipMemcpyDeviceToHost, dv.st) != hipSuccess)
        rc = AGNES_E_DEVICE;
    if (rc == AGNES_OK && hipStreamSynchronize(dv.st) != hipSuccess) rc = AGNES_E_DEVICE;
    m->bar.wait(); /* every stage written */
    for (uint32_t k = 0; k < D; ++k) /* a device whose staging failed leaves a hole: all fail */
        if (m->stage_cap[k] < bytes) rc = rc == AGNES_OK ? AGNES_E_DEVICE : rc;
    if (op == X_GATHER) {
        for (uint32_t k = 0; k < D && rc == AGNES_OK; ++k)
            if (hipMemcpyAsync(recv + k * count, m->stage[k], bytes, hipMemcpyHostToDevice, dv.st) != hipSuccess)
                rc = AGNES_E_DEVICE;
        if (rc == AGNES_OK && hipStreamSynchronize(dv.st) != hipSuccess) rc = AGNES_E_DEVICE;
        m->bar.wait(); /* the stages are free again */
        return rc;
    }
    if (rc == AGNES_OK) { /* this thread combines elements [e0, e1) of every stage into stage 0 */
        const uint64_t e0 = count * d / D, e1 = count * (d + 1) / D;
        for (uint64_t e = e0; e < e1; ++e) {
            uint64_t acc = reinterpret_cast<const uint64_t*>(m->stage[0])[e];
            for (uint32_t k = 1; k < D; ++k) {
                const uint64_t x = reinterpret_cast<const uint64_t*>(m->stage[k])[e];
                if (op == X_MIN_U64) acc = x < acc ? x : acc;
                else if (op == X_MIN_I64) acc = (int64_t)x < (int64_t)acc ? x : acc;
                else acc = (int64_t)x > (int64_t)acc ? x : acc;
            }
            reinterpret_cast<uint64_t*>(m->stage[0])[e] = acc;
        }
    }
    m->bar.wait(); /* stage 0 complete */
    if (rc == AGNES_OK && hipMemcpyAsync(recv, m->stage[0], bytes, hipMemcpyHostToDevice, dv.st) != hipSuccess)
        rc = AGNES_E_DEVICE;
    if (rc == AGNES_OK && hipStreamSynchronize(dv.st) != hipSuccess) rc = AGNES_E_DEVICE;
    m->bar.wait(); /* the stages are free again */
    return rc;
}

/* device buffers of a split-instance call */
struct OneBufs {
    uint32_t *inst = nullptr, *value = nullptr, *val = nullptr;
    uint8_t *round = nullptr, *type = nullptr, *tmask = nullptr, *codes = nullptr;
    uint64_t *segoff = nullptr, *first = nullptr, *off1 = nullptr;
    agnes_vote_count *counts = nullptr, *mine = nullptr, *ranks = nullptr, *fin = nullptr;
    agnes_state* state = nullptr;
    int64_t *marks = nullptr, *weights = nullptr;
    void release() {
        void* ps[] = {inst, value, val, round, type, tmask, codes, segoff, first, off1,
                      counts, mine, ranks, fin, state, marks, weights};
        for (void* p : ps)
            if (p) (void)hipFree(p);
        *this = OneBufs{};
    }
};

/* device d's slice [lo, hi) of the one instance.  Every thread runs the same sequence
 * of exchanges: a device that failed still takes part in them (so that no thread
 * waits forever) and reports its first error. */
int run_one(agnes_multi* m, uint32_t d, const agnes_config* cfg, const agnes_vote_batch* hb, uint64_t lo,
            uint64_t hi, uint32_t spd, uint8_t* codes, agnes_state* state, agnes_vote_count* counts_out,
            agnes_multi_stats* out) {
    Dev& dv = m->dev[d];
    const uint32_t D = (uint32_t)m->dev.size();
    const uint32_t R = cfg->max_rounds, K = 2u * R;
    const bool dedup = cfg->mode == AGNES_MODE_DEDUP;
    const bool sm = (cfg->flags & AGNES_FLAG_STATE_MACHINE) && state;
    const uint64_t nv = hi - lo;
    OneBufs b;
    int rc = AGNES_OK;
#define OTRY(expr)                                          \
    do {                                                    \
        if (rc == AGNES_OK) {                               \
            const hipError_t e_ = (expr);                   \
            if (e_ != hipSuccess) rc = status(e_);          \
        }                                                   \
    } while (0)
#define OCALL(expr)                                         \
    do {                                                    \
        if (rc == AGNES_OK) {                               \
            const int r_ = (expr);                          \
            if (r_ != AGNES_OK) rc = r_;                    \
        }                                                   \
    } while (0)
#define OXCH(expr)                                          \
    do {                                                    \
        const int r_ = (expr); /* (always: every thread) */ \
        if (rc == AGNES_OK && r_ != AGNES_OK) rc = r_;      \
    } while (0)
    OTRY(hipSetDevice(dv.device));
    const uint64_t v = nv ? nv : 4u;
    uint32_t S = spd ? spd : 2048u;
    if ((uint64_t)S > (nv + 3u) / 4u) S = (uint32_t)((nv + 3u) / 4u);
    if (S == 0u) S = 1u;
    OTRY(hipMalloc(&b.inst, 4 * v));
    OTRY(hipMalloc(&b.value, 4 * v));
    OTRY(hipMalloc(&b.val, 4 * v));
    OTRY(hipMalloc(&b.round, v));
    OTRY(hipMalloc(&b.type, v));
    OTRY(hipMalloc(&b.codes, v));
    OTRY(hipMalloc(&b.weights, 8 * v));
    OTRY(hipMalloc(&b.segoff, 8 * ((uint64_t)S + 1u)));
    OTRY(hipMalloc(&b.off1, 16));
    OTRY(hipMalloc(&b.counts, sizeof(agnes_vote_count) * (uint64_t)S * K));
    OTRY(hipMalloc(&b.mine, sizeof(agnes_vote_count) * K));
    OTRY(hipMalloc(&b.ranks, sizeof(agnes_vote_count) * K * D));
    OTRY(hipMalloc(&b.fin, sizeof(agnes_vote_count) * K));
    if (dedup) {
        OTRY(hipMalloc(&b.tmask, v));
        OTRY(hipMalloc(&b.first, 8ull * K * m->n_vals));
    }
    if (sm) {
        OTRY(hipMalloc(&b.state, sizeof(agnes_state)));
        OTRY(hipMalloc(&b.marks, 4 * sizeof(int64_t)));
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (nv) {
        OTRY(hipMemcpyAsync(b.inst, hb->instance + lo, 4 * nv, hipMemcpyHostToDevice, dv.st));
        OTRY(hipMemcpyAsync(b.round, hb->round + lo, nv, hipMemcpyHostToDevice, dv.st));
        OTRY(hipMemcpyAsync(b.type, hb->type + lo, nv, hipMemcpyHostToDevice, dv.st));
        OTRY(hipMemcpyAsync(b.value, hb->value + lo, 4 * nv, hipMemcpyHostToDevice, dv.st));
        OTRY(hipMemcpyAsync(b.val, hb->validator + lo, 4 * nv, hipMemcpyHostToDevice, dv.st));
    }
    /* the slice's segments: balanced, multiples of 4 votes (one wave each) */
    std::vector<uint64_t> so((size_t)S + 1u);
    for (uint32_t k = 0; k <= S; ++k) so[k] = ((uint64_t)k * nv / S) / 4u * 4u;
    so[S] = nv;
    const uint64_t off1[2] = {0, nv};
    OTRY(hipMemcpyAsync(b.segoff, so.data(), 8 * ((uint64_t)S + 1u), hipMemcpyHostToDevice, dv.st));
    OTRY(hipMemcpyAsync(b.off1, off1, 16, hipMemcpyHostToDevice, dv.st));
    if (sm) OTRY(hipMemcpyAsync(b.state, state, sizeof(agnes_state), hipMemcpyHostToDevice, dv.st));
    OTRY(hipStreamSynchronize(dv.st));
    const double h2d = ms_since(t0);
    const auto t1 = std::chrono::steady_clock::now();

    agnes_vote_batch sl{}; /* the slice as one batch (the DEDUP and State-machine passes) */
    sl.instance = b.inst;
    sl.round = b.round;
    sl.type = b.type;
    sl.value = b.value;
    sl.validator = b.val;
    sl.offsets = b.off1;
    sl.n_votes = nv;
    sl.n_instances = 1;
    /* the carried tally: REFERENCE over the (masked) slice, no State machine */
    const agnes_config one{AGNES_MODE_REFERENCE, (cfg->flags & ~AGNES_FLAG_STATE_MACHINE) | AGNES_FLAG_ONE_INSTANCE,
                           R, 0u};
    agnes_config scfg = *cfg; /* the State-machine passes: instance id 0 */
    scfg.reserved = 0u;
    agnes_config dcfg = scfg; /* the DEDUP passes */
    dcfg.flags &= ~AGNES_FLAG_STATE_MACHINE;
    agnes_vote_batch seg = sl; /* the slice cut into segments (the carried tally) */
    seg.offsets = b.segoff;
    seg.n_instances = S;
    if (dedup) { /* the first vote of every (round, type, validator) over all slices */
        OTRY(hipMemsetAsync(b.first, 0xFF, 8ull * K * m->n_vals, dv.st));
        OCALL(agnes_dedup_first(dv.ctx, &dcfg, &sl, lo, b.first, dv.st));
        OTRY(hipStreamSynchronize(dv.st));
        OXCH(exchange(m, d, X_MIN_U64, reinterpret_cast<const int64_t*>(b.first), reinterpret_cast<int64_t*>(b.first),
                      (uint64_t)K * m->n_vals, rc));
        OCALL(agnes_dedup_mask(dv.ctx, &dcfg, &sl, lo, b.first, b.tmask, dv.st));
        seg.type = b.tmask;
    }
    /* pass A: every segment from RoundVotes::new -> its partial (one reduction, which
     * keeps the votes' weights for pass B); this slice's total */
    OCALL(agnes_tally_partials(dv.ctx, &one, &seg, b.counts, b.weights, dv.st));
    OCALL(agnes_fold_counts(dv.ctx, b.counts, S, K, nullptr, b.mine, 0u, dv.st));
    OTRY(hipStreamSynchronize(dv.st));
    /* the exchange: every slice's total to every device */
    OXCH(exchange(m, d, X_GATHER, reinterpret_cast<const int64_t*>(b.mine), reinterpret_cast<int64_t*>(b.ranks),
                  3ull * K, rc));
    /* the slices before each device, then before each segment: pass B's carry-ins */
    OCALL(agnes_fold_counts(dv.ctx, b.ranks, D, K, nullptr, b.fin,
                            AGNES_FOLD_APPLY | AGNES_FOLD_CARRY_ZERO_NONE | AGNES_FOLD_TOTAL_ZERO_LABELS, dv.st));
    OCALL(agnes_fold_counts(dv.ctx, b.counts, S, K, b.ranks + (uint64_t)d * K, nullptr,
                            AGNES_FOLD_APPLY | AGNES_FOLD_ZERO_LABELS, dv.st));
    /* pass B: the exact rescan from the carry-ins, over the cached weights */
    agnes_config oneb = one;
    oneb.flags |= AGNES_FLAG_WEIGHTS_CACHED;
    agnes_vote_batch segb = seg;
    segb.weight = b.weights;
    OCALL(agnes_tally_carried(dv.ctx, &oneb, &segb, b.codes, b.counts, dv.st));
    if (dedup) OCALL(agnes_dedup_reject(dv.ctx, b.tmask, nv, b.codes, dv.st));
    if (sm) { /* P1 / C: MIN over slices; valid, decision round: MAX; the State */
        const int64_t init[4] = {INT64_MAX, INT64_MAX, 0, 0};
        OTRY(hipMemcpyAsync(b.marks, init, sizeof(init), hipMemcpyHostToDevice, dv.st));
        OCALL(agnes_one_sm_scan(dv.ctx, &scfg, &sl, lo, b.codes, b.state, b.marks, dv.st));
        OTRY(hipStreamSynchronize(dv.st));
        OXCH(exchange(m, d, X_MIN_I64, b.marks, b.marks, 2u, rc));
        OCALL(agnes_one_sm_apply(dv.ctx, &scfg, &sl, lo, b.codes, b.state, b.marks, dv.st));
        OTRY(hipStreamSynchronize(dv.st));
        OXCH(exchange(m, d, X_MAX_I64, b.marks + 2, b.marks + 2, 2u, rc));
        OCALL(agnes_one_sm_finish(dv.ctx, b.marks, b.state, dv.st));
    }
    OTRY(hipStreamSynchronize(dv.st));
    uint64_t bad = 0;
    OCALL(agnes_last_error_count(dv.ctx, &bad));
    const double tally = ms_since(t1);
    const auto t2 = std::chrono::steady_clock::now();
    if (nv) OTRY(hipMemcpyAsync(codes + lo, b.codes, nv, hipMemcpyDeviceToHost, dv.st));
    if (d == 0u) {
        if (counts_out) OTRY(hipMemcpyAsync(counts_out, b.fin, sizeof(agnes_vote_count) * K, hipMemcpyDeviceToHost, dv.st));
        if (sm) OTRY(hipMemcpyAsync(state, b.state, sizeof(agnes_state), hipMemcpyDeviceToHost, dv.st));
    }
    OTRY(hipStreamSynchronize(dv.st));
    if (out) {
        out->device = (uint32_t)dv.device;
        out->i0 = 0;
        out->i1 = 1;
        out->exchange = (m->used_rccl ? AGNES_MULTI_X_RCCL : 0u) | (m->rccl_bad ? AGNES_MULTI_X_FALLBACK : 0u) |
                        (D > 1u && !m->used_rccl ? AGNES_MULTI_X_HOST : 0u);
        out->n_votes = nv;
        out->n_invalid = bad;
        out->h2d_ms = h2d;
        out->tally_ms = tally;
        out->d2h_ms = ms_since(t2);
    }
    (void)hipStreamSynchronize(dv.st);
    b.release();
#undef OTRY
#undef OCALL
#undef OXCH
    return rc;
}

int ensure_exchange(agnes_multi* m) {
    const uint32_t D = (uint32_t)m->dev.size();
    if (m->stage.size() != D) {
        m->stage.assign(D, nullptr);
        m->stage_cap.assign(D, 0);
    }
    m->bar.n = D;
    m->xerr.assign(D, AGNES_OK);
    m->used_rccl = false;
    if (m->comms_dead) { /* a collective failed in an earlier call: its communicators were aborted */
        for (ncclComm_t c : m->comms)
            if (c) (void)ncclCommDestroy(c);
        m->comms.clear();
        m->comms_dead = false;
    }
    bool distinct = true;
    for (uint32_t i = 0; i < D; ++i)
        for (uint32_t j = i + 1; j < D; ++j)
            if (m->dev[i].device == m->dev[j].device) distinct = false;
    const bool want = !m->rccl_bad && (m->xmode == AGNES_MULTI_EXCHANGE_RCCL ||
                                       (m->xmode == AGNES_MULTI_EXCHANGE_AUTO && distinct && D > 1));
    if (!want) {
        for (ncclComm_t c : m->comms)
            if (c) (void)ncclCommDestroy(c);
        m->comms.clear();
        return AGNES_OK;
    }
    if (!distinct) return AGNES_E_UNSUPPORTED; /* RCCL: one communicator rank per device */
    if (m->comms.size() == D) return AGNES_OK;
    std::vector<int> devs(D);
    for (uint32_t k = 0; k < D; ++k) devs[k] = m->dev[k].device;
    m->comms.assign(D, nullptr);
    if (ncclCommInitAll(m->comms.data(), (int)D, devs.data()) != ncclSuccess) {
        m->comms.clear();
        return AGNES_E_DEVICE;
    }
    return AGNES_OK;
}

/* the device batch of range k of the last agnes_multi_tally */
agnes_vote_batch range_batch(const agnes_multi* m, uint32_t k, uint64_t nv) {
    const Dev& d = m->dev[k];
    agnes_vote_batch db{};
    db.instance = d.b.inst;
    db.round = d.b.round;
    db.type = d.b.type;
    db.value = d.b.value;
    db.validator = d.b.val;
    db.offsets = d.b.off;
    db.n_instances = m->cut[k + 1] - m->cut[k];
    db.n_votes = nv;
    return db;
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
            if (d.eoff) (void)hipFree(d.eoff);
            if (d.st) (void)hipStreamDestroy(d.st);
        }
        if (d.ctx) agnes_ctx_destroy(d.ctx);
    }
    for (ncclComm_t c : m->comms)
        if (c) (void)ncclCommDestroy(c);
    for (unsigned char* p : m->stage)
        if (p) (void)hipHostFree(p);
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
    m->n_vals = n_vals;
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
    m->have_ranges = false;
    for (uint32_t k = 0; k < D; ++k)
        th.emplace_back([&, k]() {
            rc[k] = run_range(m->dev[k], m->n_sets, cfg, hb, cut[k], cut[k + 1], codes, states,
                              stats ? stats + k : nullptr);
        });
    for (auto& t : th) t.join();
    for (int r : rc)
        if (r != AGNES_OK) return r;
    m->cut = cut;
    m->have_ranges = true;
    return AGNES_OK;
}


int agnes_multi_exchange(agnes_multi* m, uint32_t mode) {
    if (!m || mode > AGNES_MULTI_EXCHANGE_RCCL) return AGNES_E_INVALID;
    m->xmode = mode;
    return ensure_exchange(m);
}

int agnes_multi_test_corrupt(agnes_multi* m, uint32_t ops) {
    if (!m || ops > 255u) return AGNES_E_INVALID;
    m->test_corrupt = ops;
    m->rccl_checked &= ~(ops & 15u); /* the next collective of each kind in bits 0..3 is checked again */
    return AGNES_OK;
}

int agnes_multi_tally_one(agnes_multi* m, const agnes_config* cfg, const agnes_vote_batch* hb, uint8_t* codes,
                          agnes_state* state, agnes_vote_count* counts, uint32_t segments_per_device,
                          agnes_multi_stats* stats) {
    if (!m || !cfg || !hb || !hb->offsets || hb->n_instances != 1u) return AGNES_E_INVALID;
    if (cfg->max_rounds < 1u || (cfg->mode != AGNES_MODE_REFERENCE && cfg->mode != AGNES_MODE_DEDUP) ||
        (cfg->flags & (AGNES_FLAG_ROUND_SKIP | AGNES_FLAG_ONE_INSTANCE | AGNES_FLAG_DISTINCT_VALUES)))
        return AGNES_E_UNSUPPORTED;
    if (hb->weight || hb->instance_set) return AGNES_E_UNSUPPORTED; /* the power table weighs, set 0 */
    const uint64_t n = hb->offsets[1];
    if (hb->offsets[0] != 0u || n > hb->n_votes) return AGNES_E_INVALID;
    if (n && (!codes || !hb->instance || !hb->round || !hb->type || !hb->value || !hb->validator))
        return AGNES_E_INVALID;
    if (!m->n_vals) return AGNES_E_INVALID; /* no power table */
    if (n > (1ull << 31)) return AGNES_E_UNSUPPORTED;
    const int e = ensure_exchange(m);
    if (e != AGNES_OK) return e;
    const uint32_t D = (uint32_t)m->dev.size();
    std::vector<int> rc(D, AGNES_OK);
    std::vector<std::thread> th;
    th.reserve(D);
    for (uint32_t k = 0; k < D; ++k) {
        /* consecutive slices in device order, boundaries on multiples of 4 votes */
        const uint64_t lo = (n * k / D) / 4u * 4u, hi = k + 1u == D ? n : (n * (k + 1u) / D) / 4u * 4u;
        th.emplace_back([&, k, lo, hi]() {
            rc[k] = run_one(m, k, cfg, hb, lo, hi, segments_per_device, codes, state, counts,
                            stats ? stats + k : nullptr);
        });
    }
    for (auto& t : th) t.join();
    for (int r : rc)
        if (r != AGNES_OK) return r;
    return AGNES_OK;
}

int agnes_multi_edge_offsets(agnes_multi* m, const agnes_config* cfg, uint64_t* offsets) {
    if (!m || !cfg || !offsets) return AGNES_E_INVALID;
    if (!m->have_ranges) return AGNES_E_INVALID; /* no agnes_multi_tally before */
    const uint32_t D = (uint32_t)m->dev.size();
    std::vector<int> rc(D, AGNES_OK);
    std::vector<std::vector<uint64_t>> loc(D);
    std::vector<std::thread> th;
    th.reserve(D);
    for (uint32_t k = 0; k < D; ++k)
        th.emplace_back([&, k]() {
            Dev& d = m->dev[k];
            const uint32_t mi = m->cut[k + 1] - m->cut[k];
            loc[k].assign((size_t)mi + 1u, 0u);
            int r = hipSetDevice(d.device) == hipSuccess ? AGNES_OK : AGNES_E_DEVICE;
            uint64_t nv = 0;
            if (r == AGNES_OK && hipMemcpy(&nv, d.b.off + mi, 8, hipMemcpyDeviceToHost) != hipSuccess) r = AGNES_E_DEVICE;
            if (r == AGNES_OK) {
                if (d.eoff) (void)hipFree(d.eoff);
                d.eoff = nullptr;
                if (hipMalloc(&d.eoff, 8ull * (mi + 1u)) != hipSuccess) r = AGNES_E_NOMEM;
            }
            const agnes_vote_batch db = range_batch(m, k, nv);
            if (r == AGNES_OK) r = agnes_edge_offsets(d.ctx, cfg, &db, d.b.codes, d.eoff, d.st);
            if (r == AGNES_OK && hipMemcpyAsync(loc[k].data(), d.eoff, 8ull * (mi + 1u), hipMemcpyDeviceToHost, d.st) !=
                                     hipSuccess)
                r = AGNES_E_DEVICE;
            if (r == AGNES_OK && hipStreamSynchronize(d.st) != hipSuccess) r = AGNES_E_DEVICE;
            d.etotal = loc[k][mi];
            rc[k] = r;
        });
    for (auto& t : th) t.join();
    for (int r : rc)
        if (r != AGNES_OK) return r;
    uint64_t base = 0; /* the ranges' offsets made global, in range order */
    for (uint32_t k = 0; k < D; ++k) {
        const uint32_t i0 = m->cut[k], mi = m->cut[k + 1] - i0;
        for (uint32_t j = 0; j < mi; ++j) offsets[i0 + j] = base + loc[k][j];
        base += loc[k][mi];
    }
    offsets[m->cut[D]] = base;
    return AGNES_OK;
}

int agnes_multi_edges(agnes_multi* m, const agnes_config* cfg, const uint64_t* offsets, agnes_edge* out) {
    if (!m || !cfg || !offsets) return AGNES_E_INVALID;
    if (!m->have_ranges) return AGNES_E_INVALID;
    const uint32_t D = (uint32_t)m->dev.size();
    for (uint32_t k = 0; k < D; ++k)
        if (!m->dev[k].eoff) return AGNES_E_INVALID; /* agnes_multi_edge_offsets first */
    if (offsets[m->cut[D]] && !out) return AGNES_E_INVALID;
    std::vector<int> rc(D, AGNES_OK);
    std::vector<std::thread> th;
    th.reserve(D);
    for (uint32_t k = 0; k < D; ++k)
        th.emplace_back([&, k]() {
            Dev& d = m->dev[k];
            const uint32_t i0 = m->cut[k], mi = m->cut[k + 1] - i0;
            const uint64_t ne = d.etotal, at = offsets[i0];
            int r = hipSetDevice(d.device) == hipSuccess ? AGNES_OK : AGNES_E_DEVICE;
            uint64_t nv = 0;
            if (r == AGNES_OK && hipMemcpy(&nv, d.b.off + mi, 8, hipMemcpyDeviceToHost) != hipSuccess) r = AGNES_E_DEVICE;
            uint64_t v0 = 0; /* the range's first vote in the host batch: offsets rebased at 0 */
            agnes_edge* dout = nullptr;
            if (r == AGNES_OK && ne && hipMalloc(&dout, sizeof(agnes_edge) * ne) != hipSuccess) r = AGNES_E_NOMEM;
            const agnes_vote_batch db = range_batch(m, k, nv);
            if (r == AGNES_OK && ne) r = agnes_edges(d.ctx, cfg, &db, d.b.codes, d.eoff, dout, ne, d.st);
            if (r == AGNES_OK && ne &&
                hipMemcpyAsync(out + at, dout, sizeof(agnes_edge) * ne, hipMemcpyDeviceToHost, d.st) != hipSuccess)
                r = AGNES_E_DEVICE;
            if (r == AGNES_OK && hipStreamSynchronize(d.st) != hipSuccess) r = AGNES_E_DEVICE;
            if (dout) (void)hipFree(dout);
            v0 = d.v0;
            if (r == AGNES_OK) /* the batch's vote and instance numbering */
                for (uint64_t e = 0; e < ne; ++e) {
                    out[at + e].vote += v0;
                    out[at + e].instance += i0;
                }
            rc[k] = r;
        });
    for (auto& t : th) t.join();
    for (int r : rc)
        if (r != AGNES_OK) return r;
    return AGNES_OK;
}

} // extern "C"
