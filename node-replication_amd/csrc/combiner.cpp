// combiner.cpp — the Replica's flat combining on the host, native.
//
// Reference: nr/src/context.rs:88-194 (a per-thread context of at most MAX_PENDING_OPS = 32
// pending ops and their responses) and nr/src/replica.rs:345-356 (register), :414-433
// (execute_mut: enqueue, then try to combine until the response is there), :508-595
// (try_combine / combine: whoever takes the combiner lock collects every thread's pending ops,
// appends them as ONE batch, replays the log and hands each thread its responses).
//
// Here the batch is one GPU round of the replica: every posted Put of every thread is appended
// and replayed (HashMap::insert, previous-value responses), then every posted Get is answered
// against the post-round state (Replica::read_only after sync-to-tail). Gets posted beside
// Puts are linearised after the round's Puts: all of them are concurrent with it.
//
// A client thread that finds the lock taken waits on its own context (a short spin, then 10-µs
// sleeps: a round takes tens of microseconds, and the host cores are better left to the
// combining thread) until the combiner has filled in its responses, or the lock frees up while
// its ops are still pending, in which case it combines. The combiner owns pinned host staging and device buffers for max_threads * 32
// ops, so a round is two copies in, one round launch, copies out and one stream sync.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "internal.hpp"

namespace {

constexpr uint32_t MAX_PENDING = 32;  // nr/src/context.rs:12 MAX_PENDING_OPS

enum : uint32_t { EMPTY = 0, POSTED = 1, DONE = 2 };

struct alignas(64) Ctx {  // one registered thread's context
    std::atomic<uint32_t> state{EMPTY};
    uint32_t n = 0;
    bool put = false;
    const uint64_t* keys = nullptr;  // the caller's ops (valid while POSTED)
    const uint64_t* vals = nullptr;
    uint64_t* out = nullptr;  // the caller's responses: previous value / value
    uint8_t* flag = nullptr;  //   Some / found
    int rc = NRG_OK;
};

}  // namespace

struct nrg_combiner {
    nrg_ctx* ctx = nullptr;
    uint32_t max_threads = 0;
    std::atomic<uint32_t> next{0};
    Ctx* ctxs = nullptr;
    std::mutex lock;
    uint64_t cap = 0;  // ops per round: max_threads * MAX_PENDING
    // pinned host staging
    nrg_put* h_puts = nullptr;
    uint64_t* h_keys = nullptr;
    uint64_t* h_prev = nullptr;
    uint8_t* h_prevf = nullptr;
    uint64_t* h_vals = nullptr;
    uint8_t* h_found = nullptr;
    // device buffers
    nrg_put* d_puts = nullptr;
    uint64_t* d_keys = nullptr;
    uint64_t* d_prev = nullptr;
    uint8_t* d_prevf = nullptr;
    uint64_t* d_vals = nullptr;
    uint8_t* d_found = nullptr;
    std::vector<uint32_t> batch;  // contexts collected by the current combine
    uint64_t rounds = 0, ops = 0;
};

static void comb_free(nrg_combiner* m) {
    if (!m) return;
    (void)hipHostFree(m->h_puts);
    (void)hipHostFree(m->h_keys);
    (void)hipHostFree(m->h_prev);
    (void)hipHostFree(m->h_prevf);
    (void)hipHostFree(m->h_vals);
    (void)hipHostFree(m->h_found);
    (void)hipFree(m->d_puts);
    (void)hipFree(m->d_keys);
    (void)hipFree(m->d_prev);
    (void)hipFree(m->d_prevf);
    (void)hipFree(m->d_vals);
    (void)hipFree(m->d_found);
    delete[] m->ctxs;
    delete m;
}

extern "C" int nrg_combiner_open(nrg_ctx* ctx, uint32_t max_threads, nrg_combiner** out) {
    if (!ctx || !out || !max_threads || max_threads > 4096 || ctx->cfg.ds_kind != NRG_DS_HASHMAP)
        return NRG_E_INVAL;
    const uint64_t cap = (uint64_t)max_threads * MAX_PENDING;
    if (cap > ctx->cfg.max_batch || cap > ctx->cfg.max_reads) return NRG_E_CAPACITY;
    int r = nrg::ctx_use_device(ctx);
    if (r) return r;
    nrg_combiner* m = new (std::nothrow) nrg_combiner();
    if (!m) return NRG_E_NOMEM;
    m->ctx = ctx;
    m->max_threads = max_threads;
    m->cap = cap;
    m->ctxs = new (std::nothrow) Ctx[max_threads];
    m->batch.reserve(max_threads);
    bool ok = m->ctxs != nullptr;
    ok = ok && hipHostMalloc(&m->h_puts, cap * sizeof(nrg_put)) == hipSuccess;
    ok = ok && hipHostMalloc(&m->h_keys, cap * 8) == hipSuccess;
    ok = ok && hipHostMalloc(&m->h_prev, cap * 8) == hipSuccess;
    ok = ok && hipHostMalloc(&m->h_prevf, cap) == hipSuccess;
    ok = ok && hipHostMalloc(&m->h_vals, cap * 8) == hipSuccess;
    ok = ok && hipHostMalloc(&m->h_found, cap) == hipSuccess;
    ok = ok && hipMalloc(&m->d_puts, cap * sizeof(nrg_put)) == hipSuccess;
    ok = ok && hipMalloc(&m->d_keys, cap * 8) == hipSuccess;
    ok = ok && hipMalloc(&m->d_prev, cap * 8) == hipSuccess;
    ok = ok && hipMalloc(&m->d_prevf, cap) == hipSuccess;
    ok = ok && hipMalloc(&m->d_vals, cap * 8) == hipSuccess;
    ok = ok && hipMalloc(&m->d_found, cap) == hipSuccess;
    if (!ok) {
        comb_free(m);
        return NRG_E_NOMEM;
    }
    *out = m;
    return NRG_OK;
}

extern "C" int nrg_combiner_close(nrg_combiner* m) {
    if (!m) return NRG_E_INVAL;
    std::lock_guard<std::mutex> g(m->lock);
    (void)nrg::ctx_use_device(m->ctx);
    (void)hipStreamSynchronize((hipStream_t)nrg_get_stream(m->ctx));
    comb_free(m);
    return NRG_OK;
}

// Replica::register (nr/src/replica.rs:345-356): a context for the calling thread.
extern "C" int nrg_combiner_register(nrg_combiner* m, uint32_t* token) {
    if (!m || !token) return NRG_E_INVAL;
    uint32_t t = m->next.load(std::memory_order_relaxed);
    do {
        if (t >= m->max_threads) return NRG_E_CAPACITY;
    } while (!m->next.compare_exchange_weak(t, t + 1, std::memory_order_relaxed));
    *token = t;
    return NRG_OK;
}

// Replica::combine (nr/src/replica.rs:544-595), under the combiner lock: one GPU round of
// every posted op, responses scattered back to their contexts.
static void combine(nrg_combiner* m) {
    nrg_ctx* c = m->ctx;
    m->batch.clear();
    uint64_t W = 0, R = 0;
    for (uint32_t i = 0; i < m->max_threads; i++) {
        Ctx& x = m->ctxs[i];
        if (x.state.load(std::memory_order_acquire) != POSTED) continue;
        m->batch.push_back(i);
        if (x.put) {
            for (uint32_t k = 0; k < x.n; k++) m->h_puts[W + k] = nrg_put{x.keys[k], x.vals[k]};
            W += x.n;
        } else {
            std::memcpy(m->h_keys + R, x.keys, x.n * 8);
            R += x.n;
        }
    }
    if (m->batch.empty()) return;
    int rc = nrg::ctx_use_device(c);
    hipStream_t st = (hipStream_t)nrg_get_stream(c);
    if (!rc && W && hipMemcpyAsync(m->d_puts, m->h_puts, W * sizeof(nrg_put), hipMemcpyHostToDevice, st))
        rc = NRG_E_HIP;
    if (!rc && R && hipMemcpyAsync(m->d_keys, m->h_keys, R * 8, hipMemcpyHostToDevice, st)) rc = NRG_E_HIP;
    if (!rc)
        rc = nrg_hashmap_round_async(c, m->d_puts, W, c->cfg.replica_id, m->d_keys, R, m->d_vals, m->d_found,
                                     m->d_prev, m->d_prevf);
    // responses are complete once the round's deferred half (config.pipeline) has run
    if (!rc && nrg_join(c)) rc = NRG_E_HIP;
    if (!rc && W &&
        (hipMemcpyAsync(m->h_prev, m->d_prev, W * 8, hipMemcpyDeviceToHost, st) ||
         hipMemcpyAsync(m->h_prevf, m->d_prevf, W, hipMemcpyDeviceToHost, st)))
        rc = NRG_E_HIP;
    if (!rc && R &&
        (hipMemcpyAsync(m->h_vals, m->d_vals, R * 8, hipMemcpyDeviceToHost, st) ||
         hipMemcpyAsync(m->h_found, m->d_found, R, hipMemcpyDeviceToHost, st)))
        rc = NRG_E_HIP;
    if (!rc) rc = nrg_sync(c);  // waits for the copies and reports latched device errors
    W = R = 0;
    for (uint32_t i : m->batch) {
        Ctx& x = m->ctxs[i];
        if (!rc) {
            if (x.put) {
                std::memcpy(x.out, m->h_prev + W, x.n * 8);
                std::memcpy(x.flag, m->h_prevf + W, x.n);
                W += x.n;
            } else {
                std::memcpy(x.out, m->h_vals + R, x.n * 8);
                std::memcpy(x.flag, m->h_found + R, x.n);
                R += x.n;
            }
        }
        x.rc = rc;
        x.state.store(DONE, std::memory_order_release);
    }
    m->rounds++;
    m->ops += W + R;
}

// Post n ops in the calling thread's context, then combine or wait (nr/src/replica.rs:414-433).
static int post_and_wait(nrg_combiner* m, uint32_t token, bool put, const uint64_t* keys, const uint64_t* vals,
                         uint32_t n, uint64_t* out, uint8_t* flag) {
    if (!m || token >= m->max_threads || (n && (!keys || !out || !flag || (put && !vals)))) return NRG_E_INVAL;
    if (n > MAX_PENDING) return NRG_E_CAPACITY;
    if (!n) return NRG_OK;
    Ctx& x = m->ctxs[token];
    x.n = n;
    x.put = put;
    x.keys = keys;
    x.vals = vals;
    x.out = out;
    x.flag = flag;
    x.state.store(POSTED, std::memory_order_release);
    for (uint32_t spins = 0; x.state.load(std::memory_order_acquire) != DONE; spins++) {
        if (m->lock.try_lock()) {
            if (x.state.load(std::memory_order_acquire) != DONE) combine(m);
            m->lock.unlock();
        } else if (spins > 64) {
            // a round is tens of microseconds: waiting threads sleep instead of competing with
            // the combining thread for the host cores
            std::this_thread::sleep_for(std::chrono::microseconds(10));
        }
    }
    x.state.store(EMPTY, std::memory_order_relaxed);
    return x.rc;
}

// Replica::execute_mut(Put(k, v)) for up to 32 ops of one thread: prev[i] / some[i] =
// HashMap::insert's previous value (nr/examples/hashmap.rs:46-50).
extern "C" int nrg_combiner_put(nrg_combiner* m, uint32_t token, const uint64_t* keys, const uint64_t* vals,
                                uint32_t n, uint64_t* prev, uint8_t* some) {
    return post_and_wait(m, token, true, keys, vals, n, prev, some);
}

// Replica::execute(Get(k)) for up to 32 ops of one thread: vals[i] / found[i].
extern "C" int nrg_combiner_get(nrg_combiner* m, uint32_t token, const uint64_t* keys, uint32_t n, uint64_t* vals,
                                uint8_t* found) {
    return post_and_wait(m, token, false, keys, nullptr, n, vals, found);
}

// GPU rounds combined so far and the ops they carried.
extern "C" int nrg_combiner_stats(nrg_combiner* m, uint64_t* rounds, uint64_t* ops) {
    if (!m || !rounds || !ops) return NRG_E_INVAL;
    std::lock_guard<std::mutex> g(m->lock);
    *rounds = m->rounds;
    *ops = m->ops;
    return NRG_OK;
}
