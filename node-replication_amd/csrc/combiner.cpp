// combiner.cpp — the Replica's flat combining on the host, native, pipelined.
//
// Reference: nr/src/context.rs:88-194 (a per-thread context of at most MAX_PENDING_OPS = 32
// pending ops and their responses), nr/src/replica.rs:345-356 (register), :404-433 (execute /
// execute_mut: post, then try to combine until the response is there), :483-497 (reads after
// sync-to-tail), :508-595 (try_combine / combine: whoever takes the combiner lock appends every
// thread's pending ops as ONE batch, replays the log and hands each thread its responses).
//
// A batch is one GPU round of the replica. Batches live in NB slots of mapped, coherent pinned
// host memory that the round's kernels read and write directly, so a round costs no copies:
//   post   : a client thread reserves room in the OPEN batch with an atomic add (as Log::append
//            reserves log entries with a CAS on tail, nr/src/log.rs:391-399), copies its ops in
//            and waits for its round;
//   combine: the combiner seals the open batch, opens the next slot and enqueues the round on the
//            replica's stream -- Log::append + Log::exec of the batch's writes, then its reads
//            against the post-round state -- followed by an event, without waiting for the GPU:
//            batch k+1 fills while round k runs (at most DEPTH rounds in flight);
//   retire : the combiner queries the in-flight rounds' events in order; a completed round's
//            responses are already in host memory, its clients are woken and copy theirs out.
// The combining role belongs to the library's combiner thread rather than to whichever client
// takes a lock (nr/src/replica.rs:508-540): a round completes asynchronously on the GPU and needs a
// host thread polling it, and with hundreds of clients on a few cores a client that holds the
// role is descheduled while everyone waits. Clients park on a futex of their batch (a test knob
// lets some of them spin instead); the combiner thread parks when there is nothing to do and the
// first post wakes it.
// Reads ride in the round that collects them, after its writes: they see every write completed
// before they were posted (sync-to-tail) and never wait behind a later write round.
//
// Generic over the three data structures (nr's Replica<D> is generic over Dispatch,
// nr/src/replica.rs:72-115): hashmap Put/Get, stack Push-Pop/Peek, synthetic writes/ReadOnly.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <linux/futex.h>
#include <sched.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>

#include "internal.hpp"

namespace {

constexpr uint32_t MAX_PENDING = 32;  // nr/src/context.rs:12 MAX_PENDING_OPS
constexpr uint32_t WAKE_FAN = 2;  // children each woken waiter wakes (a binary wake-up tree; 4 measured:
                                  // 16 threads 16.2-16.8 vs 18.0-19.0 M ops/s, 256 threads 31 vs 43,
                                  // 64 threads 40.4 vs 37.6; profiles/r04_combiner.txt E)
constexpr int NB = 6;                 // batch slots
static_assert(NB <= (int)nrg::SERVE_SLOTS, "a doorbell per batch slot");
constexpr uint64_t DEPTH = 2;         // default rounds in flight (NRG_KNOB_COMB_DEPTH, <= NB - 2: a
                                      // slot's clients copy their responses out while later rounds run)
// With a round in flight, the open batch is sealed into a second one only once it holds this
// many ops: with few clients a small second round only splits them over more rounds (16 threads x
// 32 ops: 16.4 M ops/s one round in flight vs 13.9 with two; 128 threads 55.9 vs 60.1;
// profiles/r04_combiner.txt)
constexpr uint32_t SECOND_MIN = 512;
// With no round in flight, the open batch waits up to this long (NRG_KNOB_COMB_GATHER, us) for as
// many posts as the last round carried: the clients a round woke post again over the ~15 us their
// wake-up tree takes, and a batch sealed at the first post leaves the rest a whole round behind.
// 16 threads x 32 ops: 15.5 / 15.4 / 15.2 / 18.7 M ops/s at 0 / 5 / 10 / 20 us (256 / 256 / 285 /
// 511 ops per round); 64 threads 35.4 / 35.7 / 37.4 / 38.9 (profiles/r04_combiner.txt)
constexpr uint32_t GATHER_US = 20;

// CPUs this process may run on at once: its affinity mask, capped by a cgroup v2 CPU quota
int usable_cpus() {
    cpu_set_t set;
    int n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long long period = 0;
        if (std::fscanf(f, "%31s %llu", q, &period) == 2 && std::strcmp(q, "max") != 0 && period) {
            const unsigned long long quota = std::strtoull(q, nullptr, 10);
            const int cap = (int)((quota + period - 1) / period);
            if (cap > 0 && cap < n) n = cap;
        }
        std::fclose(f);
    }
    return n;
}

uint64_t now_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

enum : uint32_t { FREE = 0, OPEN = 1, SEALED = 2, DONE = 3 };

void futex_wait(std::atomic<uint32_t>* w, uint32_t seen, long ns = 2000000) {
    const timespec ts{0, ns};  // a lost wake-up costs at most 2 ms
    syscall(SYS_futex, (uint32_t*)w, FUTEX_WAIT_PRIVATE, seen, &ts, nullptr, 0);
}
void futex_wake_all(std::atomic<uint32_t>* w) { syscall(SYS_futex, (uint32_t*)w, FUTEX_WAKE_PRIVATE, INT32_MAX, nullptr, nullptr, 0); }
void wake_one(std::atomic<uint32_t>* w) {
    w->fetch_add(1, std::memory_order_seq_cst);
    syscall(SYS_futex, (uint32_t*)w, FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
}

struct alignas(64) Batch {
    std::atomic<uint32_t> state{FREE};
    std::atomic<uint64_t> round{~0ull};  // round number while OPEN/SEALED/DONE
    alignas(64) std::atomic<uint32_t> writers{0};  // clients copying ops in
    std::atomic<uint32_t> readers{0};              // clients yet to copy their responses out
    std::atomic<uint32_t> nw{0}, nr{0};            // write records / reads reserved
    // Waiting clients take numbers 0, 1, 2, ... and park each on its own futex word wk[i], so
    // wake-ups never contend on one kernel futex bucket (one word for the whole batch spent the
    // job's CPU quota in the kernel at 128+ threads). They wake as a binary tree: the combiner
    // thread wakes waiter 0 and waiter i wakes 2i+1 and 2i+2 -- off the combiner's path, and
    // about log2(waiters) wake-up latencies for the last one.
    // (Measured and dropped: the first 16 or 32 waiters parked on one shared word and woken by
    // one FUTEX_WAKE -- 13.7 / 16.6 vs 14.5 M ops/s at 16 threads, 30.3 / 26.7 vs 36.5 at 64;
    // profiles/r04_combiner.txt.)
    alignas(64) std::atomic<uint32_t> nwait{0};
    std::atomic<uint32_t>* wk = nullptr;  // [max_threads]
    int rc = NRG_OK;                               // launch or device error of the round
    // host buffers (mapped, coherent; device addresses equal the host ones under UVA)
    char* recs = nullptr;   // cap write records
    char* reads = nullptr;  // cap read records
    char* wresp = nullptr;  // cap write responses
    uint8_t* wsome = nullptr;
    char* rresp = nullptr;  // cap read responses
    uint8_t* rsome = nullptr;
    uint32_t* err = nullptr;  // the replica's error latch after the round (ERR_PENDING until then)
    uint32_t polls = 0;       // retire's polls of the word (the event is queried every 256th)
    uint64_t t_open = 0, t_seal = 0, t_post = 0;  // (stats) when the batch opened, was sealed, went out
    bool served = false;      // the round went to the round server (no launch, no event)
    uint64_t lo = 0;          // its first log position (a relaunched server starts there)
    hipEvent_t done = nullptr;
};

// Completion of a round: its last write is the replica's error latch, copied into the batch's
// mapped word (host memory) -- by the one-workgroup small round kernel itself, or by this kernel
// behind the round. The combiner thread polls the word: no event record or query per round.
constexpr uint32_t ERR_PENDING = 0xFFFFFFFFu;  // the round's error word until the round completes

// device: the error latch of the replica, copied to host memory and cleared after a round
__global__ void comb_err_kernel(nrg::DevCtl* ctl, uint32_t* out) {
    if (threadIdx.x == 0) {
        const uint32_t e = atomicExch(&ctl->err, 0u);
        __threadfence_system();
        *(volatile uint32_t*)out = e;
    }
}

// device: n Peeks of the stack after the round (nr/tests/stack.rs:26-29, benches/stack.rs)
__global__ void comb_peek_kernel(const nrg::DevCtl* ctl, const uint32_t* stack, uint64_t cap, uint32_t n,
                                 uint32_t* out, uint8_t* some) {
    const long long d = ctl->depth;
    const bool has = d > 0 && (uint64_t)d <= cap;
    const uint32_t top = has ? stack[d - 1] : 0u;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        out[i] = top;
        some[i] = has;
    }
}

int err_code(uint32_t e) {
    if (!e) return NRG_OK;
    if (e & nrg::ERR_TABLE_FULL) return NRG_E_TABLE_FULL;
    if (e & nrg::ERR_CAPACITY) return NRG_E_CAPACITY;
    return NRG_E_HIP;
}

}  // namespace

struct nrg_combiner {
    nrg_ctx* ctx = nullptr;
    uint32_t kind = 0;
    uint32_t max_threads = 0;
    uint64_t cap = 0;  // ops of each kind per batch: max_threads * MAX_PENDING
    uint32_t rec_b = 0, rd_b = 0, wr_b = 0, rr_b = 0;  // write record / read record / responses
    bool saved_pipeline = false;
    uint64_t saved_small = 0;
    std::atomic<uint32_t> next_tok{0};
    // one post in flight per token: keeps a batch's reservations within cap and its waiters
    // within wk[max_threads] even when two threads misuse one token
    struct alignas(64) Tok {
        std::atomic<uint32_t> busy{0};
    };
    Tok* tok = nullptr;  // [max_threads]
    Batch b[NB];
    alignas(64) std::atomic<uint64_t> open{0};       // round number of the OPEN batch
    std::atomic<uint32_t> opened{0};                 // futex word: bumped when a batch opens
    std::atomic<uint32_t> open_sleepers{0};          // clients parked until one does
    alignas(64) std::atomic<uint64_t> completed{0};  // rounds < completed are done
    std::atomic<uint64_t> launched{0};               // rounds < launched are enqueued (combiner thread)
    std::atomic<uint64_t> rounds{0}, ops{0};
    uint64_t t_n = 0, t_gather = 0, t_enqueue = 0, t_gpu = 0;  // (combiner thread) round phase sums, ns
    int32_t spin_cap = 0;                            // clients that may spin at once
    uint64_t depth = DEPTH;                          // rounds in flight
    bool depth_auto = true;                          // a second round only for a batch of SECOND_MIN ops
    uint64_t gather_ns = GATHER_US * 1000ull;        // (combiner thread) GATHER_US window
    uint32_t last_posts = 0;                         // posts of the last sealed batch
    uint64_t gather_k = ~0ull, gather_t0 = 0;        // the batch being gathered, its first sight
    alignas(64) std::atomic<int32_t> spinning{0};
    // the round server (hashmap.hip hm_serve_kernel): small hashmap rounds without a launch each
    nrg::ServeCtl* sc = nullptr;     // mapped host memory
    nrg::SmallJobBlob* hdr = nullptr;  // [NB] the jobs, by batch slot (mapped host memory)
    bool serve = false;              // policy (NRG_KNOB_COMB_SERVE)
    uint32_t serve_max = 0;          // (tests) serve only rounds of at most this many ops (0: any)
    bool srv_running = false;        // a server of session `session` is launched and not seen to exit
    uint64_t session = 0;
    uint64_t idle_t0 = 0;            // (combiner thread) when it went idle with the server running
    // the combiner thread
    std::thread worker;
    std::atomic<bool> stop{false};
    alignas(64) std::atomic<uint32_t> work{0};       // futex word: bumped by a post that finds it parked
    std::atomic<uint32_t> parked{0};
};

namespace {

void* host_alloc(uint64_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
    return p;
}

void comb_free(nrg_combiner* m) {
    if (!m) return;
    if (m->sc) (void)hipHostFree(m->sc);
    if (m->hdr) (void)hipHostFree(m->hdr);
    for (Batch& x : m->b) {
        void* ps[] = {x.recs, x.reads, x.wresp, x.wsome, x.rresp, x.rsome, x.err};
        for (void* p : ps)
            if (p) (void)hipHostFree(p);
        if (x.done) (void)hipEventDestroy(x.done);
        delete[] x.wk;
    }
    delete[] m->tok;
    delete m;
}

// ---- the round server ----------------------------------------------------------------------------
// A resident workgroup (hm_serve_kernel) serves the small hashmap rounds: the combiner thread
// writes a round's job into its slot's header and bumps `posted`; the round's error word is its
// completion as before. Any launch on the replica's stream would queue behind the server, so the
// server is stopped first (it drains every posted round, then exits); it is also stopped when the
// combiner has been idle for SERVE_IDLE_NS and at close, and exits by itself after SERVE_IDLE_TICKS
// without a post (a host that died or stalled never leaves it running).
constexpr uint64_t SERVE_IDLE_NS = 1000000;      // 1 ms idle: stop the server
constexpr uint64_t SERVE_IDLE_TICKS = 10000000;  // 100 ms of the 100-MHz wall clock: it stops itself

uint64_t vload(const uint64_t* p) { return __atomic_load_n(p, __ATOMIC_SEQ_CST); }

int serve_start(nrg_combiner* m, uint64_t first, uint64_t first_lo) {
    nrg_ctx* c = m->ctx;
    m->session++;
    __atomic_store_n(&m->sc->stop, 0u, __ATOMIC_SEQ_CST);
    if (nrg::hm_serve_launch(c, m->sc, m->hdr, NB, first, first_lo, m->session, SERVE_IDLE_TICKS) != hipSuccess)
        return NRG_E_HIP;
    m->srv_running = true;
    return NRG_OK;
}

// stop the server once every posted round is served (combiner thread)
int serve_stop(nrg_combiner* m) {
    if (!m->srv_running) return NRG_OK;
    __atomic_store_n(&m->sc->stop, 1u, __ATOMIC_SEQ_CST);
    hipStream_t st = (hipStream_t)nrg_get_stream(m->ctx);
    int rc = NRG_OK;
    for (uint32_t i = 0; vload(&m->sc->exited) != m->session; i++) {
        if ((i & 255) == 255) {  // a server that faulted never writes `exited`
            const hipError_t q = hipStreamQuery(st);
            if (q != hipErrorNotReady) {
                if (q != hipSuccess) rc = NRG_E_HIP;
                break;
            }
        }
        _mm_pause();
    }
    __atomic_store_n(&m->sc->stop, 0u, __ATOMIC_SEQ_CST);
    m->srv_running = false;
    return rc;
}

// Retire completed rounds in order and wake their clients (combiner thread). A round is complete
// when its error word leaves ERR_PENDING; its event is queried only now and then, to catch a
// round that failed on the device and will never write the word.
void retire(nrg_combiner* m) {
    uint64_t k = m->completed.load(std::memory_order_relaxed);
    while (k < m->launched.load(std::memory_order_acquire)) {
        Batch& x = m->b[k % NB];
        const uint32_t ew = *(volatile uint32_t*)x.err;
        if (ew == ERR_PENDING && x.rc == NRG_OK) {
            if ((++x.polls & 255) != 0) break;
            if (x.served) {
                // a server that exited by itself (idle bound) before this round was posted never
                // reads `posted` again: serve the rest from `served` with a new one
                if (m->srv_running && vload(&m->sc->exited) == m->session && vload(&m->sc->served) <= k) {
                    m->srv_running = false;
                    const uint64_t s0 = vload(&m->sc->served);
                    if (serve_start(m, s0, m->b[s0 % NB].lo) != NRG_OK) x.rc = NRG_E_HIP;
                }
                const hipError_t q = hipStreamQuery((hipStream_t)nrg_get_stream(m->ctx));
                if (q != hipSuccess && q != hipErrorNotReady) x.rc = NRG_E_HIP;  // the server faulted
                if (x.rc == NRG_OK) break;
            } else {
                const hipError_t q = hipEventQuery(x.done);
                if (q == hipErrorNotReady) break;
                if (*(volatile uint32_t*)x.err == ERR_PENDING) x.rc = NRG_E_HIP;  // done, and the word never came
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);  // responses after the word
        if (x.rc == NRG_OK) x.rc = err_code(*(volatile uint32_t*)x.err);
        x.state.store(DONE, std::memory_order_release);
        const uint64_t t_done = now_ns();
        m->t_n++;
        m->t_gather += x.t_seal - x.t_open;
        m->t_enqueue += x.t_post - x.t_seal;
        m->t_gpu += t_done - x.t_post;
        m->completed.store(++k, std::memory_order_seq_cst);
        if (x.nwait.load(std::memory_order_seq_cst)) wake_one(&x.wk[0]);  // the root of the wake tree
    }
}

// Enqueue the round k of sealed batch x (combiner thread): the replica's writes, then its reads.
int launch(nrg_combiner* m, Batch& x, uint64_t k, uint32_t W, uint32_t R) {
    nrg_ctx* c = m->ctx;
    int rc = nrg::ctx_use_device(c);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)nrg_get_stream(c);
    const uint32_t origin = c->cfg.replica_id;
    *(volatile uint32_t*)x.err = ERR_PENDING;
    x.polls = 0;
    x.served = false;
    if (m->serve && W <= 2048 && R <= nrg::SERVE_R && (m->serve_max == 0 || W + R <= m->serve_max)) {
        // the round server takes it: the log bookkeeping here, then the slot's doorbell with the
        // round's counts (the slot's buffers are fixed: the server read them when it started)
        uint64_t lo = 0;
        rc = nrg::hm_small_job(c, (const nrg_put*)x.recs, W, origin, (const uint64_t*)x.reads, R, (uint64_t*)x.rresp,
                               x.rsome, (uint64_t*)x.wresp, x.wsome, x.err, nullptr, &lo);
        if (rc == NRG_OK) {
            x.lo = lo;
            if (!m->srv_running && (rc = serve_start(m, k, lo)) != NRG_OK) return rc;
            __atomic_store_n(&m->sc->door[k % NB], ((k + 1) << 32) | ((uint64_t)W << 16) | R, __ATOMIC_SEQ_CST);
            x.served = true;
            return NRG_OK;
        }
        rc = NRG_OK;  // not a small round of a caught-up replica: launched below
    }
    if (m->srv_running && (rc = serve_stop(m)) != NRG_OK) return rc;  // launches queue behind the server
    // hashmap rounds of <= 2048 Puts (>= 1) and <= 8192 Gets run as ONE small-round workgroup
    // (hashmap.hip small_round), whose last write can be the error copy
    const bool small = m->kind == NRG_DS_HASHMAP && W > 0 && W <= c->small_max && W <= 2048 && R <= 8192;
    switch (m->kind) {
        case NRG_DS_HASHMAP:  // Put -> HashMap::insert's previous value (nr/examples/hashmap.rs:46-50)
            // a small round (one workgroup, the round's only launch) copies the error latch as its
            // last write and clears c->err_out; any other round leaves it set (only
            // hm_small_round_kernel takes it) and gets comb_err_kernel behind it
            if (small) c->err_out = x.err;
            rc = nrg_hashmap_round_async(c, (const nrg_put*)x.recs, W, origin, (const uint64_t*)x.reads, R,
                                         (uint64_t*)x.rresp, x.rsome, (uint64_t*)x.wresp, x.wsome);
            break;
        case NRG_DS_STACK:
            if (W) rc = nrg_stack_round_async(c, (const nrg_stack_op*)x.recs, W, origin, (uint32_t*)x.wresp, x.wsome);
            if (!rc && R) {
                comb_peek_kernel<<<1, 256, 0, st>>>(c->d_ctl, c->d_stack, c->cfg.stack_capacity, R,
                                                    (uint32_t*)x.rresp, x.rsome);
                if (hipGetLastError() != hipSuccess) rc = NRG_E_HIP;
            }
            break;
        default:  // synthetic: ReadWrite/WriteOnly sums, then ReadOnly sums
            if (W) rc = nrg_synth_round_async(c, (const nrg_synth_op*)x.recs, W, origin, (uint64_t*)x.wresp, x.wsome);
            if (!rc && R) {
                std::memset(x.rsome, 1, R);
                rc = nrg_synth_read_async(c, (const nrg_synth_rd*)x.reads, R, (uint64_t*)x.rresp);
            }
            break;
    }
    if (!rc && nrg_join(c)) rc = NRG_E_HIP;  // a deferred round tail would write responses later
    if (!rc && (!small || c->err_out)) {
        // no small round took the error copy as its last write
        c->err_out = nullptr;
        comb_err_kernel<<<1, 64, 0, st>>>(c->d_ctl, x.err);
        if (hipGetLastError() != hipSuccess) rc = NRG_E_HIP;
    }
    c->err_out = nullptr;
    return rc;
}

// Combiner thread: seal the open batch and enqueue its round if it holds ops and fewer than
// DEPTH rounds are in flight; true if it did.
bool advance(nrg_combiner* m) {
    const uint64_t k = m->open.load(std::memory_order_relaxed);
    Batch& x = m->b[k % NB];
    const uint64_t inflight = m->launched.load(std::memory_order_relaxed) - m->completed.load(std::memory_order_acquire);
    if (inflight >= m->depth) return false;
    const uint32_t ops = x.nw.load(std::memory_order_seq_cst) + x.nr.load(std::memory_order_seq_cst);
    if (!ops || (inflight && m->depth_auto && ops < SECOND_MIN)) return false;
    if (!inflight && m->gather_ns && x.readers.load(std::memory_order_relaxed) < m->last_posts) {
        const uint64_t t = now_ns();
        if (m->gather_k != k) {
            m->gather_k = k;
            m->gather_t0 = t;
        }
        if (t - m->gather_t0 < m->gather_ns) return false;
    }
    x.t_seal = now_ns();
    x.state.store(SEALED, std::memory_order_seq_cst);
    while (x.writers.load(std::memory_order_seq_cst)) _mm_pause();
    m->last_posts = x.readers.load(std::memory_order_relaxed);  // (no client has left a sealed batch)
    const uint32_t W = x.nw.load(std::memory_order_relaxed), R = x.nr.load(std::memory_order_relaxed);
    // open round k+1 in the next slot: its previous round (k+1-NB) is complete (DEPTH < NB - 1);
    // wait for that round's clients to copy their responses out
    Batch& y = m->b[(k + 1) % NB];
    while (y.readers.load(std::memory_order_acquire)) _mm_pause();
    y.nw.store(0, std::memory_order_relaxed);
    y.nr.store(0, std::memory_order_relaxed);
    y.rc = NRG_OK;
    y.nwait.store(0, std::memory_order_relaxed);
    y.round.store(k + 1, std::memory_order_relaxed);
    y.t_open = now_ns();
    y.state.store(OPEN, std::memory_order_seq_cst);
    m->open.store(k + 1, std::memory_order_seq_cst);
    m->opened.fetch_add(1, std::memory_order_seq_cst);
    if (m->open_sleepers.load(std::memory_order_seq_cst)) futex_wake_all(&m->opened);
    x.rc = launch(m, x, k, W, R);
    x.t_post = now_ns();
    hipStream_t st = (hipStream_t)nrg_get_stream(m->ctx);
    if (!x.served && hipEventRecord(x.done, st) != hipSuccess && x.rc == NRG_OK) x.rc = NRG_E_HIP;
    if (x.rc != NRG_OK) *(volatile uint32_t*)x.err = 0;  // nothing will write it: retire at once
    m->launched.store(k + 1, std::memory_order_release);
    m->rounds.fetch_add(1, std::memory_order_relaxed);
    m->ops.fetch_add(W + R, std::memory_order_relaxed);
    return true;
}

// The combiner thread: seal and launch, retire, park when idle.
void combiner_main(nrg_combiner* m) {
    (void)nrg::ctx_use_device(m->ctx);
    while (!m->stop.load(std::memory_order_acquire)) {
        const uint64_t done0 = m->completed.load(std::memory_order_relaxed);
        retire(m);
        const bool launched = advance(m);
        if (launched) m->idle_t0 = 0;
        if (launched || m->completed.load(std::memory_order_relaxed) != done0) continue;
        const bool busy = m->launched.load(std::memory_order_relaxed) != m->completed.load(std::memory_order_relaxed);
        if (busy) {  // a round is in flight: poll again shortly
            for (int i = 0; i < 16; i++) _mm_pause();
            continue;
        }
        // idle: park until a post (or close) bumps `work`; a server idle for SERVE_IDLE_NS is stopped
        if (m->srv_running) {
            const uint64_t t = now_ns();
            if (!m->idle_t0) m->idle_t0 = t;
            if (t - m->idle_t0 >= SERVE_IDLE_NS) {
                (void)serve_stop(m);  // (a fault shows up in the next round's launch)
                m->idle_t0 = 0;
            }
        }
        const uint32_t seen = m->work.load(std::memory_order_seq_cst);
        m->parked.store(1, std::memory_order_seq_cst);
        const Batch& o = m->b[m->open.load(std::memory_order_seq_cst) % NB];
        if (!o.nw.load(std::memory_order_seq_cst) && !o.nr.load(std::memory_order_seq_cst) &&
            !m->stop.load(std::memory_order_seq_cst))
            futex_wait(&m->work, seen, m->srv_running ? 250000 : 2000000);
        m->parked.store(0, std::memory_order_seq_cst);
    }
}

// Post n ops of one thread, then combine or wait until their round is done (nr/src/replica.rs:414-433).
int post_and_wait(nrg_combiner* m, uint32_t token, bool write, const void* ops, uint32_t n, void* out,
                  uint8_t* some) {
    if (!m || token >= m->max_threads || (n && (!out || !some || (!ops && (write || m->kind != NRG_DS_STACK)))))
        return NRG_E_INVAL;
    if (n > MAX_PENDING) return NRG_E_CAPACITY;
    if (!n) return NRG_OK;
    if (m->tok[token].busy.exchange(1, std::memory_order_acquire)) return NRG_E_INVAL;  // token in use
    const uint32_t in_b = write ? m->rec_b : m->rd_b, out_b = write ? m->wr_b : m->rr_b;
    uint64_t k;
    Batch* x;
    uint32_t off;
    for (uint32_t spins = 0;; spins++) {  // reserve room in the open batch (Context::enqueue)
        const uint32_t seen = m->opened.load(std::memory_order_seq_cst);
        k = m->open.load(std::memory_order_seq_cst);
        x = &m->b[k % NB];
        // a sealed batch's `writers` is left alone: the combiner thread waits for it to reach 0,
        // and hundreds of clients bumping it on every retry kept it from ever reaching 0
        const bool open = x->state.load(std::memory_order_seq_cst) == OPEN &&
                          x->round.load(std::memory_order_relaxed) == k;
        if (open) x->writers.fetch_add(1, std::memory_order_seq_cst);
        if (open && x->state.load(std::memory_order_seq_cst) == OPEN && x->round.load(std::memory_order_relaxed) == k) {
            off = (write ? x->nw : x->nr).fetch_add(n, std::memory_order_seq_cst);
            x->readers.fetch_add(1, std::memory_order_relaxed);
            if (in_b && ops) std::memcpy((write ? x->recs : x->reads) + (uint64_t)off * in_b, ops, (size_t)n * in_b);
            x->writers.fetch_sub(1, std::memory_order_release);
            break;
        }
        if (open) x->writers.fetch_sub(1, std::memory_order_relaxed);
        // the batch is sealed and the next one not open yet (the combiner waits for a slot's
        // clients to copy their responses out): do not take their cores, park until it opens
        if (spins < 64) {
            _mm_pause();
            continue;
        }
        m->open_sleepers.fetch_add(1, std::memory_order_seq_cst);
        if (m->open.load(std::memory_order_seq_cst) == k) futex_wait(&m->opened, seen);
        m->open_sleepers.fetch_sub(1, std::memory_order_seq_cst);
    }
    if (m->parked.load(std::memory_order_seq_cst)) {  // wake the combiner thread
        m->work.fetch_add(1, std::memory_order_seq_cst);
        syscall(SYS_futex, (uint32_t*)&m->work, FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
    }
    // wait for the round: spin (about a round) if a spinning slot is free (NRG_KNOB_COMB_SPIN;
    // none by default), else park on the batch's futex
    const bool spin = m->spin_cap > 0 && m->spinning.fetch_add(1, std::memory_order_relaxed) < m->spin_cap;
    if (m->spin_cap > 0 && !spin) m->spinning.fetch_sub(1, std::memory_order_relaxed);
    uint32_t me = UINT32_MAX;  // this client's number among the batch's waiters
    for (uint32_t spins = 0; m->completed.load(std::memory_order_acquire) <= k; spins++) {
        if (spin && spins < 4096) {
            for (int i = 0; i < 8; i++) _mm_pause();
            continue;
        }
        if (me == UINT32_MAX) me = x->nwait.fetch_add(1, std::memory_order_seq_cst);
        const uint32_t seen = x->wk[me].load(std::memory_order_seq_cst);
        if (m->completed.load(std::memory_order_seq_cst) <= k) futex_wait(&x->wk[me], seen);
    }
    if (spin) m->spinning.fetch_sub(1, std::memory_order_relaxed);
    // waiter `me` wakes its two children; every waiter that took a number does, parked or not,
    // and a child that takes its number after the round completed sees it and does not park
    if (me != UINT32_MAX) {
        const uint32_t nw = x->nwait.load(std::memory_order_seq_cst);
        for (uint32_t c = WAKE_FAN * me + 1; c <= WAKE_FAN * me + WAKE_FAN && c < nw; c++) wake_one(&x->wk[c]);
    }
    std::memcpy(out, (write ? x->wresp : x->rresp) + (uint64_t)off * out_b, (size_t)n * out_b);
    std::memcpy(some, (write ? x->wsome : x->rsome) + off, n);
    const int rc = x->rc;
    x->readers.fetch_sub(1, std::memory_order_release);
    m->tok[token].busy.store(0, std::memory_order_release);
    return rc;
}

}  // namespace

extern "C" int nrg_combiner_open(nrg_ctx* ctx, uint32_t max_threads, nrg_combiner** out) {
    if (!ctx || !out || !max_threads || max_threads > 4096) return NRG_E_INVAL;
    const uint32_t kind = ctx->cfg.ds_kind;
    if (kind != NRG_DS_HASHMAP && kind != NRG_DS_STACK && kind != NRG_DS_SYNTHETIC) return NRG_E_INVAL;
    const uint64_t cap = (uint64_t)max_threads * MAX_PENDING;
    if (cap > ctx->cfg.max_batch || (kind == NRG_DS_HASHMAP && cap > ctx->cfg.max_reads)) return NRG_E_CAPACITY;
    int r = nrg::ctx_use_device(ctx);
    if (r) return r;
    // the replica's queued work completes first; rounds then complete within their own launch
    // sequence (no deferred tail), so an event after a round covers all of its responses
    if ((r = nrg_sync(ctx))) return r;
    nrg_combiner* m = new (std::nothrow) nrg_combiner();
    if (!m) return NRG_E_NOMEM;
    m->ctx = ctx;
    m->kind = kind;
    m->max_threads = max_threads;
    m->cap = cap;
    m->rec_b = ctx->rec_bytes;
    switch (kind) {
        case NRG_DS_HASHMAP: m->rd_b = 8, m->wr_b = 8, m->rr_b = 8; break;            // key; previous value; value
        case NRG_DS_STACK: m->rd_b = 0, m->wr_b = 4, m->rr_b = 4; break;              // Peek; popped; top
        default: m->rd_b = sizeof(nrg_synth_rd), m->wr_b = 8, m->rr_b = 8; break;  // sums
    }
    bool ok = true;
    ok = ok && (m->tok = new (std::nothrow) nrg_combiner::Tok[max_threads]());
    for (Batch& x : m->b) {
        ok = ok && (x.recs = (char*)host_alloc(cap * m->rec_b));
        ok = ok && (x.reads = (char*)host_alloc(cap * (m->rd_b ? m->rd_b : 1)));
        ok = ok && (x.wresp = (char*)host_alloc(cap * m->wr_b));
        ok = ok && (x.wsome = (uint8_t*)host_alloc(cap));
        ok = ok && (x.rresp = (char*)host_alloc(cap * m->rr_b));
        ok = ok && (x.rsome = (uint8_t*)host_alloc(cap));
        ok = ok && (x.err = (uint32_t*)host_alloc(64));
        ok = ok && hipEventCreateWithFlags(&x.done, hipEventDisableTiming) == hipSuccess;
        ok = ok && (x.wk = new (std::nothrow) std::atomic<uint32_t>[max_threads]());
        if (ok) *x.err = 0;
    }
    if (!ok) {
        comb_free(m);
        return NRG_E_NOMEM;
    }
    if (kind == NRG_DS_HASHMAP && ctx->comb_serve != 0) {
        ok = (m->sc = (nrg::ServeCtl*)host_alloc(sizeof(nrg::ServeCtl))) &&
             (m->hdr = (nrg::SmallJobBlob*)host_alloc(NB * sizeof(nrg::SmallJobBlob)));
        if (!ok) {
            comb_free(m);
            return NRG_E_NOMEM;
        }
        std::memset((void*)m->sc, 0, sizeof(nrg::ServeCtl));
        // each slot's fixed job fields (its batch buffers), read by a server when it starts
        for (int i = 0; i < NB && ok; i++) {
            Batch& x = m->b[i];
            ok = nrg::hm_small_fill(ctx, (const nrg_put*)x.recs, 0, 1, (const uint64_t*)x.reads, 1, (uint64_t*)x.rresp,
                                    x.rsome, (uint64_t*)x.wresp, x.wsome, x.err, &m->hdr[i]);
        }
        if (!ok) {
            comb_free(m);
            return NRG_E_INVAL;
        }
        m->serve = true;
        if (ctx->comb_serve >= 2) m->serve_max = (uint32_t)ctx->comb_serve;
    }
    m->saved_pipeline = ctx->pipeline;
    ctx->pipeline = false;
    // hashmap rounds of up to 2048 Puts in one launch (hashmap.hip hm_small_round_kernel)
    m->saved_small = ctx->small_max;
    if (kind == NRG_DS_HASHMAP) ctx->small_max = 2048;
    // Waiting clients park, unless every client fits the CPUs the job may use: then up to
    // max_threads - 1 of them spin on their round (16 threads on a 16-CPU quota: 19.6 vs 18.0-19.0
    // M ops/s parked, profiles/r04_combiner.txt F). With more clients than CPUs spinning ones take
    // the quota from the combiner thread (64 threads: 22.3 vs 24.5 M ops/s parked,
    // profiles/r03_combiner_policy.txt).
    if (ctx->comb_spin >= 0) {
        m->spin_cap = ctx->comb_spin;
    } else {
        const int cpus = usable_cpus();
        m->spin_cap = (int)max_threads <= cpus ? (int)max_threads - 1 : 0;
    }
    if (ctx->comb_gather >= 0) m->gather_ns = (uint64_t)ctx->comb_gather * 1000ull;
    if (ctx->comb_depth) {  // an explicit depth: no SECOND_MIN rule
        m->depth = std::min<uint64_t>(ctx->comb_depth, NB - 2);
        m->depth_auto = false;
    }
    m->b[0].round.store(0);
    m->b[0].t_open = now_ns();
    m->b[0].state.store(OPEN);
    try {
        m->worker = std::thread(combiner_main, m);
    } catch (...) {
        ctx->pipeline = m->saved_pipeline;
        ctx->small_max = m->saved_small;
        comb_free(m);
        return NRG_E_NOMEM;
    }
    *out = m;
    return NRG_OK;
}

// No thread may be inside nrg_combiner_put/get/execute* when the combiner is closed.
extern "C" int nrg_combiner_close(nrg_combiner* m) {
    if (!m) return NRG_E_INVAL;
    int rc = NRG_OK;
    m->stop.store(true, std::memory_order_seq_cst);
    m->work.fetch_add(1, std::memory_order_seq_cst);
    syscall(SYS_futex, (uint32_t*)&m->work, FUTEX_WAKE_PRIVATE, 1, nullptr, nullptr, 0);
    if (m->worker.joinable()) m->worker.join();  // the combiner thread touches nothing after this
    (void)nrg::ctx_use_device(m->ctx);
    if (serve_stop(m) != NRG_OK) rc = NRG_E_HIP;
    if (hipStreamSynchronize((hipStream_t)nrg_get_stream(m->ctx)) != hipSuccess) rc = NRG_E_HIP;
    m->ctx->pipeline = m->saved_pipeline;
    m->ctx->small_max = m->saved_small;
    comb_free(m);
    return rc;
}

// Replica::register (nr/src/replica.rs:279-298): a context for the calling thread.
extern "C" int nrg_combiner_register(nrg_combiner* m, uint32_t* token) {
    if (!m || !token) return NRG_E_INVAL;
    uint32_t t = m->next_tok.load(std::memory_order_relaxed);
    do {
        if (t >= m->max_threads) return NRG_E_CAPACITY;
    } while (!m->next_tok.compare_exchange_weak(t, t + 1, std::memory_order_relaxed));
    *token = t;
    return NRG_OK;
}

// Replica::execute_mut for up to 32 write ops (log records of the replica's kind).
extern "C" int nrg_combiner_execute_mut(nrg_combiner* m, uint32_t token, const void* recs, uint32_t n, void* resp,
                                        uint8_t* some) {
    return post_and_wait(m, token, true, recs, n, resp, some);
}

// Replica::execute for up to 32 read ops.
extern "C" int nrg_combiner_execute(nrg_combiner* m, uint32_t token, const void* reads, uint32_t n, void* resp,
                                    uint8_t* some) {
    return post_and_wait(m, token, false, reads, n, resp, some);
}

// Replica::execute_mut(Put(k, v)) for up to 32 ops of one thread: prev[i] / some[i] =
// HashMap::insert's previous value (nr/examples/hashmap.rs:46-50).
extern "C" int nrg_combiner_put(nrg_combiner* m, uint32_t token, const uint64_t* keys, const uint64_t* vals,
                                uint32_t n, uint64_t* prev, uint8_t* some) {
    if (!m || m->kind != NRG_DS_HASHMAP || (n && (!keys || !vals))) return NRG_E_INVAL;
    if (n > MAX_PENDING) return NRG_E_CAPACITY;
    nrg_put recs[MAX_PENDING];
    for (uint32_t i = 0; i < n; i++) recs[i] = nrg_put{keys[i], vals[i]};
    return post_and_wait(m, token, true, recs, n, prev, some);
}

// Replica::execute(Get(k)) for up to 32 ops of one thread: vals[i] / found[i].
extern "C" int nrg_combiner_get(nrg_combiner* m, uint32_t token, const uint64_t* keys, uint32_t n, uint64_t* vals,
                                uint8_t* found) {
    if (!m || m->kind != NRG_DS_HASHMAP) return NRG_E_INVAL;
    return post_and_wait(m, token, false, keys, n, vals, found);
}

// (tests) the round server's words and the combiner's round counters
extern "C" int nrg_test_combiner_probe(nrg_combiner* m, uint64_t out[8]) {
    if (!m || !out) return NRG_E_INVAL;
    if (m->sc)
        std::fprintf(stderr, "serve trace: served %llu; last poll: round %llu posted-seen %llu polls %llu\n",
                     (unsigned long long)vload(&m->sc->served),
                     (unsigned long long)vload(&m->sc->trace[1]), (unsigned long long)vload(&m->sc->trace[2]),
                     (unsigned long long)vload(&m->sc->trace[3]));
    uint64_t rung = 0;  // the last rung round + 1
    for (int i = 0; m->sc && i < NB; i++) rung = std::max<uint64_t>(rung, vload(&m->sc->door[i]) >> 32);
    out[0] = rung;
    out[1] = m->sc ? vload(&m->sc->served) : 0;
    out[2] = m->sc ? vload(&m->sc->exited) : 0;
    out[3] = m->session;
    out[4] = m->srv_running ? 1 : 0;
    out[5] = m->completed.load();
    out[6] = m->launched.load();
    out[7] = m->open.load();
    return NRG_OK;
}

// (tests) round phase sums: {rounds, ns open -> sealed, ns sealed -> posted/launched, ns posted ->
// completion seen by the combiner thread}
extern "C" int nrg_test_combiner_times(nrg_combiner* m, uint64_t out[4]) {
    if (!m || !out) return NRG_E_INVAL;
    out[0] = m->t_n;
    out[1] = m->t_gather;
    out[2] = m->t_enqueue;
    out[3] = m->t_gpu;
    return NRG_OK;
}

// GPU rounds combined so far and the ops they carried.
extern "C" int nrg_combiner_stats(nrg_combiner* m, uint64_t* rounds, uint64_t* ops) {
    if (!m || !rounds || !ops) return NRG_E_INVAL;
    *rounds = m->rounds.load(std::memory_order_relaxed);
    *ops = m->ops.load(std::memory_order_relaxed);
    return NRG_OK;
}
