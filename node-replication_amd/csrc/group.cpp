// group.cpp — multi-GPU replica groups: the write segments of a round are all-gathered with RCCL
// over xGMI and every replica replays the identical global log (include/nrgpu.h, nrg_group_*).
//
// Reference: the shared Log of nr/src/log.rs, read by every replica's exec loop
// (nr/src/log.rs:494-511, :473-524) through cache-coherent memory. Here each GPU keeps its own
// copy of the log; one ncclAllGather per round moves the new entries to every copy, in rank
// order, which is the round's deterministic global log order.
//
// Per member and round e (b = e % NBUF):
//   comm stream : wait(input ready) -> wait(freed[b]) -> [pad copy] -> ncclAllGather -> gathered[b]
//   replica     : wait(gathered[b]) -> Log::append + Log::exec + reads (replay kernels) -> freed[b]
// The comm stream never waits for a replay except through freed[b] (NBUF rounds back), so the
// all-gather of round e+1 runs while round e replays.
//
// RCCL is resolved with dlopen at the first group call: the process's own librccl.so.1 when one
// is already loaded (torch ships one), else the system's. libnrgpu.so itself does not link it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "collectives.hpp"
#include "internal.hpp"
#include "../../include/nrgpu_testing.h"

namespace {

using Rccl = nrg::Collectives;

std::mutex g_rccl_mu;
bool g_rccl_tried = false;
Rccl g_rccl;
bool g_rccl_ok = false;

const Rccl* rccl() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (!g_rccl_tried) {
        g_rccl_tried = true;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (h) {
            Rccl r;
            r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
            r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
            r.init_all = (decltype(r.init_all))dlsym(h, "ncclCommInitAll");
            r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
            r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
            r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
            r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
            r.send = (decltype(r.send))dlsym(h, "ncclSend");
            r.recv = (decltype(r.recv))dlsym(h, "ncclRecv");
            r.abort = (decltype(r.abort))dlsym(h, "ncclCommAbort");
            g_rccl_ok = r.get_unique_id && r.init_rank && r.init_all && r.all_gather && r.group_start &&
                        r.group_end && r.destroy;
            if (g_rccl_ok) g_rccl = r;
        }
    }
    return g_rccl_ok ? &g_rccl : nullptr;
}

// nrg_test_loopback_collectives: groups created from now on use loopback.cpp instead of RCCL
std::atomic<int> g_loopback{0};

// the collectives a new group binds to (kept by the group for its lifetime)
const Rccl* backend() { return g_loopback.load() ? nrg::loopback_collectives() : rccl(); }

constexpr int NBUF = 3;  // gathered-log buffers in rotation per member

// A device buffer grown on demand; a reallocation first drains the streams that may use it.
struct DBuf {
    void* p = nullptr;
    uint64_t bytes = 0;
};

// Partitioned rounds (nrg_group_partitioned_round*): buffers of one member. A round's partition
// A round lives over three calls in the pipelined form (post, stage A, stage B: see pt_post), so its
// partition output and count exchange (PtPar) rotate over PT_DEPTH slots and what the owner
// received and answered (PtRecv) over two.
enum PtBuf { PB_AVAL, PB_AFOUND, PB_APREV, PB_APREVF, PB_ST, PB_ALLST, PB_DESC, PB_N };
enum PtPar { PP_POUT, PP_PPOS, PP_KOUT, PP_GPOS, PP_CNT, PP_ALLCNT, PP_N };
enum PtRecv { PR_RPUT, PR_RKEY, PR_RVAL, PR_RFOUND, PR_RPREV, PR_RPREVF, PR_N };
constexpr int PT_DEPTH = 3;

// A round's send/recv plan (stage A), kept for its answers (stage B).
struct PtPlan {
    std::vector<uint64_t> pto, gto, pfrom, gfrom, pfrom_off, gfrom_off;
    uint64_t rp = 0, rk = 0;
};

constexpr uint64_t GC_FROM_HEAD = 32 * 256;  // nr/src/log.rs:36 (the ring keeps this much free)

struct Member {
    nrg_ctx* ctx = nullptr;
    int rank = 0;
    ncclComm_t comm = nullptr;
    hipStream_t cstream = nullptr;  // library-owned: pad copies + all-gathers
    hipStream_t in_stream = nullptr;
    bool in_set = false;
    hipEvent_t in_ev = nullptr;
    void* gbuf[NBUF] = {};
    uint64_t gbytes[NBUF] = {};
    hipEvent_t gathered[NBUF] = {};
    hipEvent_t freed[NBUF] = {};
    bool used[NBUF] = {};
    void* sbuf = nullptr;  // padded send copy when a segment is shorter than the stride
    uint64_t sbytes = 0;
    DBuf pt[PB_N];                  // partitioned rounds
    DBuf pp[PT_DEPTH][PP_N];        // ... by round slot (round % PT_DEPTH)
    DBuf rv[2][PR_N];               // ... by round parity
    uint64_t* h_cnt[PT_DEPTH] = {};  // pinned: [nranks][2 * nranks + XW_N] counts, capacities, flags
    hipEvent_t cnt_ev[PT_DEPTH] = {};  // the counts of that slot are in h_cnt
    nrg_round pr[PT_DEPTH] = {};       // the caller's part of the round of that slot
    uint64_t cap_p[PT_DEPTH] = {}, cap_k[PT_DEPTH] = {};  // its owner-region capacities (n, n_gets)
    PtPlan plan[PT_DEPTH];
    uint32_t pt_epoch = 0;      // look-back descriptor tag of the last fused partition
    hipStream_t pstream = nullptr;  // a one-rank group's partitions and route-backs, beside the replay
    hipEvent_t pin_ev = nullptr;    // the replica stream's work up to a post (inputs, older rounds)
    hipEvent_t rd_ev = nullptr;     // a one-rank group: the replay launch that answered a round's reads
    uint64_t xwords[8] = {};    // this rank's host words of the exchange
    uint64_t xw1[PT_DEPTH][8] = {};  // a one-rank group: the words of the round of that slot (its
                                     // "exchange" needs no wait: its counts are its own n, n_gets)
    hipEvent_t pt_ev = nullptr;
    // Round headers and the length exchange (allocated at join, so a round cannot fail on them):
    //   hdr[b]  {n, fingerprint of seg_lens} sent with round b's segment; ghdr[b] every rank's
    //   lx      {n, local error} for a round whose lengths are exchanged; glx every rank's
    uint64_t* hdr[NBUF] = {};
    uint64_t* ghdr[NBUF] = {};
    uint64_t* lx = nullptr;
    uint64_t* glx = nullptr;
    uint64_t* h_glx = nullptr;  // pinned host copy of glx
    void* xmem = nullptr;
};

int hip_rc(hipError_t e) { return e == hipSuccess ? NRG_OK : (e == hipErrorOutOfMemory ? NRG_E_NOMEM : NRG_E_HIP); }

#define GCHK(x)                          \
    do {                                 \
        hipError_t _e = (x);             \
        if (_e != hipSuccess) return hip_rc(_e); \
    } while (0)

#define RCHK(x)                                   \
    do {                                          \
        int _r = (x);                             \
        if (_r != NRG_OK) return _r;              \
    } while (0)

int grow_buf(Member& m, DBuf& d, uint64_t bytes) {
    if (d.bytes >= bytes) return NRG_OK;
    GCHK(hipStreamSynchronize(m.cstream));
    GCHK(hipStreamSynchronize(m.ctx->stream));
    if (m.pstream) GCHK(hipStreamSynchronize(m.pstream));  // a one-rank group's partitions
    if (d.p) GCHK(hipFree(d.p));
    d.p = nullptr;
    d.bytes = 0;
    uint64_t b = bytes < 4096 ? 4096 : bytes + bytes / 4;  // headroom: rounds vary in size
    GCHK(hipMalloc(&d.p, b));
    d.bytes = b;
    return NRG_OK;
}
int grow(Member& m, PtBuf k, uint64_t bytes) { return grow_buf(m, m.pt[k], bytes); }

// `to` waits for the work queued on `from` so far
int order(Member& m, hipStream_t from, hipStream_t to) {
    GCHK(hipEventRecord(m.pt_ev, from));
    GCHK(hipStreamWaitEvent(to, m.pt_ev, 0));
    return NRG_OK;
}

// Exchange words per rank (u64) of a partitioned round: [0, G) Puts per owner, [G, 2G) Gets per
// owner, then
enum : uint64_t {
    XW_PREV = 0,    // 1 when this rank wants its Puts' previous values
    XW_RP_CAP = 1,  // received Puts its buffers hold now
    XW_RK_CAP = 2,  // received Get keys its buffers hold now
    XW_ERR = 3,     // -NRG_E_* of a local failure before the exchange, else 0
    XW_N = 4,
};

int member_init(Member& m, int nranks) {
    int r = nrg::ctx_use_device(m.ctx);
    if (r) return r;
    GCHK(hipStreamCreateWithFlags(&m.cstream, hipStreamNonBlocking));
    GCHK(hipEventCreateWithFlags(&m.in_ev, hipEventDisableTiming));
    GCHK(hipEventCreateWithFlags(&m.pt_ev, hipEventDisableTiming));
    for (int q = 0; q < PT_DEPTH; q++) GCHK(hipEventCreateWithFlags(&m.cnt_ev[q], hipEventDisableTiming));
    GCHK(hipEventCreateWithFlags(&m.pin_ev, hipEventDisableTiming));
    GCHK(hipEventCreateWithFlags(&m.rd_ev, hipEventDisableTiming));
    GCHK(hipStreamCreateWithFlags(&m.pstream, hipStreamNonBlocking));
    for (int b = 0; b < NBUF; b++) {
        GCHK(hipEventCreateWithFlags(&m.gathered[b], hipEventDisableTiming));
        GCHK(hipEventCreateWithFlags(&m.freed[b], hipEventDisableTiming));
    }
    const uint64_t G = (uint64_t)nranks;
    GCHK(hipMalloc(&m.xmem, (NBUF * (2 + 2 * G) + 2 + 2 * G) * 8));
    uint64_t* x = (uint64_t*)m.xmem;
    for (int b = 0; b < NBUF; b++, x += 2 + 2 * G) {
        m.hdr[b] = x;
        m.ghdr[b] = x + 2;
    }
    m.lx = x;
    m.glx = x + 2;
    GCHK(hipHostMalloc(&m.h_glx, 2 * G * 8, hipHostMallocDefault));
    // the fixed-size buffers of a partitioned round's count and status exchanges
    const uint64_t CW = 2 * G + XW_N;
    for (int q = 0; q < PT_DEPTH; q++) {
        if ((r = grow_buf(m, m.pp[q][PP_CNT], CW * 8)) || (r = grow_buf(m, m.pp[q][PP_ALLCNT], G * CW * 8))) return r;
        // mapped: a one-rank group's partition writes its counts here directly (no exchange)
        GCHK(hipHostMalloc(&m.h_cnt[q], G * CW * 8, hipHostMallocMapped));
    }
    if ((r = grow(m, PB_ST, 8)) || (r = grow(m, PB_ALLST, G * 8))) return r;
    return NRG_OK;
}

// Round header check (on the comm stream, after the all-gather): every rank's {n, fingerprint}
// must match this rank's view of the round. A mismatch latches ERR_GROUP in the replica, which
// nrg_sync / nrg_group_sync report as NRG_E_INVAL.
struct LensArg {
    uint64_t v[64];
};
__global__ void grp_check_kernel(const uint64_t* ghdr, uint32_t G, LensArg lens, uint64_t fp, uint32_t* err) {
    const uint32_t r = threadIdx.x;
    if (r < G && (ghdr[2 * r] != lens.v[r] || ghdr[2 * r + 1] != fp)) atomicOr(err, nrg::ERR_GROUP);
}

// dst[0] = a, dst[1] = b in stream order (kernel arguments are captured at launch)
__global__ void grp_put2_kernel(uint64_t* dst, uint64_t a, uint64_t b) {
    if (threadIdx.x < 2) dst[threadIdx.x] = threadIdx.x ? b : a;
}

// fingerprint of a round's segment lengths (every rank must pass the same ones)
uint64_t lens_fp(const std::vector<uint64_t>& lens) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ lens.size();
    for (uint64_t l : lens) h = nrg::mix64(h ^ l) + 0x632BE59BD9B4E019ull;
    return h;
}

void member_free(Member& m, const Rccl* R) {
    if (!m.ctx) return;
    (void)nrg::ctx_use_device(m.ctx);
    if (m.cstream) (void)hipStreamSynchronize(m.cstream);
    if (m.comm && R) R->destroy(m.comm);
    for (int b = 0; b < NBUF; b++) {
        if (m.gbuf[b]) (void)hipFree(m.gbuf[b]);
        if (m.gathered[b]) (void)hipEventDestroy(m.gathered[b]);
        if (m.freed[b]) (void)hipEventDestroy(m.freed[b]);
    }
    if (m.sbuf) (void)hipFree(m.sbuf);
    if (m.xmem) (void)hipFree(m.xmem);
    if (m.h_glx) (void)hipHostFree(m.h_glx);
    for (DBuf& d : m.pt)
        if (d.p) (void)hipFree(d.p);
    for (int q = 0; q < PT_DEPTH; q++) {
        for (DBuf& d : m.pp[q])
            if (d.p) (void)hipFree(d.p);
        if (m.h_cnt[q]) (void)hipHostFree(m.h_cnt[q]);
        if (m.cnt_ev[q]) (void)hipEventDestroy(m.cnt_ev[q]);
    }
    for (int q = 0; q < 2; q++)
        for (DBuf& d : m.rv[q])
            if (d.p) (void)hipFree(d.p);
    if (m.pt_ev) (void)hipEventDestroy(m.pt_ev);
    if (m.pstream) (void)hipStreamSynchronize(m.pstream);
    if (m.pstream) (void)hipStreamDestroy(m.pstream);
    if (m.pin_ev) (void)hipEventDestroy(m.pin_ev);
    if (m.rd_ev) (void)hipEventDestroy(m.rd_ev);
    if (m.in_ev) (void)hipEventDestroy(m.in_ev);
    if (m.cstream) (void)hipStreamDestroy(m.cstream);
    m = Member{};
}

}  // namespace

struct nrg_group {
    const Rccl* R = nullptr;  // RCCL, or the test loopback (fixed at creation)
    int nranks = 0;
    int rank0 = 0;
    bool owns = false;  // replicas opened by nrg_group_open
    std::vector<Member> m;
    uint64_t round = 0;
    uint32_t timeout_ms = NRG_GROUP_DEFAULT_TIMEOUT_MS;  // deadline of every wait on the peers
    int broken = NRG_OK;  // sticky: a timed-out collective or disagreeing ranks end the group
    // partitioned rounds: posted (partition + count exchange), through stage A (payload to the
    // owners, replay with its reads deferred), through stage B (answers back, route-back)
    uint64_t pt_posted = 0, pt_a = 0, pt_b = 0;
    bool pt_drop[PT_DEPTH] = {};  // the round failed in stage A (an agreed error): no stage B
    char diag[256] = {};  // what broke it (nrg_group_last_error)
};

namespace {

// The group cannot go on: remember why, give up on the communicators (RCCL's abort ends a
// collective a peer never posted, so the streams drain and close() cannot hang), and return `code`.
int group_fail(nrg_group* g, int code, const char* what) {
    if (g->broken == NRG_OK) {
        g->broken = code;
        std::snprintf(g->diag, sizeof g->diag, "nrg_group rank %d of %d, round %llu: %s", g->rank0, g->nranks,
                      (unsigned long long)g->round, what);
        std::fprintf(stderr, "%s\n", g->diag);
        if (code == NRG_E_TIMEOUT && g->R && g->R->abort)
            for (Member& m : g->m)
                if (m.comm) {
                    (void)g->R->abort(m.comm);
                    m.comm = nullptr;
                }
    }
    return g->broken;
}

// ncclGroupEnd with the group's deadline (the loopback blocks there until its peers post; RCCL
// enqueues and returns, and a missing peer shows up in the stream waits below)
int group_end(nrg_group* g, const char* phase) {
    if (g->R->set_timeout_ms) g->R->set_timeout_ms(g->timeout_ms);
    const ncclResult_t r = g->R->group_end();
    if (r == ncclSuccess) return NRG_OK;
    char what[192];
    if (r == ncclSystemError && g->R->set_timeout_ms) {
        std::snprintf(what, sizeof what, "%s: a peer rank did not post its part within %u ms", phase, g->timeout_ms);
        return group_fail(g, NRG_E_TIMEOUT, what);
    }
    std::snprintf(what, sizeof what, "%s: collective failed (ncclResult %d)", phase, (int)r);
    return group_fail(g, NRG_E_COMM, what);
}

// Wait until `s` drains, at most the group's deadline from now. A stream that does not drain is
// one whose collective a peer never joined (or a hung device): the group fails with NRG_E_TIMEOUT.
template <typename Q>
int wait_until(nrg_group* g, Q query, const char* phase) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const auto dl = t0 + std::chrono::milliseconds(g->timeout_ms);
    for (uint32_t spin = 0;; spin++) {
        const hipError_t e = query();
        if (e == hipSuccess) return NRG_OK;
        if (e != hipErrorNotReady) return hip_rc(e);
        const auto now = clk::now();
        if (now >= dl) {
            char what[192];
            std::snprintf(what, sizeof what, "%s did not complete within %u ms (a peer rank never joined the collective?)",
                          phase, g->timeout_ms);
            return group_fail(g, NRG_E_TIMEOUT, what);
        }
        // a host round trip is short: spin for the first 200 us, then back off
        if (now - t0 > std::chrono::microseconds(200))
            std::this_thread::sleep_for(std::chrono::microseconds(spin < 2000 ? 20 : 500));
    }
}
int wait_stream(nrg_group* g, hipStream_t s, const char* phase) {
    return wait_until(g, [s] { return hipStreamQuery(s); }, phase);
}
int wait_event(nrg_group* g, hipEvent_t ev, const char* phase) {
    return wait_until(g, [ev] { return hipEventQuery(ev); }, phase);
}

}  // namespace

extern "C" {

int nrg_test_loopback_collectives(int on) {
    g_loopback.store(on ? 1 : 0);
    return NRG_OK;
}

int nrg_group_unique_id(uint8_t id[NRG_GROUP_ID_BYTES]) {
    if (!id) return NRG_E_INVAL;
    const Rccl* R = backend();
    if (!R) return NRG_E_COMM;
    ncclUniqueId u;
    if (R->get_unique_id(&u) != ncclSuccess) return NRG_E_COMM;
    static_assert(sizeof(u) == NRG_GROUP_ID_BYTES, "ncclUniqueId size");
    std::memcpy(id, &u, NRG_GROUP_ID_BYTES);
    return NRG_OK;
}

int nrg_group_join(nrg_ctx* replica, const uint8_t id[NRG_GROUP_ID_BYTES], int nranks, int rank, nrg_group** out) {
    if (!replica || !id || !out || nranks < 1 || rank < 0 || rank >= nranks || nranks > 64) return NRG_E_INVAL;
    *out = nullptr;
    const Rccl* R = backend();
    if (!R) return NRG_E_COMM;
    nrg_group* g = new (std::nothrow) nrg_group();
    if (!g) return NRG_E_NOMEM;
    g->R = R;
    g->nranks = nranks;
    g->rank0 = rank;
    g->m.resize(1);
    Member& m = g->m[0];
    m.ctx = replica;
    m.rank = rank;
    int r = member_init(m, nranks);
    ncclUniqueId u;
    std::memcpy(&u, id, NRG_GROUP_ID_BYTES);
    if (r == NRG_OK && R->init_rank(&m.comm, nranks, u, rank) != ncclSuccess) r = NRG_E_COMM;
    if (r != NRG_OK) {
        member_free(m, R);
        delete g;
        return r;
    }
    *out = g;
    return NRG_OK;
}

int nrg_group_open(const int* devices, int n, const nrg_config* cfg, nrg_group** out) {
    if (!devices || n < 1 || n > 64 || !cfg || !out) return NRG_E_INVAL;
    *out = nullptr;
    const Rccl* R = backend();
    if (!R) return NRG_E_COMM;
    nrg_group* g = new (std::nothrow) nrg_group();
    if (!g) return NRG_E_NOMEM;
    g->R = R;
    g->nranks = n;
    g->rank0 = 0;
    g->owns = true;
    g->m.resize(n);
    int r = NRG_OK;
    for (int i = 0; i < n && r == NRG_OK; i++) {
        nrg_config c = *cfg;
        c.replica_id = (uint32_t)i + 1;  // Log::register hands out ids from 1 (nr/src/log.rs:272-292)
        r = nrg_open(devices[i], &c, &g->m[i].ctx);
        g->m[i].rank = i;
        if (r == NRG_OK) r = member_init(g->m[i], n);
    }
    if (r == NRG_OK) {
        std::vector<ncclComm_t> comms(n);
        if (R->init_all(comms.data(), n, devices) != ncclSuccess) r = NRG_E_COMM;
        else
            for (int i = 0; i < n; i++) g->m[i].comm = comms[i];
    }
    if (r != NRG_OK) {
        nrg_group_close(g);
        return r;
    }
    *out = g;
    return NRG_OK;
}

int nrg_group_close(nrg_group* g) {
    if (!g) return NRG_E_INVAL;
    const Rccl* R = g->R;
    for (Member& m : g->m) {
        nrg_ctx* c = m.ctx;
        member_free(m, R);
        if (g->owns && c) nrg_close(c);
    }
    delete g;
    return NRG_OK;
}

int nrg_group_info(const nrg_group* g, int* nranks, int* nlocal, int* rank0) {
    if (!g) return NRG_E_INVAL;
    if (nranks) *nranks = g->nranks;
    if (nlocal) *nlocal = (int)g->m.size();
    if (rank0) *rank0 = g->rank0;
    return NRG_OK;
}

nrg_ctx* nrg_group_replica(nrg_group* g, int member) {
    if (!g || member < 0 || member >= (int)g->m.size()) return nullptr;
    return g->m[member].ctx;
}

int nrg_group_set_input_stream(nrg_group* g, int member, void* s) {
    if (!g || member < 0 || member >= (int)g->m.size()) return NRG_E_INVAL;
    g->m[member].in_stream = (hipStream_t)s;
    g->m[member].in_set = true;
    return NRG_OK;
}

// Every rank's segment length of a round whose caller gave none (seg_lens == NULL, one member per
// process): each rank all-gathers {n, local error} and the host reads them back (one host round
// trip). A rank whose own part is bad makes every rank return NRG_E_INVAL, so no rank is left
// inside a collective its peers never post.
static int exchange_lengths(nrg_group* g, const nrg_round* rounds, const std::vector<int>& bad,
                            std::vector<uint64_t>& lens) {
    const Rccl* R = g->R;
    const int nl = (int)g->m.size(), G = g->nranks;
    for (int i = 0; i < nl; i++) {
        Member& m = g->m[i];
        RCHK(nrg::ctx_use_device(m.ctx));
        grp_put2_kernel<<<1, 64, 0, m.cstream>>>(m.lx, rounds[i].n, bad[i] ? 1 : 0);
        GCHK(hipGetLastError());
    }
    if (R->group_start() != ncclSuccess) return NRG_E_COMM;
    ncclResult_t res = ncclSuccess;
    for (int i = 0; i < nl && res == ncclSuccess; i++)
        res = R->all_gather(g->m[i].lx, g->m[i].glx, 2, ncclUint64, g->m[i].comm, g->m[i].cstream);
    RCHK(group_end(g, "length exchange"));
    if (res != ncclSuccess) return group_fail(g, NRG_E_COMM, "length exchange: all-gather refused");
    for (int i = 0; i < nl; i++) {
        Member& m = g->m[i];
        RCHK(nrg::ctx_use_device(m.ctx));
        GCHK(hipMemcpyAsync(m.h_glx, m.glx, 2 * (uint64_t)G * 8, hipMemcpyDeviceToHost, m.cstream));
        RCHK(wait_stream(g, m.cstream, "length exchange"));
    }
    const uint64_t* H = g->m[0].h_glx;  // identical on every rank
    bool any_bad = false;
    for (int r = 0; r < G; r++) {
        lens[r] = H[2 * r];
        any_bad |= H[2 * r + 1] != 0;
    }
    return any_bad ? NRG_E_INVAL : NRG_OK;
}

int nrg_group_round_async(nrg_group* g, const nrg_round* rounds, const uint64_t* seg_lens) {
    if (!g || !rounds) return NRG_E_INVAL;
    if (g->broken) return g->broken;
    const Rccl* R = g->R;
    if (!R) return NRG_E_COMM;
    const int nl = (int)g->m.size(), G = g->nranks;
    const uint32_t kind = g->m[0].ctx->cfg.ds_kind;
    const uint64_t rb = g->m[0].ctx->rec_bytes;
    // every rank's segment length, in rank order
    std::vector<uint64_t> lens(G);
    std::vector<int> bad(nl, 0);
    for (int i = 0; i < nl; i++)
        bad[i] = g->m[i].ctx->cfg.ds_kind != kind || (rounds[i].n && !rounds[i].recs);
    // Three ways to know them:
    //   whole   this process drives every rank: the members' n (or seg_lens, checked against them)
    //   given   seg_lens from the caller, who promises every rank passes the same array: a header
    //           {n, fingerprint of seg_lens} travels with each segment and a kernel on the comm
    //           stream compares it with this rank's view (mismatch -> NRG_E_INVAL at the next sync)
    //   exchanged  seg_lens == NULL: exchange_lengths (one host round trip)
    const bool whole = nl == G;
    const bool given = !whole && seg_lens;
    if (whole) {
        for (int i = 0; i < nl; i++) {
            const uint64_t n = rounds[i].n;
            if (bad[i] || (seg_lens && seg_lens[g->m[i].rank] != n)) return NRG_E_INVAL;
            lens[g->m[i].rank] = n;
        }
    } else if (given) {
        for (int r = 0; r < G; r++) lens[r] = seg_lens[r];
        for (int i = 0; i < nl; i++) bad[i] |= rounds[i].n != lens[g->m[i].rank];
    } else {
        RCHK(exchange_lengths(g, rounds, bad, lens));
    }
    uint64_t stride = 0;
    for (uint64_t l : lens) stride = l > stride ? l : stride;
    const uint64_t fp = lens_fp(lens);
    LensArg la{};
    for (int r = 0; r < G; r++) la.v[r] = lens[r];
    std::vector<uint32_t> origins(G);
    for (int r = 0; r < G; r++) origins[r] = (uint32_t)r + 1;
    const int b = (int)(g->round % NBUF);
    const uint64_t seg_bytes = stride * rb;
    std::vector<const void*> send(nl);
    if (stride || given) {
        for (int i = 0; i < nl; i++) {
            Member& m = g->m[i];
            const nrg_round& x = rounds[i];
            RCHK(nrg::ctx_use_device(m.ctx));
            // the all-gather reads the caller's segment: ordered after its producer
            GCHK(hipEventRecord(m.in_ev, m.in_set ? m.in_stream : m.ctx->stream));
            GCHK(hipStreamWaitEvent(m.cstream, m.in_ev, 0));
            // and it overwrites gathered buffer b: ordered after the replay that read it
            if (m.used[b]) GCHK(hipStreamWaitEvent(m.cstream, m.freed[b], 0));
            if (given) grp_put2_kernel<<<1, 64, 0, m.cstream>>>(m.hdr[b], bad[i] ? ~0ull : x.n, fp);
            GCHK(hipGetLastError());
            if (!stride) continue;
            const uint64_t need = (uint64_t)G * seg_bytes;
            if (m.gbytes[b] < need) {
                RCHK(wait_stream(g, m.cstream, "gathered-buffer growth"));
                if (m.gbuf[b]) GCHK(hipFree(m.gbuf[b]));
                m.gbuf[b] = nullptr;
                m.gbytes[b] = 0;
                GCHK(hipMalloc(&m.gbuf[b], need));
                m.gbytes[b] = need;
            }
            if (x.n == stride && !bad[i]) {
                send[i] = x.recs;
            } else {  // pad a short segment to the common stride (a bad one sends zeros)
                if (m.sbytes < seg_bytes) {
                    RCHK(wait_stream(g, m.cstream, "send-buffer growth"));
                    if (m.sbuf) GCHK(hipFree(m.sbuf));
                    m.sbuf = nullptr;
                    m.sbytes = 0;
                    GCHK(hipMalloc(&m.sbuf, seg_bytes));
                    m.sbytes = seg_bytes;
                }
                const uint64_t keep = bad[i] ? 0 : x.n;
                if (keep) GCHK(hipMemcpyAsync(m.sbuf, x.recs, keep * rb, hipMemcpyDeviceToDevice, m.cstream));
                GCHK(hipMemsetAsync((char*)m.sbuf + keep * rb, 0, seg_bytes - keep * rb, m.cstream));
                send[i] = m.sbuf;
            }
        }
        if (R->group_start() != ncclSuccess) return NRG_E_COMM;
        ncclResult_t res = ncclSuccess;
        for (int i = 0; i < nl && res == ncclSuccess; i++) {
            Member& m = g->m[i];
            if (given) res = R->all_gather(m.hdr[b], m.ghdr[b], 2, ncclUint64, m.comm, m.cstream);
            if (stride && res == ncclSuccess)
                res = R->all_gather(send[i], m.gbuf[b], seg_bytes / 8, ncclUint64, m.comm, m.cstream);
        }
        RCHK(group_end(g, "segment all-gather"));
        if (res != ncclSuccess) return group_fail(g, NRG_E_COMM, "segment all-gather refused");
        if (given)
            for (int i = 0; i < nl; i++) {
                Member& m = g->m[i];
                RCHK(nrg::ctx_use_device(m.ctx));
                grp_check_kernel<<<1, 64, 0, m.cstream>>>(m.ghdr[b], (uint32_t)G, la, fp, &m.ctx->d_ctl->err);
                GCHK(hipGetLastError());
            }
    }
    int rc = NRG_OK;
    for (int i = 0; i < nl; i++) {
        Member& m = g->m[i];
        const nrg_round& x = rounds[i];
        nrg_ctx* c = m.ctx;
        RCHK(nrg::ctx_use_device(c));
        if (bad[i]) {  // took part in the collectives, replays nothing
            // Its peers replay the round (with this rank's segment as zeros) and latch ERR_GROUP;
            // the replicas now differ, so the group is over for every rank (sticky error).
            rc = group_fail(g, NRG_E_INVAL, "this rank's segment disagreed with seg_lens: replicas diverged");
            continue;
        }
        if (stride) {
            GCHK(hipEventRecord(m.gathered[b], m.cstream));
            GCHK(hipStreamWaitEvent(c->stream, m.gathered[b], 0));
        }
        int r = NRG_OK;
        if (kind == NRG_DS_HASHMAP) {
            if (stride)
                r = nrg_hashmap_round_segments_async(c, (const nrg_put*)m.gbuf[b], (uint32_t)G, stride, lens.data(),
                                                     origins.data(), (uint32_t)m.rank, x.get_keys, x.n_gets,
                                                     x.get_vals, x.get_found, (uint64_t*)x.resp, x.some);
            else
                r = nrg_hashmap_round_async(c, nullptr, 0, origins[m.rank], x.get_keys, x.n_gets, x.get_vals,
                                            x.get_found, nullptr, nullptr);
        } else if (stride) {
            std::vector<uint64_t> firsts(G);
            r = nrg_log_append_segments_async(c, m.gbuf[b], (uint32_t)G, stride, lens.data(), origins.data(),
                                              firsts.data());
            if (r == NRG_OK)
                r = nrg_log_exec_async(c, firsts[m.rank], firsts[m.rank] + lens[m.rank], x.resp, x.some);
        }
        if (r) return r;
        if (stride) {
            GCHK(hipEventRecord(m.freed[b], c->stream));
            m.used[b] = true;
        }
    }
    g->round++;
    return rc;
}

// ---- cnr-style key-partitioned rounds (cnr/src/replica.rs:430-445, :673-736) ----



// Partitioned rounds, pipelined over three calls (nrg_group_partitioned_round_async):
//   call e     post(e):    the fused partition of round e's Puts and Gets into owner regions
//                          (partition.hip pt_fused, which also writes the member's exchange words)
//                          and the all-gather of every rank's counts, copied to pinned host memory
//                          behind an event;
//   call e+1   stage A(e): its counts (landed long ago: no host wait in steady state), the plan,
//                          Puts and Get keys to their owners (RCCL send/recv; a rank's own part is a
//                          device copy, or none with one rank), the owner's replay with the reads
//                          deferred: they ride in round e+1's index launch (the replicated
//                          pipeline's overlap);
//   call e+2   stage B(e): (round e's reads were launched in stage A(e+1)) answers and previous
//                          values back to the ranks that asked, one route-back launch into the
//                          caller's order.
// Everything runs on the replica's stream. Every failure before a round's first send/recv is
// agreed on by all ranks (the same exchanged words): the round is dropped everywhere and the call
// that ran its stage A returns the error.
// A one-rank group owns every key, so its partition is the identity and so is the route-back:
// the owner's replay reads the caller's records and Get keys and answers straight into the
// caller's buffers -- no data moves, as a cnr replica with one log appends and replays in place
// (cnr/src/replica.rs:673-736). NRG_KNOB_EXP bit 16 (measurement) makes a one-rank group move
// its data like a multi-rank one: partition copy on the side stream, route-back launch.
static bool pt_ident(const nrg_group* g, const Member& m) { return g->nranks == 1 && !(m.ctx->exp & 0x10000); }

static int pt_post(nrg_group* g, const nrg_round* rounds, uint64_t e) {
    const Rccl* R = g->R;
    const int G = g->nranks, nl = (int)g->m.size();
    const int sl = (int)(e % PT_DEPTH), par = (int)(e & 1);
    const uint64_t CW = 2 * (uint64_t)G + XW_N;
    for (int i = 0; i < nl; i++) {
        Member& m = g->m[i];
        const nrg_round& x = rounds[i];
        nrg_ctx* c = m.ctx;
        int err = NRG_OK;
        if (c->cfg.ds_kind != NRG_DS_HASHMAP || (x.n && !x.recs) ||
            (x.n_gets && (!x.get_keys || !x.get_vals || !x.get_found)))
            err = NRG_E_INVAL;
        else if (x.n >= (1ull << 32) || x.n_gets >= (1ull << 32) || (uint64_t)G * x.n >= (1ull << 32) ||
                 (uint64_t)G * x.n_gets >= (1ull << 32))
            err = NRG_E_CAPACITY;  // positions are u32 owner-region offsets
        RCHK(nrg::ctx_use_device(c));
        if (m.in_set && m.in_stream != c->stream) RCHK(order(m, m.in_stream, c->stream));
        const uint64_t n = err ? 0 : x.n, k = err ? 0 : x.n_gets;
        if (err == NRG_OK) {
            DBuf* pp = m.pp[sl];
            const uint64_t bytes[] = {G * n * 16, n * 4, G * k * 8, k * 4};
            const PtPar which[] = {PP_POUT, PP_PPOS, PP_KOUT, PP_GPOS};
            for (int q = 0; q < 4 && err == NRG_OK; q++) err = grow_buf(m, pp[which[q]], bytes[q]);
            if (err == NRG_OK) err = grow(m, PB_DESC, nrg::pt_desc_words(n, k, (uint32_t)G) * 8);
            // owner-region answer buffers (a single rank's answers need none: they stay in RVAL)
            if (err == NRG_OK && G > 1) {
                const PtBuf ans[] = {PB_AVAL, PB_AFOUND, PB_APREV, PB_APREVF};
                const uint64_t ab[] = {G * k * 8, G * k, G * n * 8, G * n};
                for (int q = 0; q < 4 && err == NRG_OK; q++) err = grow(m, ans[q], ab[q]);
            }
        }
        uint64_t* w = m.xwords;
        w[XW_PREV] = (x.resp && x.some) ? 1 : 0;
        // receive capacities of the round's parity (one rank replays straight from its partition
        // output: no RPUT / RKEY)
        const DBuf* rv = m.rv[par];
        const uint64_t rp_own = std::min(rv[PR_RPREV].bytes / 8, rv[PR_RPREVF].bytes);
        const uint64_t rk_own = std::min(rv[PR_RVAL].bytes / 8, rv[PR_RFOUND].bytes);
        w[XW_RP_CAP] = G == 1 ? rp_own : std::min(rv[PR_RPUT].bytes / 16, rp_own);
        w[XW_RK_CAP] = G == 1 ? rk_own : std::min(rv[PR_RKEY].bytes / 8, rk_own);
        w[XW_ERR] = (uint64_t)(-err);
        for (int q = 0; q < XW_N; q++) m.xw1[sl][q] = w[q];
        // A one-rank group partitions on a side stream, after everything queued on the replica's
        // stream so far (the inputs, the slot's previous round), beside the previous round's
        // replay queued next (with RCCL the partition stays in line: the count exchange must keep
        // its place among the communicator's operations)
        if (pt_ident(g, m)) {  // nothing to partition (the counts are n, n_gets; the words are xw1)
            m.xw1[sl][XW_RP_CAP] = m.xw1[sl][XW_RK_CAP] = ~0ull;  // nothing received: no buffer to grow
            m.pr[sl] = x;
            m.cap_p[sl] = err ? 0 : n;
            m.cap_k[sl] = err ? 0 : k;
            continue;
        }
        hipStream_t ps = c->stream;
        if (G == 1) {
            ps = m.pstream;
            GCHK(hipEventRecord(m.pin_ev, c->stream));
            GCHK(hipStreamWaitEvent(ps, m.pin_ev, 0));
        }
        if (++m.pt_epoch >= (1u << 22)) {  // the descriptor tag wraps: clear the stale ones once
            m.pt_epoch = 1;
            if (m.pt[PB_DESC].p) GCHK(hipMemsetAsync(m.pt[PB_DESC].p, 0, m.pt[PB_DESC].bytes, ps));
        }
        const bool ok = err == NRG_OK;
        const hipError_t he = nrg::pt_fused(ps, (const uint64_t*)x.recs, ok ? n : 0, n,
                                            (uint64_t*)m.pp[sl][PP_POUT].p, (uint32_t*)m.pp[sl][PP_PPOS].p,
                                            x.get_keys, ok ? k : 0, k, (uint64_t*)m.pp[sl][PP_KOUT].p,
                                            (uint32_t*)m.pp[sl][PP_GPOS].p, (uint64_t*)m.pt[PB_DESC].p, (uint32_t)G,
                                            m.pt_epoch, G == 1 ? m.h_cnt[sl] : (uint64_t*)m.pp[sl][PP_CNT].p, w,
                                            XW_N);
        if (he != hipSuccess) return hip_rc(he);
        m.pr[sl] = x;
        m.cap_p[sl] = n;
        m.cap_k[sl] = k;
    }
    if (G > 1) {  // (one rank's all-gather is the identity: its partition wrote h_cnt itself)
        if (R->group_start() != ncclSuccess) return NRG_E_COMM;
        ncclResult_t res = ncclSuccess;
        for (int i = 0; i < nl && res == ncclSuccess; i++)
            res = R->all_gather(g->m[i].pp[sl][PP_CNT].p, g->m[i].pp[sl][PP_ALLCNT].p, CW, ncclUint64,
                                g->m[i].comm, g->m[i].ctx->stream);
        RCHK(group_end(g, "partitioned count exchange"));
        if (res != ncclSuccess) return group_fail(g, NRG_E_COMM, "partitioned count exchange refused");
    }
    for (int i = 0; i < nl; i++) {
        Member& m = g->m[i];
        RCHK(nrg::ctx_use_device(m.ctx));
        if (pt_ident(g, m)) continue;
        if (G > 1)
            GCHK(hipMemcpyAsync(m.h_cnt[sl], m.pp[sl][PP_ALLCNT].p, (uint64_t)G * CW * 8, hipMemcpyDeviceToHost,
                                m.ctx->stream));
        GCHK(hipEventRecord(m.cnt_ev[sl], G == 1 ? m.pstream : m.ctx->stream));
    }
    return NRG_OK;
}

static void* at(void* base, uint64_t off) { return (void*)((char*)base + off); }

static int pt_stage_a(nrg_group* g, uint64_t e) {
    const Rccl* R = g->R;
    const int G = g->nranks, nl = (int)g->m.size();
    const int sl = (int)(e % PT_DEPTH), par = (int)(e & 1);
    const uint64_t CW = 2 * (uint64_t)G + XW_N;
    g->pt_drop[sl] = true;  // until the round's payload has moved
    // A one-rank group owns every key: its counts are its own n and n_gets and its words are its
    // own, so the host does not wait for the partition (the replay waits for it on the device).
    uint64_t H1[2 + XW_N];
    for (int i = 0; i < nl; i++) {
        Member& m = g->m[i];
        RCHK(nrg::ctx_use_device(m.ctx));
        if (G == 1) {
            if (!pt_ident(g, m)) GCHK(hipStreamWaitEvent(m.ctx->stream, m.cnt_ev[sl], 0));  // (side stream)
            H1[0] = m.cap_p[sl];
            H1[1] = m.cap_k[sl];
            for (int q = 0; q < XW_N; q++) H1[2 + q] = m.xw1[sl][q];
        } else {
            RCHK(wait_event(g, m.cnt_ev[sl], "partitioned count exchange"));
        }
    }
    const uint64_t* H = G == 1 ? H1 : g->m[0].h_cnt[sl];  // identical on every rank
    auto word = [&](int s, uint64_t k) { return H[(size_t)s * CW + 2 * G + k]; };
    for (int s = 0; s < G; s++)
        if (word(s, XW_ERR)) return -(int)word(s, XW_ERR);  // the same answer on every rank
    bool any_prev = false, any_grow = false;
    for (int s = 0; s < G; s++) {
        any_prev |= word(s, XW_PREV) != 0;
        uint64_t rp = 0, rk = 0;  // what rank s receives
        for (int o = 0; o < G; o++) {
            rp += H[(size_t)o * CW + s];
            rk += H[(size_t)o * CW + G + s];
        }
        any_grow |= rp > word(s, XW_RP_CAP) || rk > word(s, XW_RK_CAP);
    }
    // member rank r sends its owner-o region to o and receives rank s's group for r at offset
    // sum_{s' < s} (rank order = the global log order)
    std::vector<int> grow_err(nl, NRG_OK);
    for (int i = 0; i < nl; i++) {
        Member& m = g->m[i];
        PtPlan& P = m.plan[sl];
        const int r = m.rank;
        P.pto.assign(G, 0), P.gto.assign(G, 0), P.pfrom.assign(G, 0), P.gfrom.assign(G, 0);
        P.pfrom_off.assign(G, 0), P.gfrom_off.assign(G, 0);
        uint64_t a = 0, b = 0, cq = 0, d = 0;
        for (int o = 0; o < G; o++) {
            P.pto[o] = H[(size_t)r * CW + o];
            P.gto[o] = H[(size_t)r * CW + G + o];
            P.pfrom[o] = H[(size_t)o * CW + r];
            P.gfrom[o] = H[(size_t)o * CW + G + r];
            a += P.pto[o], b += P.gto[o];
            P.pfrom_off[o] = cq, cq += P.pfrom[o];
            P.gfrom_off[o] = d, d += P.gfrom[o];
        }
        if (a != m.cap_p[sl] || b != m.cap_k[sl]) grow_err[i] = NRG_E_HIP;  // partition kernel disagrees
        P.rp = cq;
        P.rk = d;
        if (any_grow && grow_err[i] == NRG_OK) {
            RCHK(nrg::ctx_use_device(m.ctx));
            const PtRecv recv[] = {PR_RPUT, PR_RPREV, PR_RPREVF, PR_RKEY, PR_RVAL, PR_RFOUND};
            const uint64_t bytes[] = {G > 1 ? P.rp * 16 : 0, P.rp * 8, P.rp, G > 1 ? P.rk * 8 : 0, P.rk * 8, P.rk};
            for (int k = 0; k < 6 && grow_err[i] == NRG_OK; k++) grow_err[i] = grow_buf(m, m.rv[par][recv[k]], bytes[k]);
        }
    }
    ncclResult_t res = ncclSuccess;
    if (any_grow) {  // every rank knows a rank had to grow: all confirm before any send/recv
        for (int i = 0; i < nl; i++) {
            Member& m = g->m[i];
            RCHK(nrg::ctx_use_device(m.ctx));
            m.xwords[0] = (uint64_t)(-grow_err[i]);
            GCHK(hipMemcpyAsync(m.pt[PB_ST].p, m.xwords, 8, hipMemcpyHostToDevice, m.ctx->stream));
        }
        if (R->group_start() != ncclSuccess) return NRG_E_COMM;
        for (int i = 0; i < nl && res == ncclSuccess; i++)
            res = R->all_gather(g->m[i].pt[PB_ST].p, g->m[i].pt[PB_ALLST].p, 1, ncclUint64, g->m[i].comm,
                                g->m[i].ctx->stream);
        RCHK(group_end(g, "partitioned status exchange"));
        if (res != ncclSuccess) return group_fail(g, NRG_E_COMM, "partitioned status exchange refused");
        std::vector<uint64_t> st(G);
        for (int i = 0; i < nl; i++) {
            Member& m = g->m[i];
            RCHK(nrg::ctx_use_device(m.ctx));
            GCHK(hipMemcpyAsync(st.data(), m.pt[PB_ALLST].p, (uint64_t)G * 8, hipMemcpyDeviceToHost, m.ctx->stream));
            RCHK(wait_stream(g, m.ctx->stream, "partitioned status exchange"));
        }
        for (int s = 0; s < G; s++)
            if (st[s]) return -(int)st[s];
    } else {
        for (int i = 0; i < nl; i++)
            if (grow_err[i]) return grow_err[i];  // cannot happen: the counts come from the same kernel
    }
    g->pt_drop[sl] = false;
    // where member i's replay reads its Puts / Get keys
    auto rput_of = [&](int i) -> const void* {
        return pt_ident(g, g->m[i]) ? (const void*)g->m[i].pr[sl].recs
               : G == 1             ? g->m[i].pp[sl][PP_POUT].p
                                    : g->m[i].rv[par][PR_RPUT].p;
    };
    auto rkey_of = [&](int i) -> const void* {
        return pt_ident(g, g->m[i]) ? (const void*)g->m[i].pr[sl].get_keys
               : G == 1             ? g->m[i].pp[sl][PP_KOUT].p
                                    : g->m[i].rv[par][PR_RKEY].p;
    };
    if (G > 1) {
        // Puts and Get keys to their owners (own part: a device copy)
        if (R->group_start() != ncclSuccess) return NRG_E_COMM;
        for (int i = 0; i < nl && res == ncclSuccess; i++) {
            Member& m = g->m[i];
            const PtPlan& P = m.plan[sl];
            const uint64_t cp = m.cap_p[sl], ck = m.cap_k[sl];
            void *pout = m.pp[sl][PP_POUT].p, *kout = m.pp[sl][PP_KOUT].p;
            hipStream_t s = m.ctx->stream;
            for (int o = 0; o < G && res == ncclSuccess; o++) {
                if (o == m.rank) continue;
                if (P.pto[o]) res = R->send(at(pout, o * cp * 16), P.pto[o] * 2, ncclUint64, o, m.comm, s);
                if (res == ncclSuccess && P.pfrom[o])
                    res = R->recv(at(m.rv[par][PR_RPUT].p, P.pfrom_off[o] * 16), P.pfrom[o] * 2, ncclUint64, o,
                                  m.comm, s);
                if (res == ncclSuccess && P.gto[o]) res = R->send(at(kout, o * ck * 8), P.gto[o], ncclUint64, o, m.comm, s);
                if (res == ncclSuccess && P.gfrom[o])
                    res = R->recv(at(m.rv[par][PR_RKEY].p, P.gfrom_off[o] * 8), P.gfrom[o], ncclUint64, o, m.comm, s);
            }
        }
        RCHK(group_end(g, "partitioned send/recv of Puts and Gets"));
        if (res != ncclSuccess) return group_fail(g, NRG_E_COMM, "partitioned send/recv refused");
        for (int i = 0; i < nl; i++) {
            Member& m = g->m[i];
            const PtPlan& P = m.plan[sl];
            const int r = m.rank;
            RCHK(nrg::ctx_use_device(m.ctx));
            if (P.pto[r])
                GCHK(hipMemcpyAsync(at(m.rv[par][PR_RPUT].p, P.pfrom_off[r] * 16),
                                    at(m.pp[sl][PP_POUT].p, r * m.cap_p[sl] * 16), P.pto[r] * 16,
                                    hipMemcpyDeviceToDevice, m.ctx->stream));
            if (P.gto[r])
                GCHK(hipMemcpyAsync(at(m.rv[par][PR_RKEY].p, P.gfrom_off[r] * 8),
                                    at(m.pp[sl][PP_KOUT].p, r * m.cap_k[sl] * 8), P.gto[r] * 8,
                                    hipMemcpyDeviceToDevice, m.ctx->stream));
        }
    }
    // each owner replays the Puts it received (rank order) and answers the Gets it received; the
    // reads (and a stamp round's apply) are deferred into the next round's first launch. A skewed
    // round can hand one owner more Puts than its max_batch (or ring) takes in one replay:
    // consecutive rounds of at most that many, the Gets answered after the last.
    for (int i = 0; i < nl; i++) {
        Member& m = g->m[i];
        const PtPlan& P = m.plan[sl];
        nrg_ctx* c = m.ctx;
        RCHK(nrg::ctx_use_device(c));
        const uint64_t ring_room = c->log_size > 2 * GC_FROM_HEAD ? c->log_size - GC_FROM_HEAD : GC_FROM_HEAD;
        const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(c->cfg.max_batch, ring_room));
        const nrg_put* rput = (const nrg_put*)rput_of(i);
        const bool ident = pt_ident(g, m);
        const nrg_round& x = m.pr[sl];
        // (identity: the caller's own answer buffers, and previous values only if it asked)
        uint64_t* rprev = ident ? (x.resp && x.some ? (uint64_t*)x.resp : nullptr)
                                : any_prev ? (uint64_t*)m.rv[par][PR_RPREV].p : nullptr;
        uint8_t* rprevf = ident ? (x.resp && x.some ? x.some : nullptr)
                                : any_prev ? (uint8_t*)m.rv[par][PR_RPREVF].p : nullptr;
        uint64_t* rval = ident ? x.get_vals : (uint64_t*)m.rv[par][PR_RVAL].p;
        uint8_t* rfound = ident ? x.get_found : (uint8_t*)m.rv[par][PR_RFOUND].p;
        uint64_t off = 0;
        do {
            const uint64_t n = std::min(chunk, P.rp - off);
            const bool last = off + n == P.rp;
            if (n || (last && P.rk))
                RCHK(nrg_hashmap_round_async(c, rput + off, n, (uint32_t)m.rank + 1,
                                             last ? (const uint64_t*)rkey_of(i) : nullptr, last ? P.rk : 0,
                                             last ? rval : nullptr, last ? rfound : nullptr,
                                             rprev ? rprev + off : nullptr, rprevf ? rprevf + off : nullptr));
            off += n;
        } while (off < P.rp);
        // a round with nothing for this owner launches nothing, and the previous round's reads
        // would wait for a later launch while its answers go back in this call's stage B: now
        if (P.rp == 0 && P.rk == 0) RCHK(nrg_join(c));
    }
    return NRG_OK;
}

// Stage B of round e: its reads and previous values are queued (launched with the next round's
// replay, or by the flush's join).
static int pt_stage_b(nrg_group* g, uint64_t e) {
    const Rccl* R = g->R;
    const int G = g->nranks, nl = (int)g->m.size();
    const int sl = (int)(e % PT_DEPTH), par = (int)(e & 1);
    if (g->pt_drop[sl]) return NRG_OK;  // dropped in stage A (its error was returned there)
    const uint64_t CW = 2 * (uint64_t)G + XW_N;
    const uint64_t* H = g->m[0].h_cnt[sl];
    auto word = [&](int s, uint64_t k) { return H[(size_t)s * CW + 2 * G + k]; };
    ncclResult_t res = ncclSuccess;
    if (G > 1) {  // answers back to the ranks that asked, into their owner regions
        if (R->group_start() != ncclSuccess) return NRG_E_COMM;
        for (int i = 0; i < nl && res == ncclSuccess; i++) {
            Member& m = g->m[i];
            const PtPlan& P = m.plan[sl];
            const bool mine = m.pr[sl].resp && m.pr[sl].some;
            const uint64_t cp = m.cap_p[sl], ck = m.cap_k[sl];
            const DBuf* rv = m.rv[par];
            hipStream_t s = m.ctx->stream;
            for (int o = 0; o < G && res == ncclSuccess; o++) {
                if (o == m.rank) continue;
                const bool theirs = word(o, XW_PREV) != 0;
                if (P.gfrom[o]) {
                    res = R->send(at(rv[PR_RVAL].p, P.gfrom_off[o] * 8), P.gfrom[o], ncclUint64, o, m.comm, s);
                    if (res == ncclSuccess)
                        res = R->send(at(rv[PR_RFOUND].p, P.gfrom_off[o]), P.gfrom[o], ncclUint8, o, m.comm, s);
                }
                if (res == ncclSuccess && P.gto[o]) {
                    res = R->recv(at(m.pt[PB_AVAL].p, o * ck * 8), P.gto[o], ncclUint64, o, m.comm, s);
                    if (res == ncclSuccess) res = R->recv(at(m.pt[PB_AFOUND].p, o * ck), P.gto[o], ncclUint8, o, m.comm, s);
                }
                if (res == ncclSuccess && theirs && P.pfrom[o]) {
                    res = R->send(at(rv[PR_RPREV].p, P.pfrom_off[o] * 8), P.pfrom[o], ncclUint64, o, m.comm, s);
                    if (res == ncclSuccess)
                        res = R->send(at(rv[PR_RPREVF].p, P.pfrom_off[o]), P.pfrom[o], ncclUint8, o, m.comm, s);
                }
                if (res == ncclSuccess && mine && P.pto[o]) {
                    res = R->recv(at(m.pt[PB_APREV].p, o * cp * 8), P.pto[o], ncclUint64, o, m.comm, s);
                    if (res == ncclSuccess) res = R->recv(at(m.pt[PB_APREVF].p, o * cp), P.pto[o], ncclUint8, o, m.comm, s);
                }
            }
        }
        RCHK(group_end(g, "partitioned answers back"));
        if (res != ncclSuccess) return group_fail(g, NRG_E_COMM, "partitioned answers back refused");
    }
    // back into the caller's order (one launch for the Gets' answers and the previous values)
    for (int i = 0; i < nl; i++) {
        Member& m = g->m[i];
        const PtPlan& P = m.plan[sl];
        const nrg_round& x = m.pr[sl];
        nrg_ctx* c = m.ctx;
        const int r = m.rank;
        if (pt_ident(g, m)) continue;  // the replay answered into the caller's buffers
        RCHK(nrg::ctx_use_device(c));
        const bool mine = x.resp && x.some;
        const uint64_t cp = m.cap_p[sl], ck = m.cap_k[sl];
        const DBuf* rv = m.rv[par];
        void *aval = m.pt[PB_AVAL].p, *afound = m.pt[PB_AFOUND].p, *aprev = m.pt[PB_APREV].p, *aprevf = m.pt[PB_APREVF].p;
        if (G == 1) {
            aval = rv[PR_RVAL].p, afound = rv[PR_RFOUND].p, aprev = rv[PR_RPREV].p, aprevf = rv[PR_RPREVF].p;
        } else {
            hipStream_t s = c->stream;
            if (P.gto[r]) {
                GCHK(hipMemcpyAsync(at(aval, r * ck * 8), at(rv[PR_RVAL].p, P.gfrom_off[r] * 8), P.gto[r] * 8,
                                    hipMemcpyDeviceToDevice, s));
                GCHK(hipMemcpyAsync(at(afound, r * ck), at(rv[PR_RFOUND].p, P.gfrom_off[r]), P.gto[r],
                                    hipMemcpyDeviceToDevice, s));
            }
            if (mine && P.pto[r]) {
                GCHK(hipMemcpyAsync(at(aprev, r * cp * 8), at(rv[PR_RPREV].p, P.pfrom_off[r] * 8), P.pto[r] * 8,
                                    hipMemcpyDeviceToDevice, s));
                GCHK(hipMemcpyAsync(at(aprevf, r * cp), at(rv[PR_RPREVF].p, P.pfrom_off[r]), P.pto[r],
                                    hipMemcpyDeviceToDevice, s));
            }
        }
        hipStream_t rs = c->stream;
        if (G == 1 && (c->exp & 0x8000)) {  // NRG_KNOB_EXP bit 15
            // (A/B) beside the next replay, on the side stream, after everything queued on the
            // replica's stream so far: the launch that answered this round's reads (the replay of
            // the round after, or a join) is the last of it
            rs = m.pstream;
            GCHK(hipEventRecord(m.rd_ev, c->stream));
            GCHK(hipStreamWaitEvent(rs, m.rd_ev, 0));
        }
        const hipError_t he = nrg::pt_route2(
            rs, (const uint64_t*)aval, (const uint8_t*)afound, (const uint32_t*)m.pp[sl][PP_GPOS].p, x.n_gets,
            x.get_vals, x.get_found, (const uint64_t*)aprev, (const uint8_t*)aprevf,
            (const uint32_t*)m.pp[sl][PP_PPOS].p, mine ? x.n : 0, mine ? (uint64_t*)x.resp : nullptr, mine ? x.some : nullptr);
        if (he != hipSuccess) return hip_rc(he);
    }
    g->round++;
    return NRG_OK;
}

// every posted round through stage B (its result: the first error)
static int pt_flush(nrg_group* g) {
    int rc = NRG_OK;
    while (g->pt_a < g->pt_posted) {
        const int r = pt_stage_a(g, g->pt_a++);
        if (g->broken) return g->broken;
        if (r && rc == NRG_OK) rc = r;
    }
    if (g->pt_b < g->pt_a) {
        for (Member& m : g->m) {  // the last round's deferred reads
            RCHK(nrg::ctx_use_device(m.ctx));
            RCHK(nrg_join(m.ctx));
        }
    }
    while (g->pt_b < g->pt_a) {
        const int r = pt_stage_b(g, g->pt_b++);
        if (g->broken) return g->broken;
        if (r && rc == NRG_OK) rc = r;
    }
    if (g->nranks == 1)  // a one-rank group's route-backs ran on its side stream: ordered again
        for (Member& m : g->m) {
            RCHK(nrg::ctx_use_device(m.ctx));
            RCHK(order(m, m.pstream, m.ctx->stream));
        }
    return rc;
}

static int pt_check(nrg_group* g) {
    if (!g) return NRG_E_INVAL;
    if (g->broken) return g->broken;
    const Rccl* R = g->R;
    if (!R || !R->send || !R->recv) return NRG_E_COMM;
    if (g->nranks > NRG_MAX_PARTS) return NRG_E_INVAL;
    return NRG_OK;
}

int nrg_group_partitioned_round_async(nrg_group* g, const nrg_round* rounds) {
    int r = pt_check(g);
    if (r) return r;
    if (!rounds) return NRG_E_INVAL;
    if ((r = pt_post(g, rounds, g->pt_posted))) return r;
    g->pt_posted++;
    int rc = NRG_OK;
    if (g->pt_posted - g->pt_a >= 2) {  // the previous round: its counts have landed by now
        rc = pt_stage_a(g, g->pt_a++);
        if (g->broken) return g->broken;
    }
    if (g->pt_a - g->pt_b >= 2) {  // the round before: its reads rode in the launch just queued
        if (rc != NRG_OK)  // (that round was dropped, so nothing launched them: now)
            for (Member& m : g->m) {
                RCHK(nrg::ctx_use_device(m.ctx));
                RCHK(nrg_join(m.ctx));
            }
        const int r2 = pt_stage_b(g, g->pt_b++);
        if (g->broken) return g->broken;
        if (r2 && rc == NRG_OK) rc = r2;
    }
    return rc;
}

int nrg_group_partitioned_flush(nrg_group* g) {
    const int r = pt_check(g);
    return r ? r : pt_flush(g);
}

int nrg_group_partitioned_round(nrg_group* g, const nrg_round* rounds) {
    int r = pt_check(g);
    if (r) return r;
    if (!rounds) return NRG_E_INVAL;
    if ((r = pt_flush(g))) return r;
    if ((r = pt_post(g, rounds, g->pt_posted))) return r;
    g->pt_posted++;
    return pt_flush(g);
}

int nrg_group_sync(nrg_group* g) {
    if (!g) return NRG_E_INVAL;
    if (g->broken) return g->broken;
    int rc = g->pt_b < g->pt_posted ? pt_flush(g) : NRG_OK;  // posted partitioned rounds complete first
    if (g->broken) return g->broken;
    for (Member& m : g->m) {
        int r = nrg::ctx_use_device(m.ctx);
        if (r) return r;
        RCHK(wait_stream(g, m.cstream, "group sync (collectives)"));
        RCHK(wait_stream(g, m.pstream, "group sync (partitions)"));
        RCHK(wait_stream(g, m.ctx->stream, "group sync (replay)"));
        // disagreeing round headers (ERR_GROUP, latched by grp_check_kernel) end the group: the
        // ranks have replayed different logs, so every later call reports it too
        uint32_t err = 0;
        GCHK(hipMemcpyAsync(&err, &m.ctx->d_ctl->err, sizeof err, hipMemcpyDeviceToHost, m.ctx->stream));
        GCHK(hipStreamSynchronize(m.ctx->stream));  // drained above: returns at once
        r = nrg_sync(m.ctx);
        if (err & nrg::ERR_GROUP)
            r = group_fail(g, NRG_E_INVAL, "ranks disagreed on a round's segment lengths: replicas diverged");
        if (r && rc == NRG_OK) rc = r;
    }
    return rc;
}

int nrg_group_set_timeout(nrg_group* g, uint32_t ms) {
    if (!g || ms == 0) return NRG_E_INVAL;
    g->timeout_ms = ms;
    return NRG_OK;
}

const char* nrg_group_last_error(const nrg_group* g) { return g ? g->diag : ""; }

}  // extern "C"
