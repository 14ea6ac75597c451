// loopback.cpp — test-only collectives for replica groups whose members all live in this
// process (include/nrgpu_testing.h, nrg_test_loopback_collectives). They replace RCCL's table
// (collectives.hpp) so that group.cpp's multi-rank code runs on the box's one GPU: segment
// strides and short-segment padding, the length exchange, rank-order origins, the rotating
// gathered buffers, the partitioned send/recv plan and its answers back.
//
// Two ways to form a world, as with RCCL:
//   ncclCommInitAll   one thread drives every rank (nrg_group_open);
//   ncclCommInitRank  one thread per rank, each joining the same unique id (nrg_group_join), as
//                     one process per GPU would. Init blocks until all ranks have joined.
//
// Semantics follow RCCL's for what group.cpp uses. The ops a thread posts between
// ncclGroupStart and ncclGroupEnd are handed to the world at ncclGroupEnd, which then blocks
// until each of them is matched: the k-th all-gather of a rank with the k-th all-gather of
// every other rank, the k-th send from a to b with the k-th receive of b from a. Whichever
// thread completes a match turns it into device copies:
//   each op records a `ready` event on its stream when it is posted (its input is ready);
//   the copies run on the receiving rank's stream after the senders' ready events, and record
//   a `done` event there; every sending stream then waits for the done events (a sender may
//   reuse its buffer afterwards, as after an RCCL op completes).
// A rank's thread is blocked while other threads enqueue onto its streams, so the copies sit
// exactly at its collective's position in stream order. Mismatched all-gather sizes or p2p
// byte counts fail on every participant (ncclInvalidArgument) instead of corrupting memory. A
// single-thread world fails an op that cannot be matched at once (ncclInvalidUsage); a
// threaded world gives up after the group's deadline (nrg_group_set_timeout; LB_TIMEOUT before
// one is set) with ncclSystemError instead of hanging the test.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <set>
#include <utility>
#include <vector>

#include "collectives.hpp"

namespace {

constexpr auto LB_TIMEOUT = std::chrono::seconds(120);

struct World;

struct Comm {
    World* w = nullptr;
    int rank = 0;
    int dev = 0;
};

enum Kind { AG, SEND, RECV };

struct Op {
    Kind kind;
    const void* sbuf;
    void* rbuf;
    size_t bytes;
    Comm* c;
    hipStream_t st;
    int peer;
    hipEvent_t ready = nullptr;
    uint64_t seq = 0;  // all-gathers: the rank's k
    bool matched = false;
    ncclResult_t res = ncclSuccess;
};

struct World {
    int n = 0;
    bool threaded = false;  // ncclCommInitRank world: one thread per rank
    int joined = 0;
    int alive = 0;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint64_t> ag_seq;                        // all-gathers posted per rank
    std::map<uint64_t, std::vector<Op*>> ag;             // k -> the k-th all-gather of each rank
    std::map<std::pair<int, int>, std::deque<Op*>> snd;  // (src, dst) FIFOs
    std::map<std::pair<int, int>, std::deque<Op*>> rcv;
    std::vector<hipEvent_t> spent;  // events whose waits are enqueued (destroyed after a sync)
    std::set<int> devs;
};

std::mutex g_reg_mu;  // worlds being formed by ncclCommInitRank, by unique id
std::map<uint64_t, World*> g_forming;
std::atomic<uint64_t> g_ids{1};

thread_local int t_depth = 0;
thread_local std::vector<Op> t_pending;
// how long this thread's collectives wait for their peers (nrg_group_set_timeout, via the
// table's set_timeout_ms; LB_TIMEOUT until a group sets it)
thread_local std::chrono::milliseconds t_timeout = std::chrono::duration_cast<std::chrono::milliseconds>(LB_TIMEOUT);

size_t dt_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8:
        case ncclUint8:
        case ncclFloat8e4m3:
        case ncclFloat8e5m2: return 1;
        case ncclFloat16:
        case ncclBfloat16: return 2;
        case ncclInt32:
        case ncclUint32:
        case ncclFloat32: return 4;
        case ncclInt64:
        case ncclUint64:
        case ncclFloat64: return 8;
        default: return 0;
    }
}

ncclResult_t hip_nccl(hipError_t e) { return e == hipSuccess ? ncclSuccess : ncclUnhandledCudaError; }

hipError_t new_event(World* w, int dev, hipEvent_t* e) {
    hipError_t r = hipSetDevice(dev);
    if (r == hipSuccess) r = hipEventCreateWithFlags(e, hipEventDisableTiming);
    if (r == hipSuccess) w->spent.push_back(*e);
    return r;
}

// Events are destroyed only once nothing can still wait on them: after every device of the
// world has drained (callers hold the world lock, so no rank enqueues meanwhile), and -- unless
// the world is going away -- while no posted op is waiting for its match: an unmatched op's
// `ready` event is in `spent` too, and the thread that completes the match waits on it later.
bool any_pending(const World* w) {
    if (!w->ag.empty()) return true;
    for (const auto* m : {&w->snd, &w->rcv})
        for (const auto& kv : *m)
            if (!kv.second.empty()) return true;
    return false;
}

void reap(World* w, bool force) {
    if (!force && (w->spent.size() < 4096 || any_pending(w))) return;
    for (int d : w->devs)
        if (hipSetDevice(d) == hipSuccess) (void)hipDeviceSynchronize();
    for (hipEvent_t e : w->spent) (void)hipEventDestroy(e);
    w->spent.clear();
}

// the k-th all-gather of every rank: copies into every rank's receive buffer
hipError_t run_ag(World* w, std::vector<Op*>& v) {
    const int n = w->n;
    for (int r = 1; r < n; r++)
        if (v[r]->bytes != v[0]->bytes) {
            for (Op* o : v) o->res = ncclInvalidArgument;
            return hipSuccess;
        }
    const size_t bytes = v[0]->bytes;
    std::vector<hipEvent_t> done(n);
    for (int r = 0; r < n; r++) {
        Op& d = *v[r];
        hipError_t e = new_event(w, d.c->dev, &done[r]);
        if (e != hipSuccess) return e;
        for (int s = 0; s < n; s++)
            if (s != r && (e = hipStreamWaitEvent(d.st, v[s]->ready, 0)) != hipSuccess) return e;
        for (int s = 0; s < n && bytes; s++) {
            char* dst = (char*)d.rbuf + (size_t)s * bytes;
            if (dst == v[s]->sbuf) continue;  // in place
            if ((e = hipMemcpyAsync(dst, v[s]->sbuf, bytes, hipMemcpyDeviceToDevice, d.st)) != hipSuccess) return e;
        }
        if ((e = hipEventRecord(done[r], d.st)) != hipSuccess) return e;
    }
    for (int s = 0; s < n; s++) {
        hipError_t e = hipSetDevice(v[s]->c->dev);
        if (e != hipSuccess) return e;
        for (int r = 0; r < n; r++)
            if (r != s && (e = hipStreamWaitEvent(v[s]->st, done[r], 0)) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t run_p2p(World* w, Op& s, Op& r) {
    if (s.bytes != r.bytes) {
        s.res = r.res = ncclInvalidArgument;
        return hipSuccess;
    }
    hipEvent_t done;
    hipError_t e = new_event(w, r.c->dev, &done);
    if (e == hipSuccess) e = hipStreamWaitEvent(r.st, s.ready, 0);
    if (e == hipSuccess && r.bytes) e = hipMemcpyAsync(r.rbuf, s.sbuf, r.bytes, hipMemcpyDeviceToDevice, r.st);
    if (e == hipSuccess) e = hipEventRecord(done, r.st);
    if (e == hipSuccess) e = hipSetDevice(s.c->dev);
    if (e == hipSuccess) e = hipStreamWaitEvent(s.st, done, 0);
    return e;
}

// Complete every match the posted ops allow (world lock held).
ncclResult_t match(World* w) {
    for (auto it = w->ag.begin(); it != w->ag.end();) {
        std::vector<Op*>& v = it->second;
        bool full = true;
        for (Op* o : v) full = full && o;
        if (!full) {
            ++it;
            continue;
        }
        hipError_t e = run_ag(w, v);
        for (Op* o : v) {
            if (e != hipSuccess) o->res = hip_nccl(e);
            o->matched = true;
        }
        it = w->ag.erase(it);
    }
    for (auto& kv : w->snd) {
        std::deque<Op*>& s = kv.second;
        std::deque<Op*>& r = w->rcv[kv.first];
        while (!s.empty() && !r.empty()) {
            hipError_t e = run_p2p(w, *s.front(), *r.front());
            for (Op* o : {s.front(), r.front()}) {
                if (e != hipSuccess) o->res = hip_nccl(e);
                o->matched = true;
            }
            s.pop_front();
            r.pop_front();
        }
    }
    return ncclSuccess;
}

// withdraw ops that were never matched (a failed or abandoned group); a rank's withdrawn
// all-gather gives its sequence number back, so the world's later all-gathers still line up
void withdraw(World* w, std::vector<Op>& ops) {
    for (Op& o : ops) {
        if (o.matched) continue;
        if (o.kind == AG) {
            auto it = w->ag.find(o.seq);
            if (it != w->ag.end() && it->second[o.c->rank] == &o) {
                it->second[o.c->rank] = nullptr;
                if (w->ag_seq[o.c->rank] == o.seq + 1) w->ag_seq[o.c->rank]--;
                bool any = false;
                for (Op* p : it->second) any = any || p;
                if (!any) w->ag.erase(it);
            }
            continue;
        }
        for (auto* m : {&w->snd, &w->rcv})
            for (auto& kv : *m)
                for (auto it = kv.second.begin(); it != kv.second.end();)
                    it = *it == &o ? kv.second.erase(it) : it + 1;
    }
}

ncclResult_t execute(std::vector<Op>& ops) {
    if (ops.empty()) return ncclSuccess;  // an empty group posts nothing (as RCCL)
    World* w = ops[0].c->w;
    for (const Op& o : ops)
        if (o.c->w != w) return ncclInvalidUsage;  // one group, one communicator set
    for (const Op& o : ops)
        if ((o.kind != AG && (o.peer < 0 || o.peer >= w->n))) return ncclInvalidArgument;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return ncclUnhandledCudaError;
    std::unique_lock<std::mutex> lk(w->mu);
    reap(w, false);
    ncclResult_t res = ncclSuccess;
    for (Op& o : ops) {  // inputs ready at this point of each stream
        hipError_t e = new_event(w, o.c->dev, &o.ready);
        if (e == hipSuccess) e = hipEventRecord(o.ready, o.st);
        if (e != hipSuccess) {
            res = hip_nccl(e);
            break;
        }
    }
    if (res == ncclSuccess)
        for (Op& o : ops) {
            w->devs.insert(o.c->dev);
            if (o.kind == AG) {
                const int r = o.c->rank;
                o.seq = w->ag_seq[r]++;
                std::vector<Op*>& v = w->ag[o.seq];
                if (v.empty()) v.assign(w->n, nullptr);
                v[r] = &o;
            } else if (o.kind == SEND) {
                w->snd[{o.c->rank, o.peer}].push_back(&o);
            } else {
                w->rcv[{o.peer, o.c->rank}].push_back(&o);
            }
        }
    if (res == ncclSuccess) res = match(w);
    auto all_matched = [&] {
        for (const Op& o : ops)
            if (!o.matched) return false;
        return true;
    };
    if (res == ncclSuccess && !all_matched()) {
        w->cv.notify_all();
        if (!w->threaded) res = ncclInvalidUsage;  // nobody else can post the other half
        else if (!w->cv.wait_for(lk, t_timeout, all_matched)) res = ncclSystemError;
    } else {
        w->cv.notify_all();
    }
    if (res != ncclSuccess) withdraw(w, ops);
    for (const Op& o : ops)
        if (res == ncclSuccess && o.res != ncclSuccess) res = o.res;
    lk.unlock();
    w->cv.notify_all();
    (void)hipSetDevice(cur);
    return res;
}

ncclResult_t post(Op o) {
    if (!o.c || !o.c->w) return ncclInvalidArgument;
    if (t_depth > 0) {
        t_pending.push_back(o);
        return ncclSuccess;
    }
    std::vector<Op> one{o};  // outside a group: a group of this op alone
    return execute(one);
}

ncclResult_t lb_get_unique_id(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id, 0, sizeof(*id));
    std::memcpy(id->internal, "NRGLOOPB", 8);
    const uint64_t k = g_ids.fetch_add(1);
    std::memcpy(id->internal + 8, &k, sizeof(k));
    return ncclSuccess;
}

World* new_world(int n) {
    World* w = new (std::nothrow) World();
    if (w) {
        w->n = w->alive = n;
        w->ag_seq.assign(n, 0);
    }
    return w;
}

// One thread per rank: the threads that pass the same id form one world. Blocks until all
// nranks have joined (ncclCommInitRank does the same).
ncclResult_t lb_init_rank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    if (std::memcmp(id.internal, "NRGLOOPB", 8) != 0) return ncclInvalidUsage;  // not a loopback id
    uint64_t key;
    std::memcpy(&key, id.internal + 8, sizeof(key));
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return ncclUnhandledCudaError;
    Comm* c = new (std::nothrow) Comm();
    if (!c) return ncclSystemError;
    c->rank = rank;
    c->dev = dev;
    World* w = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_forming.find(key);
        if (it == g_forming.end()) {
            w = new_world(nranks);
            if (!w) {
                delete c;
                return ncclSystemError;
            }
            w->threaded = true;
            w->alive = 0;
            g_forming[key] = w;
        } else {
            w = it->second;
            if (w->n != nranks) {
                delete c;
                return ncclInvalidArgument;
            }
        }
        w->alive++;
    }
    c->w = w;
    std::unique_lock<std::mutex> lk(w->mu);
    w->devs.insert(dev);
    if (++w->joined == w->n) {
        std::lock_guard<std::mutex> rl(g_reg_mu);
        g_forming.erase(key);
        w->cv.notify_all();
    } else if (!w->cv.wait_for(lk, t_timeout, [&] { return w->joined == w->n; })) {
        // A rank never joined: leave the world as if this rank had never come, so a retry with
        // the same id starts from correct counts; the last joiner to give up frees it.
        lk.unlock();
        std::lock_guard<std::mutex> rl(g_reg_mu);
        bool last = false;
        {
            // the world's lock is released before the world may be freed below
            std::lock_guard<std::mutex> wl(w->mu);
            if (w->joined == w->n) {  // the last rank arrived just now: keep this rank in the world
                *comm = reinterpret_cast<ncclComm_t>(c);
                return ncclSuccess;
            }
            w->joined--;
            last = --w->alive == 0;
        }
        delete c;
        if (last) {
            auto it = g_forming.find(key);
            if (it != g_forming.end() && it->second == w) g_forming.erase(it);
            delete w;  // nobody else holds it: it was still forming, with no joiner left
        }
        return ncclSystemError;
    }
    *comm = reinterpret_cast<ncclComm_t>(c);
    return ncclSuccess;
}

ncclResult_t lb_init_all(ncclComm_t* comms, int n, const int* devs) {
    if (!comms || n < 1) return ncclInvalidArgument;
    World* w = new_world(n);
    if (!w) return ncclSystemError;
    w->joined = n;
    for (int i = 0; i < n; i++) {
        Comm* c = new (std::nothrow) Comm();
        if (!c) return ncclSystemError;
        c->w = w;
        c->rank = i;
        c->dev = devs ? devs[i] : i;
        w->devs.insert(c->dev);
        comms[i] = reinterpret_cast<ncclComm_t>(c);
    }
    return ncclSuccess;
}

ncclResult_t lb_destroy(ncclComm_t comm) {
    Comm* c = reinterpret_cast<Comm*>(comm);
    if (!c) return ncclInvalidArgument;
    World* w = c->w;
    delete c;
    bool last = false;
    {
        std::lock_guard<std::mutex> lk(w->mu);
        last = --w->alive == 0;
        if (last) reap(w, true);
    }
    if (last) delete w;
    return ncclSuccess;
}

ncclResult_t lb_all_gather(const void* sbuf, void* rbuf, size_t count, ncclDataType_t dt, ncclComm_t comm,
                           hipStream_t st) {
    const size_t eb = dt_bytes(dt);
    Comm* c = reinterpret_cast<Comm*>(comm);
    if (!eb || !c || (count && (!sbuf || !rbuf))) return ncclInvalidArgument;
    return post(Op{AG, sbuf, rbuf, count * eb, c, st, 0});
}

ncclResult_t lb_send(const void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t st) {
    const size_t eb = dt_bytes(dt);
    Comm* c = reinterpret_cast<Comm*>(comm);
    if (!eb || !c || (count && !buf)) return ncclInvalidArgument;
    return post(Op{SEND, buf, nullptr, count * eb, c, st, peer});
}

ncclResult_t lb_recv(void* buf, size_t count, ncclDataType_t dt, int peer, ncclComm_t comm, hipStream_t st) {
    const size_t eb = dt_bytes(dt);
    Comm* c = reinterpret_cast<Comm*>(comm);
    if (!eb || !c || (count && !buf)) return ncclInvalidArgument;
    return post(Op{RECV, nullptr, buf, count * eb, c, st, peer});
}

ncclResult_t lb_group_start() {
    t_depth++;
    return ncclSuccess;
}

ncclResult_t lb_group_end() {
    if (t_depth <= 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(t_pending);
    return execute(ops);
}

void lb_set_timeout_ms(uint32_t ms) { t_timeout = std::chrono::milliseconds(ms); }

const nrg::Collectives g_loopback = [] {
    nrg::Collectives t;
    t.set_timeout_ms = lb_set_timeout_ms;
    t.get_unique_id = lb_get_unique_id;
    t.init_rank = lb_init_rank;
    t.init_all = lb_init_all;
    t.all_gather = lb_all_gather;
    t.group_start = lb_group_start;
    t.group_end = lb_group_end;
    t.destroy = lb_destroy;
    t.send = lb_send;
    t.recv = lb_recv;
    return t;
}();

}  // namespace

namespace nrg {
const Collectives* loopback_collectives() { return &g_loopback; }
}  // namespace nrg
