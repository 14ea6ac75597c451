// loopback.cpp — test-only collectives for replica groups whose members all live in this
// process (include/nrgpu_testing.h, nrg_test_loopback_collectives). They replace RCCL's table
// (collectives.hpp) so that a G-member group -- several replicas on the box's one GPU -- runs
// group.cpp's multi-rank code: segment strides and short-segment padding, rank-order origins,
// the rotating gathered buffers, the partitioned send/recv plan and its answers back.
//
// Semantics follow RCCL's for what group.cpp uses. Ops posted between ncclGroupStart and
// ncclGroupEnd are matched at ncclGroupEnd (the k-th all-gather of every rank together; the
// k-th send from a to b with the k-th receive of b from a) and become device copies:
//   every participating stream waits until every other one has reached the collective (the
//   inputs are ready), the copies run on the receiving rank's stream, then every participating
//   stream waits until all copies are done (a sender may reuse its buffer afterwards).
// Nothing here blocks the host. A group posted by one thread must carry every rank's part (one
// process drives all members), which is how nrg_group_open uses it; nrg_group_join supports
// groups of one rank only.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <utility>
#include <vector>

#include "collectives.hpp"

namespace {

struct World;

struct Comm {
    World* w = nullptr;
    int rank = 0;
    int dev = 0;
};

struct World {
    int n = 0;
    int alive = 0;
    std::map<int, std::vector<hipEvent_t>> ev;  // per device: event pool (re-recorded each group)
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
};

std::mutex g_mu;  // world lifetime (destroy may run on any thread)
thread_local int t_depth = 0;
thread_local std::vector<Op> t_pending;
std::atomic<uint64_t> g_ids{1};

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

#define LB_CHK(x)                                            \
    do {                                                     \
        hipError_t _e = (x);                                 \
        if (_e != hipSuccess) return hip_nccl(_e);           \
    } while (0)

// the k-th event of device `dev`'s pool
hipError_t pool_event(World* w, int dev, size_t k, hipEvent_t* out) {
    std::vector<hipEvent_t>& v = w->ev[dev];
    while (v.size() <= k) {
        hipEvent_t e;
        hipError_t r = hipSetDevice(dev);
        if (r == hipSuccess) r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (r != hipSuccess) return r;
        v.push_back(e);
    }
    *out = v[k];
    return hipSuccess;
}

// a stream taking part in the group, with the device it belongs to
struct Part {
    hipStream_t st;
    int dev;
};

// every stream in `parts` waits for every other one's work so far; events from slot base..
hipError_t barrier(World* w, const std::vector<Part>& parts, size_t base) {
    std::vector<hipEvent_t> evs(parts.size());
    for (size_t i = 0; i < parts.size(); i++) {
        hipError_t e = pool_event(w, parts[i].dev, base + i, &evs[i]);
        if (e == hipSuccess) e = hipSetDevice(parts[i].dev);
        if (e == hipSuccess) e = hipEventRecord(evs[i], parts[i].st);
        if (e != hipSuccess) return e;
    }
    for (size_t i = 0; i < parts.size(); i++) {
        hipError_t e = hipSetDevice(parts[i].dev);
        if (e != hipSuccess) return e;
        for (size_t j = 0; j < parts.size(); j++)
            if (j != i && (e = hipStreamWaitEvent(parts[i].st, evs[j], 0)) != hipSuccess) return e;
    }
    return hipSuccess;
}

ncclResult_t execute(std::vector<Op>& ops) {
    if (ops.empty()) return ncclSuccess;
    World* w = ops[0].c->w;
    for (const Op& o : ops)
        if (o.c->w != w) return ncclInvalidUsage;  // one group, one communicator set
    const int n = w->n;
    // all-gathers: the k-th of every rank together, equal sizes, every rank present
    std::vector<std::vector<const Op*>> ag(n);
    // send/recv: FIFO per (src, dst)
    std::map<std::pair<int, int>, std::vector<const Op*>> snd, rcv;
    std::vector<Part> parts;
    auto add_part = [&](const Op& o) {
        for (const Part& p : parts)
            if (p.st == o.st && p.dev == o.c->dev) return;
        parts.push_back(Part{o.st, o.c->dev});
    };
    for (const Op& o : ops) {
        if (o.peer < 0 || o.peer >= n) return ncclInvalidArgument;
        add_part(o);
        if (o.kind == AG) ag[o.c->rank].push_back(&o);
        else if (o.kind == SEND) snd[{o.c->rank, o.peer}].push_back(&o);
        else rcv[{o.peer, o.c->rank}].push_back(&o);
    }
    const size_t nag = ag[0].size();
    for (int r = 0; r < n; r++)
        if (ag[r].size() != nag) return ncclInvalidUsage;  // a rank missing from an all-gather
    for (size_t k = 0; k < nag; k++)
        for (int r = 0; r < n; r++)
            if (ag[r][k]->bytes != ag[0][k]->bytes) return ncclInvalidArgument;
    if (snd.size() != rcv.size()) return ncclInvalidUsage;
    for (const auto& kv : snd) {
        auto it = rcv.find(kv.first);
        if (it == rcv.end() || it->second.size() != kv.second.size()) return ncclInvalidUsage;
        for (size_t k = 0; k < kv.second.size(); k++)
            if (kv.second[k]->bytes != it->second[k]->bytes) return ncclInvalidArgument;
    }
    int cur = 0;
    LB_CHK(hipGetDevice(&cur));
    // inputs ready everywhere
    LB_CHK(barrier(w, parts, 0));
    for (size_t k = 0; k < nag; k++)
        for (int r = 0; r < n; r++) {
            const Op& dst = *ag[r][k];
            LB_CHK(hipSetDevice(dst.c->dev));
            for (int s = 0; s < n; s++)
                if (dst.bytes)
                    LB_CHK(hipMemcpyAsync((char*)dst.rbuf + (size_t)s * dst.bytes, ag[s][k]->sbuf, dst.bytes,
                                          hipMemcpyDeviceToDevice, dst.st));
        }
    for (const auto& kv : snd) {
        const std::vector<const Op*>& rv = rcv[kv.first];
        for (size_t k = 0; k < kv.second.size(); k++) {
            const Op& r = *rv[k];
            LB_CHK(hipSetDevice(r.c->dev));
            if (r.bytes) LB_CHK(hipMemcpyAsync(r.rbuf, kv.second[k]->sbuf, r.bytes, hipMemcpyDeviceToDevice, r.st));
        }
    }
    // copies done everywhere before any rank goes on (senders may overwrite their buffers)
    LB_CHK(barrier(w, parts, parts.size()));
    LB_CHK(hipSetDevice(cur));
    return ncclSuccess;
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
    if (w) w->n = w->alive = n;
    return w;
}

ncclResult_t lb_init_rank(ncclComm_t* comm, int nranks, ncclUniqueId, int rank) {
    if (!comm || nranks != 1 || rank != 0) return ncclInvalidUsage;  // one process drives every member
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return ncclUnhandledCudaError;
    World* w = new_world(1);
    Comm* c = new (std::nothrow) Comm();
    if (!w || !c) {
        delete w;
        delete c;
        return ncclSystemError;
    }
    c->w = w;
    c->dev = dev;
    *comm = reinterpret_cast<ncclComm_t>(c);
    return ncclSuccess;
}

ncclResult_t lb_init_all(ncclComm_t* comms, int n, const int* devs) {
    if (!comms || n < 1) return ncclInvalidArgument;
    World* w = new_world(n);
    if (!w) return ncclSystemError;
    for (int i = 0; i < n; i++) {
        Comm* c = new (std::nothrow) Comm();
        if (!c) return ncclSystemError;
        c->w = w;
        c->rank = i;
        c->dev = devs ? devs[i] : i;
        comms[i] = reinterpret_cast<ncclComm_t>(c);
    }
    return ncclSuccess;
}

ncclResult_t lb_destroy(ncclComm_t comm) {
    Comm* c = reinterpret_cast<Comm*>(comm);
    if (!c) return ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(g_mu);
    World* w = c->w;
    delete c;
    if (w && --w->alive == 0) {
        for (auto& kv : w->ev)
            for (hipEvent_t e : kv.second) (void)hipEventDestroy(e);
        delete w;
    }
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

const nrg::Collectives g_loopback = [] {
    nrg::Collectives t;
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
