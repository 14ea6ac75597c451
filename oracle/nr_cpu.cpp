// nr_cpu.cpp — C++ restatement of the `nr` crate's control plane (Log, Context, RwLock,
// Replica with flat combining) over the oracle's sequential data structures.
//
// TEST INFRASTRUCTURE ONLY: it is (1) the subject of the ported deterministic unit tests of
// nr/src/log.rs:708-1131, nr/src/context.rs:209-399 and nr/src/replica.rs:598-788, and
// (2) bench.py's `cpu_baseline` leg ("C++ restatement of nr", kind "port"), timed on the
// GPU box's host cores with one Replica per NUMA node. The product
// (node-replication_amd/) never links or loads it.
//
// The reference is Rust (#![no_std], nightly) and cannot be compiled here; each piece below
// cites the function it restates.

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "nr_oracle.h"

namespace nrcpu {

// nr/src/log.rs:22,26,36,43 ; nr/src/context.rs:12 ; nr/src/replica.rs:56 ; nr/src/rwlock.rs:19
constexpr size_t DEFAULT_LOG_BYTES = 32 * 1024 * 1024;
constexpr size_t MAX_REPLICAS = 192;
constexpr size_t MAX_PENDING_OPS = 32;
constexpr size_t MAX_THREADS_PER_REPLICA = 256;
constexpr size_t GC_FROM_HEAD = MAX_PENDING_OPS * MAX_THREADS_PER_REPLICA;  // 8192
constexpr size_t MAX_READER_THREADS = 192;

struct alignas(64) Padded {
    std::atomic<size_t> v{0};
};

static inline void spin_pause() { __builtin_ia32_pause(); }

// ---- Log<T> (nr/src/log.rs:88-131) -----------------------------------------------------
template <typename T>
struct alignas(64) Entry {  // nr/src/log.rs:51-65 — one 64-byte line per entry
    T operation{};
    bool has_op = false;
    size_t replica = 0;
    std::atomic<bool> alivef{false};
};

template <typename T>
class Log {
   public:
    // Log::new (nr/src/log.rs:179-242): entries = bytes/64, at least 2*GC_FROM_HEAD,
    // rounded up to a power of two.
    explicit Log(size_t bytes) {
        size_t num = bytes / entry_size();
        if (num < 2 * GC_FROM_HEAD) num = 2 * GC_FROM_HEAD;
        size_t p = 1;
        while (p < num) p <<= 1;
        num = p;
        size_ = num;
        rawb_ = num * entry_size();
        slog_ = static_cast<Entry<T>*>(::operator new[](rawb_, std::align_val_t(64)));
        for (size_t i = 0; i < num; i++) new (&slog_[i]) Entry<T>();
        for (size_t i = 0; i < MAX_REPLICAS; i++) lmasks_[i] = true;
        next_.v = 1;
    }
    ~Log() {
        for (size_t i = 0; i < size_; i++) slog_[i].~Entry<T>();
        ::operator delete[](slog_, std::align_val_t(64));
    }
    static size_t entry_size() { return sizeof(Entry<T>); }

    // Log::register (:272-292): ids start at 1, None once MAX_REPLICAS is reached.
    long reg() {
        for (;;) {
            size_t n = next_.v.load(std::memory_order_relaxed);
            if (n >= MAX_REPLICAS) return -1;
            if (next_.v.compare_exchange_weak(n, n + 1)) return (long)n;
        }
    }

    // Log::append (:343-427)
    template <typename F>
    void append(const T* ops, size_t nops, size_t idx, F&& s) {
        for (;;) {
            size_t tail = tail_.v.load(std::memory_order_relaxed);
            size_t head = head_.v.load(std::memory_order_relaxed);
            if (tail > head + size_ - GC_FROM_HEAD) {  // wait for GC, keep replaying
                exec(idx, s);
                continue;
            }
            bool advance = tail + nops > head + size_ - GC_FROM_HEAD;
            if (!tail_.v.compare_exchange_weak(tail, tail + nops, std::memory_order_acquire))
                continue;
            for (size_t i = 0; i < nops; i++) {
                Entry<T>* e = &slog_[index(tail + i)];
                bool m = lmasks_[idx - 1];
                if (e->alivef.load(std::memory_order_relaxed) == m) m = !m;  // wrapped
                e->operation = ops[i];
                e->has_op = true;
                e->replica = idx;
                e->alivef.store(m, std::memory_order_release);
            }
            if (advance) advance_head(idx, s);
            return;
        }
    }

    // Log::exec (:473-524)
    template <typename F>
    void exec(size_t idx, F&& d) {
        size_t l = ltails_[idx - 1].v.load(std::memory_order_relaxed);
        size_t t = tail_.v.load(std::memory_order_relaxed);
        if (l == t) return;
        size_t h = head_.v.load(std::memory_order_relaxed);
        if (l > t || l < h) {
            exec_panicked_ = true;  // panic!("Local tail not within the shared log!")
            return;
        }
        for (size_t i = l; i < t; i++) {
            Entry<T>* e = &slog_[index(i)];
            while (e->alivef.load(std::memory_order_acquire) != lmasks_[idx - 1]) spin_pause();
            d(e->operation, e->replica);
            if (index(i) == size_ - 1) lmasks_[idx - 1] = !lmasks_[idx - 1];
        }
        size_t c = ctail_.v.load(std::memory_order_relaxed);
        while (c < t && !ctail_.v.compare_exchange_weak(c, t, std::memory_order_relaxed)) {
        }
        ltails_[idx - 1].v.store(t, std::memory_order_relaxed);
    }

    size_t index(size_t logical) const { return logical & (size_ - 1); }

    // Log::advance_head (:536-580)
    template <typename F>
    void advance_head(size_t rid, F&& s) {
        for (;;) {
            size_t r = next_.v.load(std::memory_order_relaxed);
            size_t global_head = head_.v.load(std::memory_order_relaxed);
            size_t f = tail_.v.load(std::memory_order_relaxed);
            size_t min_local_tail = ltails_[0].v.load(std::memory_order_relaxed);
            for (size_t i = 1; i < r; i++) {
                size_t cur = ltails_[i - 1].v.load(std::memory_order_relaxed);
                if (min_local_tail > cur) min_local_tail = cur;
            }
            if (min_local_tail == global_head) {
                if (rid >= 1) exec(rid, s);
                else return;  // test hook: no replica to make progress with
                continue;
            }
            head_.v.store(min_local_tail, std::memory_order_relaxed);
            if (f < min_local_tail + size_ - GC_FROM_HEAD) return;
            exec(rid, s);
        }
    }

    // Log::reset (:593-611)
    void reset() {
        head_.v = 0;
        tail_.v = 0;
        next_.v = 1;
        for (size_t r = 0; r < MAX_REPLICAS; r++) {
            ltails_[r].v = 0;
            lmasks_[r] = true;
        }
        for (size_t i = 0; i < size_; i++) slog_[i].alivef.store(false, std::memory_order_release);
    }

    bool is_replica_synced_for_reads(size_t idx, size_t ctail) const {  // :671-673
        return ltails_[idx - 1].v.load(std::memory_order_relaxed) >= ctail;
    }
    size_t get_ctail() const { return ctail_.v.load(std::memory_order_relaxed); }  // :677-679

    // fields (tests reach in exactly like the reference's in-module tests do)
    size_t size_ = 0, rawb_ = 0;
    Entry<T>* slog_ = nullptr;
    Padded head_, tail_, ctail_, next_;
    Padded ltails_[MAX_REPLICAS];
    bool lmasks_[MAX_REPLICAS];
    bool exec_panicked_ = false;
};

// ---- Context (nr/src/context.rs:32-194) ------------------------------------------------
template <typename T, typename R>
struct alignas(64) Context {
    struct alignas(64) Slot {
        T op{};
        bool has_op = false;
        R resp{};
        bool has_resp = false;
    };
    Slot batch[MAX_PENDING_OPS];
    alignas(64) std::atomic<size_t> tail{0};
    alignas(64) std::atomic<size_t> head{0};
    alignas(64) std::atomic<size_t> comb{0};
    bool panicked = false;

    static size_t index(size_t l) { return l & (MAX_PENDING_OPS - 1); }

    bool enqueue(const T& op) {  // :88-106
        size_t t = tail.load(std::memory_order_relaxed), h = head.load(std::memory_order_acquire);
        if (t - h == MAX_PENDING_OPS) return false;
        batch[index(t)].op = op;
        batch[index(t)].has_op = true;
        tail.store(t + 1, std::memory_order_release);
        return true;
    }
    void enqueue_resps(const R* r, size_t n) {  // :112-131
        size_t h = comb.load(std::memory_order_relaxed);
        if (n == 0) return;
        for (size_t i = 0; i < n; i++) {
            batch[index(h + i)].resp = r[i];
            batch[index(h + i)].has_resp = true;
        }
        comb.store(h + n, std::memory_order_release);
    }
    size_t ops(std::vector<T>& buffer) {  // :136-175
        size_t h = comb.load(std::memory_order_relaxed), t = tail.load(std::memory_order_acquire);
        if (h == t) return 0;
        if (h > t) { panicked = true; return 0; }
        size_t n = 0;
        for (; h != t; h++, n++) buffer.push_back(batch[index(h)].op);
        return n;
    }
    bool res(R* out) {  // :179-194
        size_t s = head.load(std::memory_order_relaxed), f = comb.load(std::memory_order_acquire);
        if (s == f) return false;
        if (s > f) { panicked = true; return false; }
        *out = batch[index(s)].resp;
        head.store(s + 1, std::memory_order_release);
        return true;
    }
};

// ---- RwLock (nr/src/rwlock.rs:47-197) ---------------------------------------------------
class RwLock {
   public:
    void write_lock(size_t n) {  // :103-129
        for (;;) {
            bool f = false;
            if (wlock_.v.load(std::memory_order_relaxed)) { spin_pause(); continue; }
            size_t expect = 0;
            (void)f;
            if (wlock_.v.compare_exchange_weak(expect, 1, std::memory_order_acquire)) break;
        }
        size_t lim = n < MAX_READER_THREADS ? n : MAX_READER_THREADS;
        for (size_t i = 0; i < lim; i++)
            while (rlock_[i].v.load(std::memory_order_acquire) != 0) spin_pause();
    }
    void write_unlock() { wlock_.v.store(0, std::memory_order_release); }
    void read_lock(size_t tid) {  // :148-179
        for (;;) {
            while (wlock_.v.load(std::memory_order_acquire)) spin_pause();
            rlock_[tid].v.fetch_add(1, std::memory_order_acquire);
            if (!wlock_.v.load(std::memory_order_acquire)) return;
            rlock_[tid].v.fetch_sub(1, std::memory_order_release);
        }
    }
    void read_unlock(size_t tid) { rlock_[tid].v.fetch_sub(1, std::memory_order_release); }

   private:
    Padded wlock_;
    Padded rlock_[MAX_READER_THREADS];
};

// ---- Replica<D> (nr/src/replica.rs:72-595) ----------------------------------------------
// D provides: using W, Rd, Resp; Resp dispatch_mut(const W&); Resp dispatch(const Rd&) const
template <typename D>
class Replica {
   public:
    using W = typename D::W;
    using Rd = typename D::Rd;
    using Resp = typename D::Resp;

    Replica(Log<W>* log, D* data) : slog_(log), data_(data) {
        long id = log->reg();
        idx_ = id < 0 ? 0 : (size_t)id;
        contexts_ = new Context<W, Resp>[MAX_THREADS_PER_REPLICA];
        buffer_.reserve(MAX_THREADS_PER_REPLICA * MAX_PENDING_OPS);
        result_.reserve(MAX_THREADS_PER_REPLICA * MAX_PENDING_OPS);
        next_.v = 1;
        combiner_.v = 0;
    }
    ~Replica() { delete[] contexts_; }

    long reg() {  // :279-298
        for (;;) {
            size_t idx = next_.v.load();
            if (idx > MAX_THREADS_PER_REPLICA) return -1;
            if (next_.v.compare_exchange_weak(idx, idx + 1)) return (long)idx;
        }
    }

    Resp execute_mut(const W& op, size_t tid) {  // :345-356
        while (!contexts_[tid - 1].enqueue(op)) {
        }
        try_combine(tid);
        return get_response(tid);
    }

    Resp execute(const Rd& op, size_t tid) { return read_only(op, tid); }  // :404-410

    void sync(size_t tid) {  // :473-479
        size_t ctail = slog_->get_ctail();
        while (!slog_->is_replica_synced_for_reads(idx_, ctail)) {
            try_combine(tid);
            spin_pause();
        }
    }

    template <typename F>
    void verify(F&& v) {  // :443-467
        size_t expect = 0;
        while (!combiner_.v.compare_exchange_weak(expect, MAX_THREADS_PER_REPLICA + 2,
                                                  std::memory_order_acquire)) {
            expect = 0;
            spin_pause();
        }
        lock_.write_lock(next_.v.load(std::memory_order_relaxed));
        auto f = [&](const W& o, size_t) { data_->dispatch_mut(o); };
        slog_->exec(idx_, f);
        v(*data_);
        lock_.write_unlock();
        combiner_.v.store(0, std::memory_order_release);
    }

    bool make_pending(const W& op, size_t tid) { return contexts_[tid - 1].enqueue(op); }

    void try_combine(size_t tid) {  // :508-540
        for (int i = 0; i < 4; i++)
            if (combiner_.v.load(std::memory_order_relaxed) != 0) return;
        size_t expect = 0;
        if (!combiner_.v.compare_exchange_weak(expect, tid, std::memory_order_acquire)) return;
        combine();
        combiner_.v.store(0, std::memory_order_release);
    }

    Resp get_response(size_t tid) {  // :414-433
        size_t iter = 0;
        const size_t interval = 1ull << 29;
        Resp r{};
        for (;;) {
            if (contexts_[tid - 1].res(&r)) return r;
            if (++iter == interval) {
                try_combine(tid);
                iter = 0;
            }
        }
    }

    void combine() {  // :544-595
        buffer_.clear();
        result_.clear();
        size_t next = next_.v.load(std::memory_order_relaxed);
        for (size_t i = 1; i < next; i++) inflight_[i - 1] = contexts_[i - 1].ops(buffer_);
        {
            auto f = [&](const W& o, size_t i) {
                lock_.write_lock(next);
                Resp r = data_->dispatch_mut(o);
                lock_.write_unlock();
                if (i == idx_) result_.push_back(r);
            };
            slog_->append(buffer_.data(), buffer_.size(), idx_, f);
        }
        {
            lock_.write_lock(next);
            auto f = [&](const W& o, size_t i) {
                Resp r = data_->dispatch_mut(o);
                if (i == idx_) result_.push_back(r);
            };
            slog_->exec(idx_, f);
            lock_.write_unlock();
        }
        size_t s = 0;
        for (size_t i = 1; i < next; i++) {
            if (inflight_[i - 1] == 0) continue;
            contexts_[i - 1].enqueue_resps(result_.data() + s, inflight_[i - 1]);
            s += inflight_[i - 1];
            inflight_[i - 1] = 0;
        }
    }

    Resp read_only(const Rd& op, size_t tid) {  // :483-497
        size_t ctail = slog_->get_ctail();
        while (!slog_->is_replica_synced_for_reads(idx_, ctail)) {
            try_combine(tid);
            spin_pause();
        }
        size_t rt = (tid - 1) % MAX_READER_THREADS;  // the reference indexes rlock[tid-1]
        lock_.read_lock(rt);
        Resp r = data_->dispatch(op);
        lock_.read_unlock(rt);
        return r;
    }

    size_t idx_ = 0;
    Padded combiner_, next_;
    Context<W, Resp>* contexts_ = nullptr;
    std::vector<W> buffer_;
    size_t inflight_[MAX_THREADS_PER_REPLICA] = {};
    std::vector<Resp> result_;
    Log<W>* slog_;
    RwLock lock_;
    D* data_;
};

// ---- Data structures plugged into Replica -------------------------------------------------
struct HmOp {  // benches/hashmap.rs:52-63 (Put) / Get
    uint64_t key, val;
};
struct HmResp {
    uint64_t val;
    uint8_t some;
};
struct HashMapD {  // NrHashMap over the oracle map (benches/hashmap.rs:77-122)
    using W = HmOp;
    using Rd = uint64_t;
    using Resp = HmResp;
    orc_hm* m;
    HmResp dispatch_mut(const HmOp& o) {
        uint64_t pv = 0;
        int f = orc_hm_insert(m, o.key, o.val, &pv);
        return HmResp{f ? pv : 0, (uint8_t)f};
    }
    HmResp dispatch(const uint64_t& k) const {
        uint64_t v = 0;
        int f = orc_hm_get(m, k, &v);
        return HmResp{f ? v : 0, (uint8_t)f};
    }
};

// The `Data{junk}` fake of nr/src/replica.rs:605-624: dispatch_mut => junk += 1, Ok(107);
// dispatch => Ok(junk).
struct JunkD {
    using W = uint64_t;
    using Rd = uint64_t;
    using Resp = uint64_t;
    uint64_t junk = 0;
    uint64_t dispatch_mut(const uint64_t&) {
        junk += 1;
        return 107;
    }
    uint64_t dispatch(const uint64_t&) const { return junk; }
};


// Stack (benches/stack.rs:36-84): a Vec<u32>, Push -> None, Pop -> Vec::pop. Stack::default
// holds 0..50000 (:50-63). Op encoding: bit 32 = Push, low 32 bits = the value.
struct StackD {
    using W = uint64_t;
    using Rd = uint64_t;  // OpRd is empty in the reference (:29-30); never dispatched
    using Resp = uint64_t;  // Option<u32>: bit 32 = Some
    std::vector<uint32_t> storage;
    uint64_t dispatch_mut(const uint64_t& op) {
        if ((op >> 32) & 1) {
            storage.push_back((uint32_t)op);
            return 0;
        }
        if (storage.empty()) return 0;
        uint32_t v = storage.back();
        storage.pop_back();
        return (1ull << 32) | v;
    }
    uint64_t dispatch(const uint64_t&) const { return 0; }
};

// AbstractDataStructure (benches/synthetic.rs:60-195) with the bench's default
// new(200_000, 20, 5, 2, 1) (:75-79) and its CachePadded<usize> words (:72). Wrapping usize
// arithmetic as a release build; the hot loop is empty when rnd2 + hot_writes wraps.
struct SyOp {
    uint64_t tid, r1, r2, kind;  // kind 1 = ReadWrite, 0 = WriteOnly
};
struct SynthD {
    using W = SyOp;
    using Rd = SyOp;
    using Resp = uint64_t;
    struct alignas(128) Word {
        uint64_t v;
    };
    uint64_t n = 200000, cold_reads = 20, cold_writes = 5, hot_reads = 2, hot_writes = 1;
    std::vector<Word> storage;
    void init() {
        storage.resize(n);
        for (uint64_t i = 0; i < n; i++) storage[i].v = i;  // :97-100
    }
    uint64_t hot_count(uint64_t b) const { return b + hot_writes < b ? 0 : hot_writes; }
    uint64_t dispatch_mut(const SyOp& o) {
        uint64_t hc = hot_count(o.r2), begin = o.r1 * o.tid, sum = 0;
        if (o.kind) {  // read_write (:154-174)
            for (uint64_t j = 0; j < hc; j++) storage[(o.r2 + j) % hot_reads].v += 1;
            for (uint64_t k = 0; k < cold_writes; k++) {
                uint64_t idx = begin % (n - hot_reads) + hot_reads;
                begin += o.r2;
                sum += storage[idx].v;
                storage[idx].v += 1;
            }
            return sum;
        }
        for (uint64_t j = 0; j < hc; j++) storage[(o.r2 + j) % hot_reads].v = o.tid;  // write (:134-152)
        for (uint64_t k = 0; k < cold_writes; k++) {
            uint64_t idx = begin % (n - hot_reads) + hot_reads;
            begin += o.r2;
            storage[idx].v = o.tid;
        }
        return 0;
    }
    uint64_t dispatch(const SyOp& o) const {  // read (:112-132)
        uint64_t hc = hot_count(o.r2), begin = o.r1 * o.tid, sum = 0;
        for (uint64_t j = 0; j < hc; j++) sum += storage[(o.r2 + j) % hot_reads].v;
        for (uint64_t k = 0; k < cold_reads; k++) {
            sum += storage[begin % (n - hot_reads) + hot_reads].v;
            begin += o.r2;
        }
        return sum;
    }
};

// The scale-out harness (benches/mkbench.rs:611-831) over any D: one Replica per CPU group,
// each replica's D built by a thread pinned to its first core (node-local memory, :611-629),
// pinned worker threads that each walk their own shuffled copy of the op stream (:705-706),
// 128 ops per clock check (:737-773), and a final sync so finished replicas keep combining
// for the others' GC (:799-821). init(D&) builds a replica's data; run(rep, tok, i, cpu)
// issues op i of the shared stream and returns 1 for a write.
static inline void pin_to(int cpu) {
    if (cpu < 0) return;
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

template <typename D, typename Init, typename Run, typename Fini>
static void scale_out(uint32_t nreplicas, const int* cpus, const uint32_t* cpu_replica, uint32_t nthreads,
                      double duration_s, uint64_t nop, uint64_t seed, uint64_t log_bytes, Init&& init,
                      Run&& run, Fini&& fini, double* seconds, uint64_t* ops, uint64_t* writes) {
    Log<typename D::W> log(log_bytes ? log_bytes : DEFAULT_LOG_BYTES);
    std::vector<D> ds(nreplicas);
    std::vector<std::unique_ptr<Replica<D>>> reps;
    for (uint32_t r = 0; r < nreplicas; r++) {
        int cpu = -1;
        for (uint32_t t = 0; t < nthreads; t++)
            if (cpu_replica[t] == r) {
                cpu = cpus[t];
                break;
            }
        std::thread b([&, r, cpu] {
            pin_to(cpu);
            init(ds[r]);
        });
        b.join();
        reps.emplace_back(new Replica<D>(&log, &ds[r]));
    }
    std::atomic<int> ready{0};
    std::atomic<bool> go{false}, stop{false};
    std::vector<uint64_t> cnt(nthreads * 8, 0), wcnt(nthreads * 8, 0);
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < nthreads; t++) {
        th.emplace_back([&, t] {
            pin_to(cpus[t]);
            Replica<D>* rep = reps[cpu_replica[t]].get();
            long tok = rep->reg();
            std::vector<uint32_t> order(nop);
            for (uint64_t i = 0; i < nop; i++) order[i] = (uint32_t)i;
            for (uint64_t i = nop; i > 1; i--) {
                uint64_t j = (uint64_t)(((unsigned __int128)orc_sm64_at(seed + 1000 + t, nop - i) * i) >> 64);
                std::swap(order[i - 1], order[j]);
            }
            ready.fetch_add(1);
            while (!go.load()) spin_pause();
            uint64_t n = 0, w = 0, pos = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                for (int b = 0; b < 128; b++) {
                    w += run(rep, (size_t)tok, order[pos], cpus[t]);
                    pos = pos + 1 == nop ? 0 : pos + 1;
                }
                n += 128;
            }
            cnt[t * 8] = n;
            wcnt[t * 8] = w;
            rep->sync((size_t)tok);
        });
    }
    while (ready.load() < (int)nthreads) std::this_thread::yield();
    auto t0 = std::chrono::steady_clock::now();
    go.store(true);
    std::this_thread::sleep_for(std::chrono::duration<double>(duration_s));
    stop.store(true);
    auto t1 = std::chrono::steady_clock::now();
    for (auto& x : th) x.join();
    uint64_t tot = 0, wt = 0;
    for (uint32_t t = 0; t < nthreads; t++) {
        tot += cnt[t * 8];
        wt += wcnt[t * 8];
    }
    *seconds = std::chrono::duration<double>(t1 - t0).count();
    *ops = tot;
    *writes = wt;
    for (auto& d : ds) fini(d);
}

}  // namespace nrcpu

using namespace nrcpu;

// ======================================================================================
// C API for the ported unit tests (tests/test_control_plane.py).
// Log<u64> with ops encoded as the reference test's `Operation` enum
// (nr/src/log.rs:716-730): 0 = Read, (1<<63)|v = Write(v), 1 = Invalid.
// ======================================================================================
extern "C" {

typedef Log<uint64_t> OLog;

void* orc_log_new(uint64_t bytes) { return new OLog(bytes); }
void* orc_log_default(void) { return new OLog(DEFAULT_LOG_BYTES); }
void orc_log_free(void* l) { delete (OLog*)l; }
uint64_t orc_log_entry_size(void) { return OLog::entry_size(); }
uint64_t orc_log_const(int which) {
    switch (which) {
        case 0: return DEFAULT_LOG_BYTES;
        case 1: return MAX_REPLICAS;
        case 2: return GC_FROM_HEAD;
        case 3: return MAX_PENDING_OPS;
        case 4: return MAX_THREADS_PER_REPLICA;
        default: return 0;
    }
}
// field access: 0 size, 1 rawb, 2 head, 3 tail, 4 ctail, 5 next
uint64_t orc_log_get(void* l, int f) {
    OLog* g = (OLog*)l;
    switch (f) {
        case 0: return g->size_;
        case 1: return g->rawb_;
        case 2: return g->head_.v.load();
        case 3: return g->tail_.v.load();
        case 4: return g->ctail_.v.load();
        case 5: return g->next_.v.load();
        case 6: return g->exec_panicked_;
        default: return 0;
    }
}
void orc_log_set(void* l, int f, uint64_t v) {
    OLog* g = (OLog*)l;
    switch (f) {
        case 2: g->head_.v.store(v); break;
        case 3: g->tail_.v.store(v); break;
        case 4: g->ctail_.v.store(v); break;
        case 5: g->next_.v.store(v); break;
        default: break;
    }
}
uint64_t orc_log_ltail(void* l, uint64_t r) { return ((OLog*)l)->ltails_[r].v.load(); }
void orc_log_set_ltail(void* l, uint64_t r, uint64_t v) { ((OLog*)l)->ltails_[r].v.store(v); }
int orc_log_lmask(void* l, uint64_t r) { return ((OLog*)l)->lmasks_[r]; }
uint64_t orc_log_index(void* l, uint64_t logical) { return ((OLog*)l)->index(logical); }
long orc_log_register(void* l) { return ((OLog*)l)->reg(); }
// entry inspection: returns has_op; *op, *replica
int orc_log_entry(void* l, uint64_t phys, uint64_t* op, uint64_t* replica) {
    OLog* g = (OLog*)l;
    *op = g->slog_[phys].operation;
    *replica = g->slog_[phys].replica;
    return g->slog_[phys].has_op;
}
// append; GC-path dispatches are recorded into (gc_ops, gc_rids) up to cap; returns count
uint64_t orc_log_append(void* l, const uint64_t* ops, uint64_t n, uint64_t idx, uint64_t* gc_ops,
                        uint64_t* gc_rids, uint64_t cap) {
    uint64_t cnt = 0;
    auto s = [&](const uint64_t& o, size_t r) {
        if (cnt < cap) { gc_ops[cnt] = o; gc_rids[cnt] = r; }
        cnt++;
    };
    ((OLog*)l)->append(ops, n, idx, s);
    return cnt;
}
uint64_t orc_log_exec(void* l, uint64_t idx, uint64_t* ops, uint64_t* rids, uint64_t cap) {
    uint64_t cnt = 0;
    auto d = [&](const uint64_t& o, size_t r) {
        if (cnt < cap) { ops[cnt] = o; rids[cnt] = r; }
        cnt++;
    };
    ((OLog*)l)->exec(idx, d);
    return cnt;
}
void orc_log_advance_head(void* l, uint64_t rid) {
    auto d = [](const uint64_t&, size_t) {};
    ((OLog*)l)->advance_head(rid, d);
}
void orc_log_reset(void* l) { ((OLog*)l)->reset(); }
int orc_log_synced(void* l, uint64_t idx, uint64_t ctail) {
    return ((OLog*)l)->is_replica_synced_for_reads(idx, ctail);
}
uint64_t orc_log_get_ctail(void* l) { return ((OLog*)l)->get_ctail(); }

// ---- Context test API (u64 ops, u64 responses) ----
typedef Context<uint64_t, uint64_t> OCtx;
void* orc_ctx_new(void) { return new OCtx(); }
void orc_ctx_free(void* c) { delete (OCtx*)c; }
int orc_ctx_enqueue(void* c, uint64_t op) { return ((OCtx*)c)->enqueue(op); }
void orc_ctx_enqueue_resps(void* c, const uint64_t* r, uint64_t n) { ((OCtx*)c)->enqueue_resps(r, n); }
uint64_t orc_ctx_ops(void* c, uint64_t* out, uint64_t cap) {
    std::vector<uint64_t> b;
    uint64_t n = ((OCtx*)c)->ops(b);
    for (uint64_t i = 0; i < n && i < cap; i++) out[i] = b[i];
    return n;
}
int orc_ctx_res(void* c, uint64_t* out) { return ((OCtx*)c)->res(out); }
// 0 tail, 1 head, 2 comb, 3 panicked
uint64_t orc_ctx_get(void* c, int f) {
    OCtx* x = (OCtx*)c;
    return f == 0 ? x->tail.load() : f == 1 ? x->head.load() : f == 2 ? x->comb.load() : x->panicked;
}
void orc_ctx_set(void* c, int f, uint64_t v) {
    OCtx* x = (OCtx*)c;
    if (f == 0) x->tail.store(v);
    else if (f == 1) x->head.store(v);
    else if (f == 2) x->comb.store(v);
}

// ---- Replica<JunkD> test API (nr/src/replica.rs:598-788) ----
struct JunkReplica {
    OLog log;
    JunkD d;
    Replica<JunkD> r;
    explicit JunkReplica(uint64_t bytes) : log(bytes), r(&log, &d) {}
};
void* orc_rep_new(uint64_t log_bytes) { return new JunkReplica(log_bytes ? log_bytes : DEFAULT_LOG_BYTES); }
void orc_rep_free(void* p) { delete (JunkReplica*)p; }
long orc_rep_register(void* p) { return ((JunkReplica*)p)->r.reg(); }
// 0 idx, 1 combiner, 2 next, 3 junk
uint64_t orc_rep_get(void* p, int f) {
    JunkReplica* x = (JunkReplica*)p;
    return f == 0 ? x->r.idx_ : f == 1 ? x->r.combiner_.v.load() : f == 2 ? x->r.next_.v.load() : x->d.junk;
}
void orc_rep_set(void* p, int f, uint64_t v) {
    JunkReplica* x = (JunkReplica*)p;
    if (f == 1) x->r.combiner_.v.store(v);
    if (f == 2) x->r.next_.v.store(v);
}
int orc_rep_make_pending(void* p, uint64_t op, uint64_t tid) { return ((JunkReplica*)p)->r.make_pending(op, tid); }
void orc_rep_try_combine(void* p, uint64_t tid) { ((JunkReplica*)p)->r.try_combine(tid); }
uint64_t orc_rep_execute_mut(void* p, uint64_t op, uint64_t tid) { return ((JunkReplica*)p)->r.execute_mut(op, tid); }
uint64_t orc_rep_execute(void* p, uint64_t op, uint64_t tid) { return ((JunkReplica*)p)->r.execute(op, tid); }
uint64_t orc_rep_get_response(void* p, uint64_t tid) { return ((JunkReplica*)p)->r.get_response(tid); }
int orc_rep_ctx_res(void* p, uint64_t tid, uint64_t* out) { return ((JunkReplica*)p)->r.contexts_[tid - 1].res(out); }
// raw slog.append(&o, rid, ..) + slog.exec(rid, ..) "off the side" (replica.rs:781-783)
void orc_rep_log_append_exec(void* p, const uint64_t* ops, uint64_t n, uint64_t rid) {
    JunkReplica* x = (JunkReplica*)p;
    auto f = [](const uint64_t&, size_t) {};
    x->log.append(ops, n, rid, f);
    x->log.exec(rid, f);
}

// ======================================================================================
// Multi-threaded CPU baseline: NrHashMap scale-out (benches/hashmap.rs:226-259 through
// benches/mkbench.rs:640-831), one Replica per CPU group, pinned worker threads, each
// thread replaying its own shuffled copy of the op stream; 128 ops per clock check.
// ======================================================================================
struct BenchResult {
    double seconds;
    uint64_t ops;
    uint64_t writes;
    uint64_t reads;
};

int orc_nr_hashmap_bench(uint32_t nreplicas, const int* cpus, const uint32_t* cpu_replica,
                         uint32_t nthreads, double duration_s, uint32_t write_ratio,
                         uint64_t key_space, uint64_t prefill, uint64_t nop, uint64_t seed,
                         uint64_t log_bytes, BenchResult* out) {
    if (nreplicas == 0 || nthreads == 0) return -1;
    std::vector<uint8_t> isput(nop);
    std::vector<uint64_t> keys(nop), vals(nop);
    orc_gen_hashmap_ops(isput.data(), keys.data(), vals.data(), nop, seed, key_space, write_ratio);
    volatile uint64_t sink = 0;
    scale_out<HashMapD>(
        nreplicas, cpus, cpu_replica, nthreads, duration_s, nop, seed, log_bytes,
        [&](HashMapD& d) {
            d.m = orc_hm_new(prefill);
            orc_hm_prefill_range(d.m, prefill, 1);
        },
        [&](Replica<HashMapD>* rep, size_t tok, uint32_t i, int) -> uint64_t {
            if (isput[i]) {  // benches/hashmap.rs:226-259
                sink += rep->execute_mut(HmOp{keys[i], vals[i]}, tok).some;
                return 1;
            }
            sink += rep->execute(keys[i], tok).val;
            return 0;
        },
        [](HashMapD& d) { orc_hm_free(d.m); }, &out->seconds, &out->ops, &out->writes);
    out->reads = out->ops - out->writes;
    return 0;
}

// Stack scale-out (benches/stack.rs:115-134): every op an execute_mut of Push/Pop from the
// shared stream (orc_gen_stack_ops, 50/50), Stack::default (0..50000) per replica.
int orc_nr_stack_bench(uint32_t nreplicas, const int* cpus, const uint32_t* cpu_replica, uint32_t nthreads,
                       double duration_s, uint64_t nop, uint64_t seed, uint64_t log_bytes, BenchResult* out) {
    if (nreplicas == 0 || nthreads == 0) return -1;
    std::vector<uint32_t> v(nop), o(nop);
    orc_gen_stack_ops(v.data(), o.data(), nop, seed);
    std::vector<uint64_t> ops(nop);
    for (uint64_t i = 0; i < nop; i++) ops[i] = ((uint64_t)(o[i] & 1) << 32) | v[i];
    volatile uint64_t sink = 0;
    scale_out<StackD>(
        nreplicas, cpus, cpu_replica, nthreads, duration_s, nop, seed, log_bytes,
        [](StackD& d) {
            d.storage.reserve(1 << 20);
            for (uint32_t e = 0; e < 50000; e++) d.storage.push_back(e);
        },
        [&](Replica<StackD>* rep, size_t tok, uint32_t i, int) -> uint64_t {
            sink += rep->execute_mut(ops[i], tok);
            return 1;
        },
        [](StackD&) {}, &out->seconds, &out->ops, &out->writes);
    out->reads = 0;
    return 0;
}

// Synthetic scale-out (benches/synthetic.rs:296-335): ReadWrite ops only
// (generate_operations(NOP, 0, false, false, true)), tid set to the issuing thread's core id
// (o.set_tid(cid)), r1/r2 from the seeded stream.
int orc_nr_synth_bench(uint32_t nreplicas, const int* cpus, const uint32_t* cpu_replica, uint32_t nthreads,
                       double duration_s, uint64_t nop, uint64_t seed, uint64_t log_bytes, BenchResult* out) {
    if (nreplicas == 0 || nthreads == 0) return -1;
    std::vector<uint64_t> raw(2 * nop);
    orc_gen_raw(raw.data(), 2 * nop, seed);
    volatile uint64_t sink = 0;
    scale_out<SynthD>(
        nreplicas, cpus, cpu_replica, nthreads, duration_s, nop, seed, log_bytes, [](SynthD& d) { d.init(); },
        [&](Replica<SynthD>* rep, size_t tok, uint32_t i, int cpu) -> uint64_t {
            SyOp o{(uint64_t)(cpu < 0 ? 0 : cpu), raw[2 * i], raw[2 * i + 1], 1};
            sink += rep->execute_mut(o, tok);
            return 1;
        },
        [](SynthD&) {}, &out->seconds, &out->ops, &out->writes);
    out->reads = 0;
    return 0;
}

// Parity hooks for the two D's above (tests/test_control_plane.py): one thread replays a
// given op stream through Replica<D> (append + exec + responses) and returns every response
// and the final state, to be compared with the sequential oracle.
uint64_t orc_nr_stack_run(const uint32_t* init, uint64_t ninit, const uint32_t* vals, const uint32_t* kinds,
                          uint64_t n, uint64_t* resp, uint32_t* final_out, uint64_t cap) {
    Log<uint64_t> log(2 * 1024 * 1024);
    StackD d;
    d.storage.assign(init, init + ninit);
    Replica<StackD> rep(&log, &d);
    long tok = rep.reg();
    for (uint64_t i = 0; i < n; i++) resp[i] = rep.execute_mut(((uint64_t)(kinds[i] & 1) << 32) | vals[i], (size_t)tok);
    rep.sync((size_t)tok);
    uint64_t len = d.storage.size();
    for (uint64_t i = 0; i < len && i < cap; i++) final_out[i] = d.storage[i];
    return len;
}

void orc_nr_synth_run(const uint64_t* ops4, uint64_t n, const uint64_t* reads3, uint64_t nr, uint64_t* resp,
                      uint64_t* rresp, uint64_t* final_out) {
    Log<SyOp> log(2 * 1024 * 1024);
    SynthD d;
    d.init();
    Replica<SynthD> rep(&log, &d);
    long tok = rep.reg();
    for (uint64_t i = 0; i < n; i++)
        resp[i] = rep.execute_mut(SyOp{ops4[4 * i], ops4[4 * i + 1], ops4[4 * i + 2], ops4[4 * i + 3]}, (size_t)tok);
    for (uint64_t i = 0; i < nr; i++)
        rresp[i] = rep.execute(SyOp{reads3[3 * i], reads3[3 * i + 1], reads3[3 * i + 2], 0}, (size_t)tok);
    for (uint64_t i = 0; i < d.n; i++) final_out[i] = d.storage[i].v;
}

}  // extern "C"
