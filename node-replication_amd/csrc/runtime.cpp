// runtime.cpp — the nrgpu C ABI (include/nrgpu.h): replica lifetime, the per-replica HBM
// log ring with the reference's head/tail/ctail/ltail bookkeeping, and dispatch of the
// replay pipelines (hashmap.hip, stack.hip, synthetic.hip).
//
// Log bookkeeping follows nr/src/log.rs: Log::new sizing (:179-242), append with GC when
// fewer than GC_FROM_HEAD entries would remain (:343-427, :536-580), exec of
// [ltail, tail) (:473-524) followed by ctail = max(ctail, tail) and ltail = tail (:522-523).
// Each GPU context holds its own copy of the shared log (the all-gather of write segments
// makes every copy identical), so head = min over replicas = this ltail.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>

#include "internal.hpp"
#include "../../include/nrgpu_testing.h"

using namespace nrg;

namespace {

constexpr uint64_t GC_FROM_HEAD = 32 * 256;  // MAX_PENDING_OPS * MAX_THREADS_PER_REPLICA
constexpr uint64_t ENTRY_BYTES = 64;         // size_of::<Entry<T>>() in the reference
constexpr uint64_t DEFAULT_LOG_BYTES = 32ull << 20;

uint64_t pow2_at_least(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

uint32_t bits_for(uint64_t maxval) {  // smallest b with (1<<b)-1 >= maxval
    uint32_t b = 1;
    while (((1ull << b) - 1) < maxval) b++;
    return b;
}

int hip_fail(hipError_t e) {
    if (e == hipSuccess) return NRG_OK;
    if (e == hipErrorOutOfMemory) return NRG_E_NOMEM;
    return NRG_E_HIP;
}

#define HIPCHK(x)                                \
    do {                                         \
        hipError_t _e = (x);                     \
        if (_e != hipSuccess) return hip_fail(_e); \
    } while (0)

uint32_t rec_bytes_for(uint32_t kind) {
    switch (kind) {
        case NRG_DS_HASHMAP: return sizeof(nrg_put);
        case NRG_DS_STACK: return sizeof(nrg_stack_op);
        case NRG_DS_SYNTHETIC: return sizeof(nrg_synth_op);
        default: return 0;
    }
}

thread_local int g_dev_set = -1;

int use_device(nrg_ctx* c) {
    if (g_dev_set != c->device) {
        HIPCHK(hipSetDevice(c->device));
        g_dev_set = c->device;
    }
    return NRG_OK;
}

// the deferred half of the last hashmap round (hashmap.hip), the deferred finish of the last
// stack chunk (stack.hip) or the deferred sums of the last synthetic chunk (synthetic.hip),
// launched now if there is one
hipError_t hm_flush_if(nrg_ctx* c) {
    if (c->cfg.ds_kind == NRG_DS_HASHMAP) return hm_flush(c);
    if (c->cfg.ds_kind == NRG_DS_STACK) return st_flush(c);
    return sy_flush(c);
}

// Log GC boundary: the slowest replica's tail (this replica's ltail), held back to the first
// record of a deferred hashmap stamp round, whose apply and reads take values from the ring.
uint64_t gc_head(const nrg_ctx* c) {
    const nrg::HmDeferred& p = c->pend;
    if (p.valid && p.apply && !p.src && p.lo < c->ltail) return p.lo;
    return c->ltail;
}

// wait for everything queued on this replica, including a deferred hashmap round
hipError_t sync_all(nrg_ctx* c) {
    hipError_t e = hm_flush_if(c);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(c->stream);
}

int check_err(nrg_ctx* c) {
    uint32_t err = 0;
    HIPCHK(hipMemcpyAsync(&err, &c->d_ctl->err, sizeof(err), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(sync_all(c));
    if (err) {
        uint32_t z = 0;
        HIPCHK(hipMemcpyAsync(&c->d_ctl->err, &z, sizeof(z), hipMemcpyHostToDevice, c->stream));
        HIPCHK(sync_all(c));
        if (err & ERR_TABLE_FULL) return NRG_E_TABLE_FULL;
        if (err & ERR_CAPACITY) return NRG_E_CAPACITY;
        if (err & ERR_GROUP) return NRG_E_INVAL;
        return NRG_E_HIP;
    }
    return NRG_OK;
}

// replay [ltail, tail) in order, in chunks of at most max_batch records
int exec_range(nrg_ctx* c, uint64_t resp_lo, uint64_t resp_hi, void* d_resp, uint8_t* d_some) {
    while (c->ltail < c->tail) {
        uint64_t n = c->tail - c->ltail;
        if (n > c->cfg.max_batch) n = c->cfg.max_batch;
        const uint64_t lo = c->ltail;
        hipError_t e = hipSuccess;
        switch (c->cfg.ds_kind) {
            case NRG_DS_HASHMAP:
                e = hm_replay_chunk(c, nullptr, lo, n, false, nullptr, 0, nullptr, nullptr, resp_lo, resp_hi,
                                    (u64*)d_resp, d_some);
                break;
            case NRG_DS_STACK:
                e = st_replay_chunk(c, lo, n, resp_lo, resp_hi, (uint32_t*)d_resp, d_some);
                break;
            case NRG_DS_SYNTHETIC:
                e = sy_replay_chunk(c, lo, n, resp_lo, resp_hi, (u64*)d_resp, d_some);
                break;
            default: return NRG_E_INVAL;
        }
        if (e != hipSuccess) return hip_fail(e);
        c->ltail = lo + n;
    }
    if (c->ctail < c->ltail) c->ctail = c->ltail;
    return NRG_OK;
}

// Make room for n records (Log::append's GC path): advance head to the slowest replica's
// tail (this replica's ltail), replaying first if nothing can be freed.
int reserve(nrg_ctx* c, uint64_t n) {
    if (n > c->log_size - GC_FROM_HEAD) return NRG_E_RING_FULL;
    if (c->tail + n > c->head + c->log_size - GC_FROM_HEAD) {
        c->head = gc_head(c);
        if (c->tail + n > c->head + c->log_size - GC_FROM_HEAD) {
            int r = exec_range(c, 0, 0, nullptr, nullptr);
            if (r != NRG_OK) return r;
            HIPCHK(hm_flush_if(c));
            c->head = gc_head(c);
        }
    }
    return NRG_OK;
}

void note_origin(nrg_ctx* c, uint64_t first, uint64_t n, uint32_t origin) {
    if (!c->origins.empty()) {
        HostRun& b = c->origins.back();
        if (b.origin == origin && b.first + b.count == first) {
            b.count += n;
            return;
        }
    }
    c->origins.push_back(HostRun{first, n, origin});
    // keep only runs that are still inside the live window
    size_t drop = 0;
    while (drop < c->origins.size() && c->origins[drop].first + c->origins[drop].count <= c->head) drop++;
    if (drop) c->origins.erase(c->origins.begin(), c->origins.begin() + drop);
}

int copy_into_ring(nrg_ctx* c, const void* src, uint64_t n, hipMemcpyKind kind) {
    const uint64_t phys = c->tail & (c->log_size - 1);
    const uint64_t first = n < c->log_size - phys ? n : c->log_size - phys;
    char* ring = (char*)c->d_ring;
    const char* s = (const char*)src;
    HIPCHK(hipMemcpyAsync(ring + phys * c->rec_bytes, s, first * c->rec_bytes, kind, c->stream));
    if (first < n)
        HIPCHK(hipMemcpyAsync(ring, s + first * c->rec_bytes, (n - first) * c->rec_bytes, kind, c->stream));
    return NRG_OK;
}

int staging(nrg_ctx* c, Staging& st, uint64_t bytes) {
    if (st.bytes >= bytes) return NRG_OK;
    if (st.p) (void)hipFree(st.p);
    st.p = nullptr;
    st.bytes = 0;
    uint64_t b = bytes < 4096 ? 4096 : bytes;
    HIPCHK(hipMalloc(&st.p, b));
    st.bytes = b;
    (void)c;
    return NRG_OK;
}

}  // namespace

namespace nrg {
int ctx_use_device(nrg_ctx* c) { return use_device(c); }

int hm_small_job(nrg_ctx* c, const nrg_put* recs, u64 W, u32 origin, const u64* keys, u64 R, u64* vals,
                 uint8_t* found, u64* prev, uint8_t* prevf, u32* e_out, SmallJobBlob* blob, u64* lo_out) {
    if (!c || c->cfg.ds_kind != NRG_DS_HASHMAP || W > c->cfg.max_batch || c->ltail != c->tail) return NRG_E_INVAL;
    if ((W && !recs) || (R && (!keys || !vals || !found))) return NRG_E_INVAL;
    if (W > c->log_size - GC_FROM_HEAD) return NRG_E_INVAL;
    int r = reserve(c, W);  // (caught up and nothing deferred: only moves head, launches nothing)
    if (r) return r;
    const uint64_t lo = c->tail;
    if (!hm_small_fill(c, recs, lo, W, keys, R, vals, found, prev, prevf, e_out, blob)) return NRG_E_INVAL;
    if (lo_out) *lo_out = lo;
    c->rounds++;
    if (W) note_origin(c, lo, W, origin);
    c->tail = lo + W;
    c->ltail = c->tail;
    if (c->ctail < c->tail) c->ctail = c->tail;
    return NRG_OK;
}
// c->timing_only: empty (time every kernel) or a comma-separated list of kernel names
static bool timer_match(const nrg_ctx* c, const char* name) {
    if (c->timing_only.empty()) return true;
    const std::string& w = c->timing_only;
    const size_t n = std::strlen(name);
    for (size_t p = 0; (p = w.find(name, p)) != std::string::npos; p++)
        if ((p == 0 || w[p - 1] == ',') && (p + n == w.size() || w[p + n] == ',')) return true;
    return false;
}
// HIP events around a kernel, recorded on the stream that kernel is launched on. When
// c->timing_only is set, only the kernels it names are bracketed (keeps event packets off
// the others).
void timer_begin(nrg_ctx* c, const char* name, hipStream_t s) {
    if (!c->timing || !timer_match(c, name)) return;
    KTimer& t = c->timers[name];
    t.open = false;
    if (++t.seen % c->timing_every != 0) return;  // sampled, as timer_events
    const size_t idx = t.pending * 2;
    while (t.ev.size() < idx + 2) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return;
        t.ev.push_back(e);
    }
    (void)hipEventRecord(t.ev[idx], s ? s : c->stream);
    t.open = true;
}
bool timer_events(nrg_ctx* c, const char* name, hipEvent_t* start, hipEvent_t* stop) {
    if (!c->timing || !timer_match(c, name)) return false;
    KTimer& t = c->timers[name];
    // sampled: launches every-1, 2*every-1, ... (skips a stream's first launch when every > 1)
    if (++t.seen % c->timing_every != 0) return false;
    const size_t idx = t.pending * 2;
    while (t.ev.size() < idx + 2) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return false;
        t.ev.push_back(e);
    }
    *start = t.ev[idx];
    *stop = t.ev[idx + 1];
    t.pending++;
    return true;
}
void timer_end(nrg_ctx* c, const char* name, hipStream_t s) {
    if (!c->timing || !timer_match(c, name)) return;
    KTimer& t = c->timers[name];
    if (!t.open) return;
    (void)hipEventRecord(t.ev[t.pending * 2 + 1], s ? s : c->stream);
    t.pending++;
    t.open = false;
}
}  // namespace nrg

static Staging* stg(nrg_ctx* c) { return c->stg; }

extern "C" {

void nrg_config_default(nrg_config* cfg, uint32_t ds_kind) {
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->ds_kind = ds_kind;
    cfg->log2_slots = 26;
    cfg->log_bytes = DEFAULT_LOG_BYTES;
    cfg->max_batch = 1u << 20;
    cfg->max_reads = 1u << 20;
    cfg->stack_capacity = 1u << 24;
    cfg->synth_n = 200000;
    cfg->synth_cold_reads = 20;
    cfg->synth_cold_writes = 5;
    cfg->synth_hot_reads = 2;
    cfg->synth_hot_writes = 1;
    cfg->stack_push_resp = 0;
    cfg->replica_id = 1;
    cfg->pipeline = 0;  // opt-in: see nrg_config.pipeline
}

const char* nrg_strerror(int code) {
    switch (code) {
        case NRG_OK: return "ok";
        case NRG_E_INVAL: return "invalid argument";
        case NRG_E_HIP: return "HIP runtime error";
        case NRG_E_TABLE_FULL: return "hash table full";
        case NRG_E_RING_FULL: return "log ring full";
        case NRG_E_NOMEM: return "device out of memory";
        case NRG_E_NOT_SYNCED: return "replica not synced to the log tail";
        case NRG_E_CAPACITY: return "capacity exceeded";
        case NRG_E_NODEV: return "no such HIP device";
        case NRG_E_COMM: return "RCCL unavailable or a collective failed";
        case NRG_E_TIMEOUT: return "a peer rank missed the replica group's deadline for a collective";
        default: return "unknown error";
    }
}

const char* nrg_version(void) { return "nrgpu 0.2 gfx950"; }

int nrg_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int nrg_close(nrg_ctx* c);

int nrg_open(int dev, const nrg_config* cfg_in, nrg_ctx** out) {
    if (!cfg_in || !out) return NRG_E_INVAL;
    *out = nullptr;
    const uint32_t rb = rec_bytes_for(cfg_in->ds_kind);
    if (!rb) return NRG_E_INVAL;
    int ndev = nrg_device_count();
    if (dev < 0 || dev >= ndev) return NRG_E_NODEV;
    nrg_ctx* c = new (std::nothrow) nrg_ctx();
    if (!c) return NRG_E_NOMEM;
    c->device = dev;
    c->cfg = *cfg_in;
    nrg_config& cf = c->cfg;
    if (!cf.max_batch) cf.max_batch = 1u << 20;
    if (!cf.max_reads) cf.max_reads = 1u << 20;
    if (!cf.replica_id) cf.replica_id = 1;
    if (cf.max_batch >= (1ull << 30)) { delete c; return NRG_E_INVAL; }
    c->rec_bytes = rb;
    g_dev_set = -1;
    int rc = use_device(c);
    if (rc != NRG_OK) { delete c; return rc; }
#define OPEN_CHK(x)                   \
    do {                              \
        hipError_t _e = (x);          \
        if (_e != hipSuccess) {       \
            nrg_close(c);             \
            return hip_fail(_e);      \
        }                             \
    } while (0)
    OPEN_CHK(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
    c->stream = c->own_stream;

    // Log::new(bytes): entries = bytes / 64, at least 2*GC_FROM_HEAD, power of two.
    uint64_t lb = cf.log_bytes ? cf.log_bytes : DEFAULT_LOG_BYTES;
    uint64_t num = lb / ENTRY_BYTES;
    if (num < 2 * GC_FROM_HEAD) num = 2 * GC_FROM_HEAD;
    c->log_size = pow2_at_least(num);
    OPEN_CHK(hipMalloc(&c->d_ring, c->log_size * rb));
    OPEN_CHK(hipMalloc(&c->d_ctl, sizeof(DevCtl)));
    OPEN_CHK(hipMemsetAsync(c->d_ctl, 0, sizeof(DevCtl), c->stream));

    const uint64_t mb = cf.max_batch;
    if (cf.ds_kind == NRG_DS_HASHMAP) {
        // slot ids are < 2^30 (entry ids carry two flag values above them, hashmap.hip);
        // replay chunks are bounded by the partition rounds' 16-bit tile offsets (HM_MAX_BATCH)
        if (cf.log2_slots < 4 || cf.log2_slots > 30 || mb > HM_MAX_BATCH) { nrg_close(c); return NRG_E_INVAL; }
        c->slots = 1ull << cf.log2_slots;
        c->slot_shift = 64 - cf.log2_slots;
        OPEN_CHK(hipMalloc(&c->d_table, c->slots * sizeof(Slot)));
        OPEN_CHK(hm_init(c));
        OPEN_CHK(hipMalloc(&c->d_created, HM_CREATED_SLOTS * sizeof(uint64_t)));
        OPEN_CHK(hipMemsetAsync(c->d_created, 0, HM_CREATED_SLOTS * sizeof(uint64_t), c->stream));
        // rounds without previous values replay in one launch (stamp rounds) unless the key
        // stream is skewed (hashmap.hip skew_sample) or the round is large (PART_MIN); skewed,
        // large and previous-value rounds take partition rounds
        c->stamp_max = HM_MAX_BATCH;  // (NRG_KNOB_STAMP_MAX lowers it for tests)
        OPEN_CHK(hm_alloc(c, mb));       // clamps stamp_max to max_batch (the put_slot arrays' size)
        c->stamp_alloc = c->stamp_max;
        c->pipeline = cf.pipeline != 0;
    } else if (cf.ds_kind == NRG_DS_STACK) {
        // max_batch <= 2^24: the finish stages one minimum per tile in LDS (stack.hip)
        if (!cf.stack_capacity || cf.stack_capacity >= (1ull << 31) || mb > (1ull << 24)) {
            nrg_close(c);
            return NRG_E_INVAL;
        }
        OPEN_CHK(hipMalloc(&c->d_stack, cf.stack_capacity * sizeof(uint32_t)));
        // look-back descriptors of both tile parities (stack.hip st_pass), and at least what
        // nrg_test_maxscan's 2048-key tiles use
        c->scan_desc_words = std::max<uint64_t>(st_desc_words(mb), 2 * (32 + (mb + 2047) / 2048));
        OPEN_CHK(hipMalloc(&c->d_scan_desc, c->scan_desc_words * 4));
        OPEN_CHK(hipMemsetAsync(c->d_scan_desc, 0, c->scan_desc_words * 4, c->stream));
        OPEN_CHK(hipMalloc(&c->d_st_aux, st_aux_bytes(mb)));
        c->pipeline = cf.pipeline != 0;
    } else {
        const uint64_t T = cf.synth_hot_writes + cf.synth_cold_writes;
        if (!cf.synth_n || cf.synth_hot_reads == 0 || cf.synth_n <= cf.synth_hot_reads || T == 0 || T > 64 ||
            mb * T >= (1ull << 31) || cf.synth_n >= (1ull << 31)) {
            nrg_close(c);
            return NRG_E_INVAL;
        }
        OPEN_CHK(hipMalloc(&c->d_words, cf.synth_n * sizeof(uint64_t)));
        c->synth_key_bits = bits_for(cf.synth_n);
        OPEN_CHK(hipMalloc(&c->d_tmp_u64, mb * T * sizeof(uint64_t)));
        c->tmp_words = mb * T;
        OPEN_CHK(hipMalloc(&c->d_sort_aux, mb * T * sizeof(uint32_t)));
        c->scan_desc_words = 2 * (32 + (mb * T + 2047) / 2048);
        OPEN_CHK(hipMalloc(&c->d_scan_desc, c->scan_desc_words * 4));
        if (sort_alloc(c->sort, mb * T) != NRG_OK) { nrg_close(c); return NRG_E_NOMEM; }
        // sort-free bucket replay where the config allows it (the sort path stays for the rest;
        // nrg_test_set_knob(NRG_KNOB_SY_SORT) forces it for tests)
        if (sy_bucket_eligible(cf)) {
            OPEN_CHK(hipMalloc(&c->d_sy_aux, sy_bucket_aux_bytes(cf)));
            OPEN_CHK(sy_aux_init(c));
        }
        c->pipeline = cf.pipeline != 0;
        OPEN_CHK(sy_init(c));
    }
    OPEN_CHK(hipStreamSynchronize(c->stream));
#undef OPEN_CHK
    *out = c;
    return NRG_OK;
}

int nrg_close(nrg_ctx* c) {
    if (!c) return NRG_E_INVAL;
    (void)hipSetDevice(c->device);
    g_dev_set = c->device;
    if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
    if (c->stream && c->stream != c->own_stream) (void)hipStreamSynchronize(c->stream);
    void* ptrs[] = {c->d_ring,    c->d_ctl,      c->d_table,    c->d_stack,  c->d_words,
                    c->d_sort_aux, c->d_tmp_u64, c->d_scan_desc, c->d_created, c->d_st_aux,
                    c->d_sy_aux,  c->d_bk_ent,   c->d_bk_idx,   c->d_bk_cnt, c->d_dbg,     c->d_pt};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    sort_free(c->sort);
    hm_free(c);
    Staging* s = stg(c);
    for (int i = 0; i < 4; i++)
        if (s[i].p) (void)hipFree(s[i].p);
    for (auto& kv : c->timers)
        for (hipEvent_t e : kv.second.ev) (void)hipEventDestroy(e);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return NRG_OK;
}

int nrg_set_stream(nrg_ctx* c, void* s) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    // deferred hashmap work belongs to the old stream: launch it there first
    hipError_t e = hm_flush_if(c);
    if (e != hipSuccess) return hip_fail(e);
    hipStream_t ns = (hipStream_t)s;  // NULL: the device's null stream, as in HIP
    if (ns != c->stream) {
        // everything already queued on the old stream (the replica's table, ring and scratch)
        // comes before anything the new stream runs from now on
        hipEvent_t ev;
        HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        e = hipEventRecord(ev, c->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(ns, ev, 0);
        (void)hipEventDestroy(ev);
        if (e != hipSuccess) return hip_fail(e);
    }
    c->stream = ns;
    return NRG_OK;
}

void* nrg_get_stream(nrg_ctx* c) { return c ? (void*)c->stream : nullptr; }

void* nrg_own_stream(nrg_ctx* c) { return c ? (void*)c->own_stream : nullptr; }

int nrg_sync(nrg_ctx* c) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    HIPCHK(sync_all(c));
    return check_err(c);
}

int nrg_join(nrg_ctx* c) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    HIPCHK(hm_flush_if(c));
    return NRG_OK;
}

// ---- Log -------------------------------------------------------------------------------
static int append_common(nrg_ctx* c, const void* recs, uint64_t n, uint32_t origin, uint64_t* first_idx,
                         hipMemcpyKind kind) {
    if (!c || (!recs && n)) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    if (n == 0) {
        if (first_idx) *first_idx = c->tail;
        return NRG_OK;
    }
    if ((r = reserve(c, n)) != NRG_OK) return r;
    if ((r = copy_into_ring(c, recs, n, kind)) != NRG_OK) return r;
    if (first_idx) *first_idx = c->tail;
    note_origin(c, c->tail, n, origin);
    c->tail += n;
    return NRG_OK;
}

int nrg_log_append(nrg_ctx* c, const void* recs, uint64_t n, uint32_t origin, uint64_t* first_idx) {
    int r = append_common(c, recs, n, origin, first_idx, hipMemcpyHostToDevice);
    if (r) return r;
    HIPCHK(sync_all(c));
    return NRG_OK;
}

int nrg_log_append_async(nrg_ctx* c, const void* d_recs, uint64_t n, uint32_t origin, uint64_t* first_idx) {
    return append_common(c, d_recs, n, origin, first_idx, hipMemcpyDeviceToDevice);
}

int nrg_log_append_segments_async(nrg_ctx* c, const void* d_base, uint32_t nseg, uint64_t seg_stride,
                                  const uint64_t* lens, const uint32_t* origins, uint64_t* first_idx) {
    if (!c || !lens || nseg == 0 || nseg > 64) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    uint64_t total = 0;
    for (uint32_t s = 0; s < nseg; s++) {
        if (lens[s] > seg_stride) return NRG_E_INVAL;
        total += lens[s];
    }
    if ((r = reserve(c, total)) != NRG_OK) return r;
    hipError_t e = copy_segments(c, d_base, nseg, seg_stride, lens, c->tail);
    if (e != hipSuccess) return hip_fail(e);
    for (uint32_t s = 0; s < nseg; s++) {
        if (first_idx) first_idx[s] = c->tail;
        if (lens[s]) note_origin(c, c->tail, lens[s], origins ? origins[s] : s + 1);
        c->tail += lens[s];
    }
    return NRG_OK;
}

int nrg_log_exec_async(nrg_ctx* c, uint64_t resp_lo, uint64_t resp_hi, void* d_resp, uint8_t* d_some) {
    if (!c || resp_hi < resp_lo) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    if (!d_resp || !d_some) {
        d_resp = nullptr;
        d_some = nullptr;
    }
    return exec_range(c, resp_lo, resp_hi, d_resp, d_some);
}

static uint64_t resp_elem_bytes(const nrg_ctx* c) {
    return c->cfg.ds_kind == NRG_DS_STACK ? 4 : 8;
}

int nrg_log_exec(nrg_ctx* c, uint64_t resp_lo, uint64_t resp_hi, void* resp, uint8_t* some) {
    if (!c || resp_hi < resp_lo) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    const uint64_t w = (resp && some) ? resp_hi - resp_lo : 0;
    void* dr = nullptr;
    uint8_t* ds = nullptr;
    Staging* s = stg(c);
    if (w) {
        const uint64_t eb = resp_elem_bytes(c);
        if ((r = staging(c, s[0], w * eb)) || (r = staging(c, s[1], w))) return r;
        dr = s[0].p;
        ds = (uint8_t*)s[1].p;
        HIPCHK(hipMemsetAsync(dr, 0, w * eb, c->stream));
        HIPCHK(hipMemsetAsync(ds, 0, w, c->stream));
    }
    if ((r = exec_range(c, resp_lo, resp_hi, dr, ds))) return r;
    HIPCHK(hm_flush_if(c));  // deferred work writes responses too: complete them before the copy
    if (w) {
        HIPCHK(hipMemcpyAsync(resp, dr, w * resp_elem_bytes(c), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(some, ds, w, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(sync_all(c));
    return check_err(c);
}

int nrg_log_state(const nrg_ctx* c, nrg_log_info* o) {
    if (!c || !o) return NRG_E_INVAL;
    o->size = c->log_size;
    o->head = c->head;
    o->tail = c->tail;
    o->ctail = c->ctail;
    o->ltail = c->ltail;
    o->replica_id = c->cfg.replica_id;
    o->ds_kind = c->cfg.ds_kind;
    return NRG_OK;
}

int nrg_log_reset(nrg_ctx* c) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    // a deferred hashmap read batch belongs to the log positions being reset: answer it now
    HIPCHK(hm_flush_if(c));
    c->head = c->tail = c->ctail = c->ltail = 0;
    c->origins.clear();
    return NRG_OK;
}

// ---- NrHashMap ---------------------------------------------------------------------------
static int need(nrg_ctx* c, uint32_t kind) {
    if (!c) return NRG_E_INVAL;
    if (c->cfg.ds_kind != kind) return NRG_E_INVAL;
    return use_device(c);
}

int nrg_hashmap_get_async(nrg_ctx* c, const uint64_t* d_keys, uint64_t n, uint64_t* d_vals, uint8_t* d_found) {
    int r = need(c, NRG_DS_HASHMAP);
    if (r) return r;
    if (c->ltail != c->tail) return NRG_E_NOT_SYNCED;
    if (n && (!d_keys || !d_vals || !d_found)) return NRG_E_INVAL;
    return hip_fail(hm_get_only(c, d_keys, n, d_vals, d_found));
}

int nrg_hashmap_get(nrg_ctx* c, const uint64_t* keys, uint64_t n, uint64_t* vals, uint8_t* found) {
    int r = need(c, NRG_DS_HASHMAP);
    if (r) return r;
    if (c->ltail != c->tail) return NRG_E_NOT_SYNCED;
    if (n == 0) return NRG_OK;
    Staging* s = stg(c);
    if ((r = staging(c, s[0], n * 8)) || (r = staging(c, s[1], n * 8)) || (r = staging(c, s[2], n))) return r;
    HIPCHK(hipMemcpyAsync(s[0].p, keys, n * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hm_get_only(c, (u64*)s[0].p, n, (u64*)s[1].p, (uint8_t*)s[2].p));
    HIPCHK(hipMemcpyAsync(vals, s[1].p, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(found, s[2].p, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(sync_all(c));
    return check_err(c);
}

int nrg_hashmap_round_async(nrg_ctx* c, const nrg_put* d_puts, uint64_t W, uint32_t origin,
                            const uint64_t* d_get_keys, uint64_t R, uint64_t* d_get_vals, uint8_t* d_get_found,
                            uint64_t* d_prev, uint8_t* d_prev_found) {
    int r = need(c, NRG_DS_HASHMAP);
    if (r) return r;
    if (W > c->cfg.max_batch) return NRG_E_CAPACITY;
    if ((W && !d_puts) || (R && (!d_get_keys || !d_get_vals || !d_get_found))) return NRG_E_INVAL;
    // catch up on anything appended by others first (Replica::combine execs the whole log)
    if ((r = exec_range(c, 0, 0, nullptr, nullptr))) return r;
    if ((r = reserve(c, W))) return r;
    const uint64_t lo = c->tail;
    if (!d_prev || !d_prev_found) d_prev = nullptr, d_prev_found = nullptr;
    HIPCHK(hm_replay_chunk(c, d_puts, lo, W, true, d_get_keys, R, d_get_vals, d_get_found, lo, lo + W, d_prev,
                           d_prev_found));
    if (W) note_origin(c, lo, W, origin);
    c->tail = lo + W;
    c->ltail = c->tail;
    if (c->ctail < c->tail) c->ctail = c->tail;
    return NRG_OK;
}

// replay [ltail, tail) and answer R reads against the final state, fused into the last chunk
static int hm_exec_with_gets(nrg_ctx* c, uint64_t resp_lo, uint64_t resp_hi, uint64_t* d_prev, uint8_t* d_prevf,
                             const uint64_t* d_get_keys, uint64_t R, uint64_t* d_get_vals, uint8_t* d_get_found) {
    if (c->ltail == c->tail) return hip_fail(hm_get_only(c, d_get_keys, R, d_get_vals, d_get_found));
    while (c->ltail < c->tail) {
        uint64_t n = c->tail - c->ltail;
        if (n > c->cfg.max_batch) n = c->cfg.max_batch;
        const uint64_t lo = c->ltail;
        const bool last = lo + n == c->tail;
        HIPCHK(hm_replay_chunk(c, nullptr, lo, n, false, last ? d_get_keys : nullptr, last ? R : 0,
                               last ? d_get_vals : nullptr, last ? d_get_found : nullptr, resp_lo, resp_hi, d_prev,
                               d_prevf));
        c->ltail = lo + n;
    }
    if (c->ctail < c->ltail) c->ctail = c->ltail;
    return NRG_OK;
}

int nrg_hashmap_round_segments_async(nrg_ctx* c, const nrg_put* d_base, uint32_t nseg, uint64_t seg_stride,
                                     const uint64_t* lens, const uint32_t* origins, uint32_t resp_seg,
                                     const uint64_t* d_get_keys, uint64_t R, uint64_t* d_get_vals,
                                     uint8_t* d_get_found, uint64_t* d_prev, uint8_t* d_prev_found) {
    int r = need(c, NRG_DS_HASHMAP);
    if (r) return r;
    if (!lens || nseg == 0 || nseg > 64 || !d_base) return NRG_E_INVAL;
    if (R && (!d_get_keys || !d_get_vals || !d_get_found)) return NRG_E_INVAL;
    if (!d_prev || !d_prev_found) d_prev = nullptr, d_prev_found = nullptr;
    uint64_t total = 0, own_off = 0;
    bool dense = true;
    for (uint32_t s = 0; s < nseg; s++) {
        if (lens[s] > seg_stride) return NRG_E_INVAL;
        if (s == resp_seg) own_off = total;
        if (s + 1 < nseg && lens[s] != seg_stride) dense = false;
        total += lens[s];
    }
    if ((r = exec_range(c, 0, 0, nullptr, nullptr))) return r;
    if ((r = reserve(c, total))) return r;
    const uint64_t lo = c->tail;
    const uint64_t rlo = resp_seg < nseg ? lo + own_off : 0;
    const uint64_t rhi = resp_seg < nseg ? rlo + lens[resp_seg] : 0;
    if (dense && total <= c->cfg.max_batch) {
        // the gathered segments are already the contiguous round W_0 || W_1 || ...: replay them
        // in place while K1 writes the log copy (no separate append pass)
        HIPCHK(hm_replay_chunk(c, d_base, lo, total, true, d_get_keys, R, d_get_vals, d_get_found, rlo, rhi, d_prev,
                               d_prev_found));
        for (uint32_t s = 0, off = 0; s < nseg; off += (uint32_t)lens[s], s++)
            if (lens[s]) note_origin(c, lo + off, lens[s], origins ? origins[s] : s + 1);
        c->tail = lo + total;
        c->ltail = c->tail;
        if (c->ctail < c->tail) c->ctail = c->tail;
        return NRG_OK;
    }
    HIPCHK(copy_segments(c, d_base, nseg, seg_stride, lens, lo));
    for (uint32_t s = 0; s < nseg; s++) {
        if (lens[s]) note_origin(c, c->tail, lens[s], origins ? origins[s] : s + 1);
        c->tail += lens[s];
    }
    return hm_exec_with_gets(c, rlo, rhi, d_prev, d_prev_found, d_get_keys, R, d_get_vals, d_get_found);
}

int nrg_hashmap_prefill(nrg_ctx* c, const uint64_t* keys, const uint64_t* vals, uint64_t n) {
    int r = need(c, NRG_DS_HASHMAP);
    if (r) return r;
    Staging* s = stg(c);
    uint64_t done = 0;
    const uint64_t chunk = c->cfg.max_batch;
    if ((r = staging(c, s[0], (n < chunk ? n : chunk) * sizeof(nrg_put)))) return r;
    while (done < n) {
        const uint64_t m = n - done < chunk ? n - done : chunk;
        nrg_put* h = (nrg_put*)std::malloc(m * sizeof(nrg_put));
        if (!h) return NRG_E_NOMEM;
        for (uint64_t i = 0; i < m; i++) h[i] = nrg_put{keys[done + i], vals[done + i]};
        hipError_t e = hipMemcpyAsync(s[0].p, h, m * sizeof(nrg_put), hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        std::free(h);
        if (e != hipSuccess) return hip_fail(e);
        // direct insert (no log traffic): replay the records through the round pipeline
        // with a private log position, so duplicate keys keep last-writer-wins order.
        HIPCHK(hm_replay_chunk(c, s[0].p, 0, m, false, nullptr, 0, nullptr, nullptr, 0, 0, nullptr, nullptr));
        done += m;
    }
    HIPCHK(sync_all(c));
    return check_err(c);
}

int nrg_hashmap_prefill_range(nrg_ctx* c, uint64_t n, uint64_t off) {
    int r = need(c, NRG_DS_HASHMAP);
    if (r) return r;
    HIPCHK(hm_prefill_range(c, n, off));
    HIPCHK(sync_all(c));
    return check_err(c);
}

// ---- cnr-style key partitioning (partition.hip) ----------------------------
uint32_t nrg_key_owner(uint64_t key, uint32_t parts) { return parts ? nrg::key_owner(key, parts) : 0u; }

int nrg_hashmap_partition_async(nrg_ctx* c, const nrg_put* d_puts, uint64_t W, const uint64_t* d_keys, uint64_t R,
                                uint32_t parts, nrg_put* d_puts_out, uint32_t* d_put_pos, uint64_t* d_keys_out,
                                uint32_t* d_get_pos, uint64_t* d_counts) {
    int r = need(c, NRG_DS_HASHMAP);
    if (r) return r;
    if (parts == 0 || parts > NRG_MAX_PARTS || !d_counts) return NRG_E_INVAL;
    if ((W && (!d_puts || !d_puts_out || !d_put_pos)) || (R && (!d_keys || !d_keys_out || !d_get_pos)))
        return NRG_E_INVAL;
    if (W >= (1ull << 32) || R >= (1ull << 32)) return NRG_E_CAPACITY;
    HIPCHK(pt_partition(c, (const u64*)d_puts, W, 2, parts, (u64*)d_puts_out, d_put_pos, d_counts));
    HIPCHK(pt_partition(c, d_keys, R, 1, parts, d_keys_out, d_get_pos, d_counts + parts));
    return NRG_OK;
}

int nrg_route_back_async(nrg_ctx* c, const uint64_t* d_src, const uint8_t* d_src8, const uint32_t* d_pos, uint64_t n,
                         uint64_t* d_dst, uint8_t* d_dst8) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    if (n && (!d_pos || (d_dst && !d_src) || (d_dst8 && !d_src8))) return NRG_E_INVAL;
    HIPCHK(pt_gather(c, d_src, d_src8, d_pos, n, d_dst, d_dst8));
    return NRG_OK;
}

int nrg_hashmap_prefill_partition(nrg_ctx* c, uint64_t n, uint64_t off, uint32_t part, uint32_t parts) {
    int r = need(c, NRG_DS_HASHMAP);
    if (r) return r;
    if (parts == 0 || parts > NRG_MAX_PARTS || part >= parts) return NRG_E_INVAL;
    HIPCHK(hm_prefill_range(c, n, off, part, parts));
    HIPCHK(sync_all(c));
    return check_err(c);
}

int nrg_hashmap_size(nrg_ctx* c, uint64_t* n) {
    int r = need(c, NRG_DS_HASHMAP);
    if (r) return r;
    HIPCHK(hm_count(c));
    HIPCHK(hipMemcpyAsync(n, &c->d_ctl->nkeys_total, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(sync_all(c));
    return check_err(c);
}

int nrg_hashmap_dump(nrg_ctx* c, uint64_t* keys, uint64_t* vals, uint64_t cap, uint64_t* n) {
    int r = nrg_hashmap_size(c, n);
    if (r) return r;
    if (*n > cap) return NRG_E_CAPACITY;
    if (*n == 0) return NRG_OK;
    Staging* s = stg(c);
    if ((r = staging(c, s[0], *n * 8)) || (r = staging(c, s[1], *n * 8))) return r;
    HIPCHK(hm_dump(c, (u64*)s[0].p, (u64*)s[1].p));
    HIPCHK(hipMemcpyAsync(keys, s[0].p, *n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(vals, s[1].p, *n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(sync_all(c));
    return check_err(c);
}

int nrg_hashmap_digest(nrg_ctx* c, uint64_t out[3]) {
    int r = need(c, NRG_DS_HASHMAP);
    if (r) return r;
    Staging* s = stg(c);
    if ((r = staging(c, s[3], 64))) return r;
    HIPCHK(hm_digest(c, (u64*)s[3].p));
    HIPCHK(hipMemcpyAsync(out, s[3].p, 24, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(sync_all(c));
    return check_err(c);
}

// ---- Stack ---------------------------------------------------------------------------------
int nrg_stack_round_async(nrg_ctx* c, const nrg_stack_op* d_ops, uint64_t n, uint32_t origin, uint32_t* d_pop_vals,
                          uint8_t* d_some_bits) {
    int r = need(c, NRG_DS_STACK);
    if (r) return r;
    if (n > c->cfg.max_batch) return NRG_E_CAPACITY;
    if (n && !d_ops) return NRG_E_INVAL;
    if (!d_pop_vals || !d_some_bits) d_pop_vals = nullptr, d_some_bits = nullptr;
    // catch up on anything appended by others first (Replica::combine execs the whole log)
    if ((r = exec_range(c, 0, 0, nullptr, nullptr))) return r;
    if ((r = reserve(c, n))) return r;
    const uint64_t lo = c->tail;
    // one replay pass that also writes the log copy (Log::append + Log::exec of this batch)
    HIPCHK(st_replay_chunk(c, lo, n, lo, lo + n, d_pop_vals, d_some_bits, d_ops));
    if (n) note_origin(c, lo, n, origin);
    c->tail = lo + n;
    c->ltail = c->tail;
    if (c->ctail < c->tail) c->ctail = c->tail;
    return NRG_OK;
}

int nrg_synth_round_async(nrg_ctx* c, const nrg_synth_op* d_ops, uint64_t n, uint32_t origin, uint64_t* d_resp,
                          uint8_t* d_some) {
    int r = need(c, NRG_DS_SYNTHETIC);
    if (r) return r;
    if (n > c->cfg.max_batch) return NRG_E_CAPACITY;
    if (n && !d_ops) return NRG_E_INVAL;
    if (!d_resp || !d_some) d_resp = nullptr, d_some = nullptr;
    if ((r = exec_range(c, 0, 0, nullptr, nullptr))) return r;
    if ((r = reserve(c, n))) return r;
    const uint64_t lo = c->tail;
    HIPCHK(sy_replay_chunk(c, lo, n, lo, lo + n, d_resp, d_some, d_ops));
    if (n) note_origin(c, lo, n, origin);
    c->tail = lo + n;
    c->ltail = c->tail;
    if (c->ctail < c->tail) c->ctail = c->tail;
    return NRG_OK;
}

int nrg_stack_init(nrg_ctx* c, const uint32_t* vals, uint64_t n) {
    int r = need(c, NRG_DS_STACK);
    if (r) return r;
    if (n > c->cfg.stack_capacity) return NRG_E_CAPACITY;
    HIPCHK(hm_flush_if(c));  // a deferred chunk finish commits before the stack is replaced
    if (n) HIPCHK(hipMemcpyAsync(c->d_stack, vals, n * 4, hipMemcpyHostToDevice, c->stream));
    long long d = (long long)n;
    HIPCHK(hipMemcpyAsync(&c->d_ctl->depth, &d, sizeof(d), hipMemcpyHostToDevice, c->stream));
    // the depth slot the next chunk starts from (stack.hip: chunk of parity p reads slot p ^ 1)
    HIPCHK(hipMemcpyAsync(&c->d_ctl->depth0 + (c->st_par ^ 1), &d, sizeof(d), hipMemcpyHostToDevice, c->stream));
    HIPCHK(sync_all(c));
    return NRG_OK;
}

int nrg_stack_len(nrg_ctx* c, uint64_t* n) {
    int r = need(c, NRG_DS_STACK);
    if (r) return r;
    long long d = 0;
    HIPCHK(hm_flush_if(c));  // a deferred chunk finish publishes the length
    HIPCHK(hipMemcpyAsync(&d, &c->d_ctl->depth, sizeof(d), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(sync_all(c));
    // an overflowing chunk latches ERR_CAPACITY once but keeps counting: never report (or
    // let dump/peek copy) more elements than the allocation holds
    if (d < 0) d = 0;
    if ((uint64_t)d > c->cfg.stack_capacity) d = (long long)c->cfg.stack_capacity;
    *n = (uint64_t)d;
    return check_err(c);
}

int nrg_stack_peek(nrg_ctx* c, uint32_t* val, uint8_t* some) {
    int r = need(c, NRG_DS_STACK);
    if (r) return r;
    if (c->ltail != c->tail) return NRG_E_NOT_SYNCED;
    uint64_t n = 0;
    if ((r = nrg_stack_len(c, &n))) return r;
    *some = n > 0;
    *val = 0;
    if (n) {
        HIPCHK(hipMemcpyAsync(val, c->d_stack + (n - 1), 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(sync_all(c));
    }
    return NRG_OK;
}

int nrg_stack_dump(nrg_ctx* c, uint32_t* vals, uint64_t cap, uint64_t* n) {
    int r = nrg_stack_len(c, n);
    if (r) return r;
    if (*n > cap) return NRG_E_CAPACITY;
    if (*n) {
        HIPCHK(hipMemcpyAsync(vals, c->d_stack, *n * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(sync_all(c));
    }
    return NRG_OK;
}

// ---- Synthetic ---------------------------------------------------------------------------
int nrg_synth_read_async(nrg_ctx* c, const nrg_synth_rd* d_ops, uint64_t n, uint64_t* d_sums) {
    int r = need(c, NRG_DS_SYNTHETIC);
    if (r) return r;
    if (c->ltail != c->tail) return NRG_E_NOT_SYNCED;
    return hip_fail(sy_read(c, d_ops, n, d_sums));
}

int nrg_synth_read(nrg_ctx* c, const nrg_synth_rd* ops, uint64_t n, uint64_t* sums) {
    int r = need(c, NRG_DS_SYNTHETIC);
    if (r) return r;
    if (c->ltail != c->tail) return NRG_E_NOT_SYNCED;
    if (!n) return NRG_OK;
    Staging* s = stg(c);
    if ((r = staging(c, s[0], n * sizeof(nrg_synth_rd))) || (r = staging(c, s[1], n * 8))) return r;
    HIPCHK(hipMemcpyAsync(s[0].p, ops, n * sizeof(nrg_synth_rd), hipMemcpyHostToDevice, c->stream));
    HIPCHK(sy_read(c, (const nrg_synth_rd*)s[0].p, n, (u64*)s[1].p));
    HIPCHK(hipMemcpyAsync(sums, s[1].p, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(sync_all(c));
    return check_err(c);
}

int nrg_synth_dump(nrg_ctx* c, uint64_t* words, uint64_t cap, uint64_t* n) {
    int r = need(c, NRG_DS_SYNTHETIC);
    if (r) return r;
    *n = c->cfg.synth_n;
    if (*n > cap) return NRG_E_CAPACITY;
    HIPCHK(hm_flush_if(c));  // deferred sums fold the hot words
    HIPCHK(hipMemcpyAsync(words, c->d_words, *n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(sync_all(c));
    return check_err(c);
}

// ---- device memory helpers -----------------------------------------------------------------
int nrg_dev_alloc(nrg_ctx* c, uint64_t bytes, void** p) {
    if (!c || !p) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    HIPCHK(hipMalloc(p, bytes ? bytes : 1));
    return NRG_OK;
}
int nrg_dev_free(nrg_ctx* c, void* p) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    HIPCHK(sync_all(c));
    HIPCHK(hipFree(p));
    return NRG_OK;
}
int nrg_memcpy_h2d(nrg_ctx* c, void* d, const void* h, uint64_t bytes) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    HIPCHK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(sync_all(c));
    return NRG_OK;
}
int nrg_memcpy_d2h(nrg_ctx* c, void* h, const void* d, uint64_t bytes) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    HIPCHK(hm_flush_if(c));
    HIPCHK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(sync_all(c));
    return NRG_OK;
}

// ---- generators ------------------------------------------------------------------------------
int nrg_gen_uniform_async(nrg_ctx* c, uint64_t* d, uint64_t n, uint64_t seed, uint64_t span) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    return hip_fail(gen_uniform(c, d, n, seed, span));
}
int nrg_gen_raw_async(nrg_ctx* c, uint64_t* d, uint64_t n, uint64_t seed) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    return hip_fail(gen_raw(c, d, n, seed));
}
int nrg_gen_puts_async(nrg_ctx* c, nrg_put* d, const uint64_t* k, const uint64_t* v, uint64_t n) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    return hip_fail(gen_puts(c, d, k, v, n));
}

int nrg_gen_zipf_async(nrg_ctx* c, uint64_t* d, uint64_t n, uint64_t seed, uint64_t N, double theta,
                       int scramble) {
    if (!c || (n && !d)) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    if (N == 0 || !(theta > 0.0) || theta == 1.0) return NRG_E_INVAL;
    return hip_fail(gen_zipf(c, d, n, seed, N, theta, scramble));
}

int nrg_gen_stack_ops_async(nrg_ctx* c, nrg_stack_op* d, uint64_t n, uint64_t seed) {
    if (!c || (n && !d)) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    return hip_fail(gen_stack_ops(c, d, n, seed));
}

// ---- kernel timing -------------------------------------------------------------------------------
int nrg_kernel_timing(nrg_ctx* c, int enable) {
    if (!c || enable < 0) return NRG_E_INVAL;
    c->timing = enable != 0;
    c->timing_every = enable > 1 ? (uint32_t)enable : 1;
    for (auto& kv : c->timers) kv.second.seen = 0;
    return NRG_OK;
}

int nrg_kernel_timing_only(nrg_ctx* c, const char* which) {
    if (!c) return NRG_E_INVAL;
    c->timing_only = which ? which : "";
    return NRG_OK;
}

int nrg_kernel_time(nrg_ctx* c, const char* which, uint64_t* launches, double* total_ms) {
    if (!c || !which) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    HIPCHK(sync_all(c));
    auto it = c->timers.find(which);
    if (it == c->timers.end()) {
        *launches = 0;
        *total_ms = 0;
        return NRG_OK;
    }
    KTimer& t = it->second;
    for (uint64_t p = 0; p < t.pending; p++) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, t.ev[2 * p], t.ev[2 * p + 1]));
        t.total_ms += ms;
    }
    t.launches += t.pending;
    t.pending = 0;
    *launches = t.launches;
    *total_ms = t.total_ms;
    return NRG_OK;
}

}  // extern "C"

// ---- test hooks (include/nrgpu_testing.h) -----------------------------------------------------
extern "C" int nrg_test_sort_pairs(nrg_ctx* c, const uint32_t* d_keys, const uint32_t* d_vals, uint64_t n,
                                   int key_bits, uint32_t* d_ok, uint32_t* d_ov) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    if (n > c->sort.cap) {  // stack contexts replay without sorting: scratch on demand
        HIPCHK(sync_all(c));
        sort_free(c->sort);
        if (sort_alloc(c->sort, n) != NRG_OK) return NRG_E_NOMEM;
    }
    u32 *sk = nullptr, *sv = nullptr;
    HIPCHK(sort_pairs(c->sort, d_keys, d_vals, n, key_bits, c->stream, &sk, &sv));
    if (n) {
        HIPCHK(hipMemcpyAsync(d_ok, sk, n * 4, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(d_ov, sv, n * 4, hipMemcpyDeviceToDevice, c->stream));
    }
    HIPCHK(sync_all(c));
    return NRG_OK;
}

extern "C" int nrg_test_maxscan(nrg_ctx* c, const uint32_t* d_keys, const uint32_t* d_vals, uint64_t n,
                                uint32_t* d_out) {
    if (!c || !c->d_scan_desc || (n + 2047) / 2048 + 32 > c->scan_desc_words / 2) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    HIPCHK(sy_maxscan(c, d_keys, d_vals, n, d_out));
    // stack contexts keep their look-back descriptors zero between chunks
    if (c->cfg.ds_kind == NRG_DS_STACK)
        HIPCHK(hipMemsetAsync(c->d_scan_desc, 0, c->scan_desc_words * 4, c->stream));
    HIPCHK(sync_all(c));
    return NRG_OK;
}

extern "C" int nrg_test_lds_add_order(nrg_ctx* c, uint32_t keys, uint32_t trials, uint32_t blocks,
                                      uint64_t out[2]) {
    if (!c || !out || keys < 1 || keys > 512 || blocks < 1 || blocks > 65536 || trials > 4096) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    u64* d = nullptr;
    HIPCHK(hipMallocAsync((void**)&d, 16, c->stream));
    HIPCHK(hipMemsetAsync(d, 0, 16, c->stream));
    HIPCHK(sy_lds_add_order(c, keys, trials, blocks, d));
    HIPCHK(hipMemcpyAsync(out, d, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipFreeAsync(d, c->stream));
    HIPCHK(sync_all(c));
    return NRG_OK;
}

extern "C" int nrg_test_ring_read(nrg_ctx* c, uint64_t phys, void* out) {
    if (!c || !out || phys >= c->log_size) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    HIPCHK(sync_all(c));
    HIPCHK(hipMemcpy(out, (const char*)c->d_ring + phys * c->rec_bytes, c->rec_bytes, hipMemcpyDeviceToHost));
    return NRG_OK;
}

extern "C" int nrg_test_hm_skewed(nrg_ctx* c, int* out) {
    if (!c || !out || c->cfg.ds_kind != NRG_DS_HASHMAP) return NRG_E_INVAL;
    *out = c->skewed ? 1 : 0;
    return NRG_OK;
}

extern "C" int nrg_test_debug_read(nrg_ctx* c, uint64_t* out, uint64_t words) {
    if (!c || !out) return NRG_E_INVAL;
    if (!c->d_dbg || words > c->dbg_words) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    // diagnostic timestamps of the launches so far: no flush of deferred work (it would stamp over them)
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(out, c->d_dbg, words * 8, hipMemcpyDeviceToHost));
    return NRG_OK;
}

// Tuning and diagnostic knobs (include/nrgpu_testing.h): the only way to change them.
extern "C" int nrg_test_set_knob(nrg_ctx* c, int knob, uint64_t v) {
    if (!c) return NRG_E_INVAL;
    int r = use_device(c);
    if (r) return r;
    HIPCHK(sync_all(c));  // deferred work of the old setting completes first
    const bool hm = c->cfg.ds_kind == NRG_DS_HASHMAP, sy = c->cfg.ds_kind == NRG_DS_SYNTHETIC;
    switch (knob) {
        case NRG_KNOB_STAMP_MAX:
            if (!hm) return NRG_E_INVAL;
            c->stamp_max = std::min<uint64_t>(v, c->stamp_alloc);
            return NRG_OK;
        case NRG_KNOB_SKEW_EVERY:
            if (!hm || v < 1 || v > (1u << 30)) return NRG_E_INVAL;
            c->dup_every = (uint32_t)v;
            return NRG_OK;
        case NRG_KNOB_EPOCH_LIMIT:
            if (!hm || v < 2 || v > 0xFFFFFFF0ull) return NRG_E_INVAL;
            c->epoch_limit = (uint32_t)v;
            return NRG_OK;
        case NRG_KNOB_K1:
            if (!hm || v > 4) return NRG_E_INVAL;
            c->k1_items = (uint32_t)v;
            return NRG_OK;
        case NRG_KNOB_EXP: {
            if (v > 0xFFFFFFFFull) return NRG_E_INVAL;
            c->exp = (uint32_t)v;
            // timestamp buffer: stack tiles (+ finish workgroups at 128..), synthetic buckets
            // (<= 1024), partition tiles and sum workgroups; 16 words each
            uint64_t words = 0;
            if (c->cfg.ds_kind == NRG_DS_STACK && (c->exp & 2))
                words = std::max<uint64_t>(256, (c->cfg.max_batch + 2047) / 2048) * 16;
            if (sy && (c->exp & 2)) words = 3072 * 16;  // synthetic.hip SY_DBG_ROWS
            if (hm && (c->exp & 2)) words = (uint64_t)HM_BK_MAX * 8;  // partition-round apply buckets
            if (words > c->dbg_words) {
                if (c->d_dbg) HIPCHK(hipFree(c->d_dbg));
                c->d_dbg = nullptr;
                c->dbg_words = 0;
                HIPCHK(hipMalloc(&c->d_dbg, words * sizeof(uint64_t)));
                HIPCHK(hipMemsetAsync(c->d_dbg, 0, words * sizeof(uint64_t), c->stream));
                c->dbg_words = words;
            }
            return NRG_OK;
        }
        case NRG_KNOB_SY_SORT:
            if (!sy || v > 1) return NRG_E_INVAL;
            if (v && c->d_sy_aux) {  // sort path: the bucket scratch goes away
                HIPCHK(hipFree(c->d_sy_aux));
                c->d_sy_aux = nullptr;
            } else if (!v && !c->d_sy_aux && sy_bucket_eligible(c->cfg)) {
                HIPCHK(hipMalloc(&c->d_sy_aux, sy_bucket_aux_bytes(c->cfg)));
                HIPCHK(sy_aux_init(c));
            }
            return NRG_OK;
        case NRG_KNOB_STALL:
            if (v > 3) return NRG_E_INVAL;
            c->stall = (uint32_t)v;
            return NRG_OK;
        case NRG_KNOB_PART:
            if (!hm || v > 2) return NRG_E_INVAL;  // 0: partition rounds only where stamp rounds cannot
            c->part_mode = (uint32_t)v;
            return NRG_OK;
        case NRG_KNOB_PA_TPB:
            if (!hm || (v != 0 && v != 256 && v != 512 && v != 1024)) return NRG_E_INVAL;
            c->pa_tpb = (uint32_t)v;
            return NRG_OK;
        case NRG_KNOB_SMALL_MAX:
            if (!hm || v > 2048) return NRG_E_INVAL;
            c->small_max = v;
            return NRG_OK;
        case NRG_KNOB_COMB_SPIN:
            if (v > 4096) return NRG_E_INVAL;
            c->comb_spin = (int32_t)v;
            return NRG_OK;
        case NRG_KNOB_COMB_GATHER:
            if (v > 1000) return NRG_E_INVAL;
            c->comb_gather = (int32_t)v;
            return NRG_OK;
        case NRG_KNOB_COMB_SERVE:
            if (v > (1u << 20)) return NRG_E_INVAL;
            c->comb_serve = (int32_t)v;
            return NRG_OK;
        case NRG_KNOB_COMB_DEPTH:
            if (v < 1 || v > 4) return NRG_E_INVAL;
            c->comb_depth = (uint32_t)v;
            return NRG_OK;
        case NRG_KNOB_SY_FUSED:
            if (!sy || v > 1) return NRG_E_INVAL;
            c->sy_fused = v != 0;
            return NRG_OK;
        case NRG_KNOB_PIPELINE:
            if (v > 1) return NRG_E_INVAL;
            c->pipeline = v != 0;
            return NRG_OK;
        default: return NRG_E_INVAL;
    }
}
