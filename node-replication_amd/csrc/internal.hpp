// internal.hpp — host-side structures shared by the runtime and the kernel launchers.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

#include "../../include/nrgpu.h"
#include "common.hpp"

namespace nrg {

// Scratch for the stable LSD radix sort of (u32 key, u32 value) pairs (radix_sort.hip).
struct SortScratch {
    u64 cap = 0;           // max elements
    u32* k[2] = {nullptr, nullptr};
    u32* v[2] = {nullptr, nullptr};
    u32* ctlmem = nullptr;  // [hist: 4*256][tickets: 64][desc: 4 * max_tiles * 256]
    u64 max_tiles = 0;
    u64 ctl_words = 0;
};

int sort_alloc(SortScratch& s, u64 cap);
void sort_free(SortScratch& s);
// Sort n pairs by the low `key_bits` bits of key (stable). vals_in == nullptr means
// values are 0..n-1. Result pointers are returned (inside the scratch).
hipError_t sort_pairs(SortScratch& s, const u32* keys_in, const u32* vals_in, u64 n, int key_bits,
                      hipStream_t st, u32** out_k, u32** out_v);
// The same in two steps, for a caller that builds the digit histograms itself (fused into the
// pass that produces the keys): sort_prepare clears the control words and returns the
// [4][256] histogram array to add into; sort_run runs the digit passes.
hipError_t sort_prepare(SortScratch& s, u64 n, int key_bits, hipStream_t st, u32** hist);
hipError_t sort_run(SortScratch& s, const u32* keys_in, const u32* vals_in, u64 n, int key_bits, hipStream_t st,
                    u32** out_k, u32** out_v);

struct KTimer {
    std::vector<hipEvent_t> ev;  // pairs
    u64 pending = 0;             // recorded pairs not yet harvested
    u64 launches = 0;
    double total_ms = 0.0;
    u64 seen = 0;                // launches of this kernel since timing was enabled
    bool open = false;           // timer_begin recorded a start event not yet closed
};

struct Staging {  // growable device scratch for the host-pointer entry points
    void* p = nullptr;
    uint64_t bytes = 0;
};

// The second half of the last replayed hashmap round, run in the next launch (beside the next
// round's index pass) or by a flush: its reads and, for a stamp round, its apply.
struct HmDeferred {
    bool valid = false;
    u32 epoch = 0;
    bool apply = false;            // stamp round: the elected writers still store their values
    const nrg_put* src = nullptr;  // records: src[i] if set, else ring[(lo + i) & mask]
    u64 lo = 0, n = 0;
    const u64* keys = nullptr;     // the round's reads (R may be 0)
    u64 R = 0;
    u64* vals = nullptr;
    uint8_t* found = nullptr;
};

// A stack chunk whose finish (cross-tile Pops, commit) has not run yet (stack.hip).
struct StDeferred {
    bool valid = false;
    u64 lo = 0, n = 0;
    u32 tiles = 0, par = 0;
    u64 rlo = 0, rhi = 0;
    uint32_t* resp = nullptr;
    uint8_t* some = nullptr;
};

// A synthetic chunk whose bucket pass or per-op sums and hot-word fold have not run yet
// (synthetic.hip); its scratch slots follow from its epoch.
struct SyDeferred {
    bool valid = false;
    u32 epoch = 0;
    u64 lo = 0, n = 0;
    u32 ntiles = 0, want = 0, t0 = 0, t1 = 1;
    u64 rlo = 0, rhi = 0;
    u64* resp = nullptr;
    uint8_t* some = nullptr;
};

struct HostRun {  // origin tags of appended log ranges (the Entry::replica field)
    u64 first, count;
    u32 origin;
};

}  // namespace nrg

struct nrg_ctx {
    int device = 0;
    nrg_config cfg{};
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;

    // ---- Log (per-replica HBM ring) ----
    uint64_t log_size = 0;  // entries (power of two), as Log::new computes it
    uint64_t head = 0, tail = 0, ctail = 0, ltail = 0;
    uint32_t rec_bytes = 0;
    void* d_ring = nullptr;
    std::vector<nrg::HostRun> origins;

    nrg::DevCtl* d_ctl = nullptr;

    // ---- NrHashMap ----
    uint32_t slot_shift = 0;  // 64 - log2_slots
    uint64_t slots = 0;
    nrg::Slot* d_table = nullptr;
    uint64_t rounds = 0;             // replay rounds launched (statistics)
    // tuning and diagnostic knobs: set only through nrg_test_set_knob (include/nrgpu_testing.h)
    uint32_t k1_items = 0;           // Puts per index thread (0: by round size; NRG_KNOB_K1)
    uint32_t exp = 0;                // diagnostic bits (NRG_KNOB_EXP; see hashmap.hip StampJob)
    // Reads of the last replayed round: answered in the next launch beside the next round's
    // index pass, or by nrg_join / nrg_sync / any call that reads the table. With
    // pipeline == false they are flushed at the end of every call.
    bool pipeline = false;
    nrg::HmDeferred pend;
    nrg::StDeferred st_pend;  // stack: the last chunk's finish, if deferred
    uint32_t st_par = 0;      // stack: buffer parity of the next chunk
    nrg::SyDeferred sy_pend;    // synthetic: the chunk whose sums are deferred, if any
    nrg::SyDeferred sy_pend_b;  // synthetic, one launch per round: the chunk whose bucket pass is deferred
    bool sy_fused = true;       // synthetic: one launch per round, chunks three deep (NRG_KNOB_SY_FUSED)
    uint32_t sy_round = 0;      // synthetic: chunks replayed (the chunk epoch: scratch slots, 32-bit seen values)
    int32_t comb_spin = -1;   // combiner knobs (NRG_KNOB_COMB_SPIN / _DEPTH): -1 / 0 = defaults
    uint64_t small_max = 0;   // hashmap: rounds of <= small_max Puts take the one-launch small round
    uint32_t comb_depth = 0;
    int32_t comb_gather = -1;  // NRG_KNOB_COMB_GATHER (us; -1 = default)
    int32_t comb_serve = -1;   // NRG_KNOB_COMB_SERVE (-1 = default: on)
    uint32_t stall = 0;       // NRG_KNOB_STALL (tests): 1 odd waves sleep at LDS reuse points, 2 (synthetic,
                              // diagnostic: wrong results) without the bucket pass's tile-map barrier
    uint64_t* d_created = nullptr;  // [HM_CREATED_SLOTS] keys created by replay rounds
    void* d_bk_ent = nullptr;       // partition rounds: [tiles][tile] 16-B {key, value} entries
    uint32_t* d_bk_idx = nullptr;   // partition rounds with previous values: [tiles][tile] round offset
    uint32_t* d_bk_cnt = nullptr;   // [index tiles][bucket] offset << 16 | count
    // Stamp rounds (<= stamp_max Puts, no previous values): per-Put slot ids by epoch parity.
    uint64_t stamp_max = 0;
    // Partition rounds (hashmap.hip part_role + hm_papply_kernel), NRG_KNOB_PART: 1 (default) for
    // previous values, skewed streams and rounds of >= 393216 Puts; 2 for every round; 0 only
    // where a stamp round cannot (previous values, skew).
    uint32_t part_mode = 1;
    uint32_t pa_tpb = 0;      // NRG_KNOB_PA_TPB: partition-round apply workgroup width (0 = by round)
    uint64_t stamp_alloc = 0;  // Puts the put_slot arrays hold (stamp_max <= stamp_alloc)
    uint32_t epoch = 1;  // epoch of the last replay round (1: prefill / before any round)
    uint32_t epoch_limit = 0xFFFFFFF0u;  // renormalise stamps here (NRG_KNOB_EPOCH_LIMIT for tests)
    uint32_t* d_put_slot[2] = {nullptr, nullptr};
    // Key skew (hm_dup_sample_kernel): Puts combined inside their index block, sampled every
    // dup_every rounds into mapped host memory; a skewed stream takes partition rounds.
    uint64_t* d_dup = nullptr;            // [HM_DUP_SLOTS]
    void* d_pt = nullptr;                 // partition.hip tile counts / offsets
    uint64_t pt_words = 0;
    volatile uint64_t* h_dup = nullptr;   // {seq, dups}, mapped pinned host memory
    uint64_t* h_dup_dev = nullptr;        // its device address
    uint64_t dup_seq = 0, dup_puts = 0, dup_puts_sampled = 0;
    uint64_t sample_seq = 0;  // a sample the next hm_round launch takes (0: none pending)
    uint32_t* err_out = nullptr;  // the next hm_round launch copies (and clears) the error latch here
    uint32_t dup_rounds = 0, dup_every = 16;
    bool skewed = false;
    // Zipf generator cache: zeta(zipf_n, zipf_theta)
    uint64_t zipf_n = 0;
    double zipf_theta = 0.0, zipf_zetan = 0.0;
    // ---- Stack ----
    uint32_t* d_stack = nullptr;
    void* d_st_aux = nullptr;  // per-tile minima, last-Push tables and cross-tile Pops (stack.hip)

    // ---- Synthetic ----
    uint64_t* d_words = nullptr;
    uint64_t* d_sort_aux = nullptr;  // per-touch max-scan output
    uint32_t synth_key_bits = 0;
    void* d_sy_aux = nullptr;  // bucket replay scratch (synthetic.hip); nullptr: sort path

    // ---- shared scratch ----
    nrg::SortScratch sort;
    uint64_t* d_tmp_u64 = nullptr;  // general scratch (max_batch words)
    uint64_t tmp_words = 0;
    uint32_t* d_scan_desc = nullptr;  // decoupled look-back descriptors for scans
    uint64_t scan_desc_words = 0;

    nrg::Staging stg[4];
    uint64_t* d_dbg = nullptr;  // diagnostic phase timestamps (NRG_KNOB_EXP), [tiles][16]
    uint64_t dbg_words = 0;     // u64 words d_dbg holds

    // ---- timing ----
    bool timing = false;
    uint32_t timing_every = 1;  // event-stamp every n-th launch (nrg_kernel_timing(ctx, n))
    std::string timing_only;  // if non-empty, only this kernel is timed
    std::map<std::string, nrg::KTimer> timers;
};

namespace nrg {
// timing helpers (runtime.cpp)
void timer_begin(nrg_ctx* c, const char* name, hipStream_t s = nullptr);
void timer_end(nrg_ctx* c, const char* name, hipStream_t s = nullptr);
// Event pair for one launch of kernel `name` when it is being timed (false otherwise). The
// pair is passed to hipExtLaunchKernelGGL, which stamps it from the kernel's own dispatch:
// no marker packets between kernels, so timing does not perturb the timed stream.
bool timer_events(nrg_ctx* c, const char* name, hipEvent_t* start, hipEvent_t* stop);

#define NRG_LAUNCH(CTX, NAME, KERNEL, GRID, BLOCK, SHMEM, STREAM, ...)                                  \
    do {                                                                                                \
        hipEvent_t nrg_e0_, nrg_e1_;                                                                    \
        if (timer_events((CTX), (NAME), &nrg_e0_, &nrg_e1_))                                            \
            hipExtLaunchKernelGGL((KERNEL), dim3(GRID), dim3(BLOCK), (SHMEM), (STREAM), nrg_e0_, nrg_e1_, 0, \
                                  __VA_ARGS__);                                                         \
        else                                                                                            \
            KERNEL<<<(GRID), (BLOCK), (SHMEM), (STREAM)>>>(__VA_ARGS__);                                \
    } while (0)
// make the context's device current for this thread (runtime.cpp; cached per thread)
int ctx_use_device(nrg_ctx* c);
// launch the deferred reads of the last hashmap round, if any (hashmap.hip)
hipError_t hm_flush(nrg_ctx* c);
hipError_t st_flush(nrg_ctx* c);
hipError_t sy_flush(nrg_ctx* c);

// hashmap.hip
hipError_t hm_replay_chunk(nrg_ctx* c, const void* src_recs, u64 lo, u64 n, bool write_ring,
                           const u64* d_get_keys, u64 R, u64* d_get_vals, uint8_t* d_get_found,
                           u64 resp_lo, u64 resp_hi, u64* d_prev, uint8_t* d_prev_found);
hipError_t hm_get_only(nrg_ctx* c, const u64* d_keys, u64 n, u64* d_vals, uint8_t* d_found);
hipError_t hm_init(nrg_ctx* c);
hipError_t hm_alloc(nrg_ctx* c, u64 max_batch);  // per-round scratch (entries, counts, overlays)
void hm_free(nrg_ctx* c);
hipError_t hm_prefill_range(nrg_ctx* c, u64 n, u64 off, u32 part = 0, u32 parts = 1);
// partition.hip: stable partition of records (key in word 0) by key owner; answers routed back
hipError_t pt_partition(nrg_ctx* c, const u64* in, u64 n, u32 words, u32 parts, u64* out, u32* pos, u64* total);
hipError_t pt_gather(nrg_ctx* c, const u64* src, const uint8_t* src8, const u32* pos, u64 n, u64* dst, uint8_t* dst8);
// the flat combiner's round server (hashmap.hip hm_serve_kernel), in mapped host memory
// The host's words and the device's sit on separate 128-B lines: the GPU's L2 keeps host memory
// lines it has written, and a poll of a word on a line the server itself dirtied read that stale
// line (its buffer_inv keeps dirty lines), so the server never saw the next round.
constexpr uint32_t SERVE_SLOTS = 8;
struct ServeCtl {
    alignas(128) uint64_t door[SERVE_SLOTS];  // (host) slot k % NB: (k + 1) << 32 | Puts << 16 | Gets
    uint32_t stop;                            // (host) exit once every rung round is served
    alignas(128) uint64_t served;             // rounds served (device)
    uint64_t exited;                          // session of the last server that exited (device)
    uint64_t trace[4];                        // (diagnostic) -, round, doorbell seen, polls
};
// Gets per served round (4 per thread of the 1024: the resident loop's registers; the combiner
// launches rounds with more)
constexpr uint32_t SERVE_R = 4096;
struct SmallJobBlob {  // one small round's job (hashmap.hip SmallJob)
    alignas(16) unsigned char b[192];
};
bool hm_small_fill(nrg_ctx* c, const nrg_put* recs, u64 lo, u64 W, const u64* keys, u64 R, u64* vals, uint8_t* found,
                   u64* prev, uint8_t* prevf, u32* e_out, SmallJobBlob* blob);
// runtime.cpp: a round as nrg_hashmap_round_async would run it as a small round, its log bookkeeping
// done and nothing launched (the server runs it); *lo = its first log position. NRG_E_INVAL: not a
// small round of a caught-up replica. blob (optional): the round's whole job.
int hm_small_job(nrg_ctx* c, const nrg_put* recs, u64 W, u32 origin, const u64* keys, u64 R, u64* vals,
                 uint8_t* found, u64* prev, uint8_t* prevf, u32* e_out, SmallJobBlob* blob, u64* lo);
hipError_t hm_serve_launch(nrg_ctx* c, ServeCtl* sc, const SmallJobBlob* hdr, u32 nslots, u64 first, u64 first_lo,
                           u64 session, u64 idle_ticks);
// the replica group's partitioned rounds (partition.hip): one fused launch for the Puts and Get
// keys into owner regions of capacity cap_p / cap_k; counts[0, parts) Puts and [parts, 2 parts)
// Gets per owner, then the nxw host words xw; desc: pt_desc_words() look-back descriptors
constexpr u32 PT_XW_MAX = 8;
hipError_t pt_fused(hipStream_t s, const u64* puts, u64 W, u64 cap_p, u64* pout, u32* ppos, const u64* keys, u64 R,
                    u64 cap_k, u64* kout, u32* gpos, u64* desc, u32 parts, u32 epoch, u64* counts, const u64* xw,
                    u32 nxw);
u64 pt_desc_words(u64 W, u64 R, u32 parts);
hipError_t pt_route2(hipStream_t s, const u64* src_a, const uint8_t* src8_a, const u32* pos_a, u64 n_a, u64* dst_a,
                     uint8_t* dst8_a, const u64* src_b, const uint8_t* src8_b, const u32* pos_b, u64 n_b, u64* dst_b,
                     uint8_t* dst8_b);
hipError_t hm_dump(nrg_ctx* c, u64* d_keys, u64* d_vals);
hipError_t hm_count(nrg_ctx* c);  // DevCtl::nkeys_total = number of keys
hipError_t hm_digest(nrg_ctx* c, u64* d_out3);
hipError_t gen_uniform(nrg_ctx* c, u64* d, u64 n, u64 seed, u64 span);
hipError_t gen_raw(nrg_ctx* c, u64* d, u64 n, u64 seed);
hipError_t gen_puts(nrg_ctx* c, nrg_put* d, const u64* k, const u64* v, u64 n);
// workload.hip (also holds the three generators above)
hipError_t gen_stack_ops(nrg_ctx* c, nrg_stack_op* d, u64 n, u64 seed);
hipError_t gen_zipf(nrg_ctx* c, u64* d, u64 n, u64 seed, u64 N, double theta, int scramble);
hipError_t copy_segments(nrg_ctx* c, const void* d_base, u32 nseg, u64 seg_stride, const u64* lens,
                         u64 dst_lo);

// stack.hip
hipError_t st_replay_chunk(nrg_ctx* c, u64 lo, u64 n, u64 resp_lo, u64 resp_hi, uint32_t* d_resp,
                           uint8_t* d_some, const nrg_stack_op* src = nullptr);
u64 st_aux_bytes(u64 max_batch);   // size of nrg_ctx::d_st_aux
u64 st_desc_words(u64 max_batch);  // u32 words of look-back descriptors the stack needs

// synthetic.hip
hipError_t sy_init(nrg_ctx* c);
hipError_t sy_replay_chunk(nrg_ctx* c, u64 lo, u64 n, u64 resp_lo, u64 resp_hi, u64* d_resp,
                           uint8_t* d_some, const nrg_synth_op* src = nullptr);
hipError_t sy_read(nrg_ctx* c, const nrg_synth_rd* d_ops, u64 n, u64* d_sums);
bool sy_bucket_eligible(const nrg_config& cf);  // configs the sort-free bucket replay handles
u64 sy_bucket_aux_bytes(const nrg_config& cf);  // size of nrg_ctx::d_sy_aux
hipError_t sy_aux_init(nrg_ctx* c);              // after (re)allocating d_sy_aux
hipError_t sy_maxscan(nrg_ctx* c, const u32* sk, const u32* sv, u64 n, u32* M);
hipError_t sy_lds_add_order(nrg_ctx* c, u32 K, u32 trials, u32 blocks, u64* d_out);
}  // namespace nrg
