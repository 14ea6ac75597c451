// synthetic.hip — AbstractDataStructure replica replay on gfx950 (benches/synthetic.rs:60-195).
//
// Every write op touches hot_writes hot words (index (r2+j) % hot_reads, skipped when
// r2 + hot_writes wraps) and cold_writes cold words (index (r1*tid + k*r2) % (n-hot_reads) +
// hot_reads, wrapping u64 arithmetic as in the release build). WriteOnly sets each touched
// word to tid; ReadWrite adds 1 to each and sums the cold words' values as read (before
// its own increment). Replay:
//   sy_expand   one thread per op: emits (word, order|SET) touch pairs, order = op*T + t
//   radix sort  stable by word → every word's touches in log order
//   sy_maxscan  inclusive max-scan of "segment head or SET" positions (decoupled
//               look-back): the value a touch sees = last SET's tid (or the pre-batch word)
//               + the number of increments since
//   sy_resolve  ReadWrite cold touches add their value to the op's sum (integer atomics:
//               wrapping u64 adds commute, so the sum is exact whatever the order)
//   sy_commit   each word's last touch writes its final value
#include "internal.hpp"

namespace nrg {

constexpr u32 SETBIT = 0x80000000u;

// Streaming (nt) stores for the streamed outputs (log copy, touch records, seen values,
// responses), an A/B variant (NRG_KNOB_EXP bits 6 / 7 / 8 / 9 for the log copy / touch records /
// seen values / responses): they drain during the kernel instead of in the
// kernel-end L2 write-back, which pays on the stack and the hashmap's partition rounds, but not
// here (56.6-56.9 vs 56.1-56.6 us per round plain; profiles/r04_nt_stores.txt): plain by default.
typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
// Round 6: the compiler merges st_out's two branches into one plain store and drops the hint, so
// bits 7-9 compile to plain stores; only the 16-B log copy (st_op, bit 6) is streamed. Streamed
// for real (the plain branch as a relaxed atomic store, not merged) every variant was slower on
// one box, and the atomic form cost the plain default its merged wider stores: 44.9-45.8 us per
// round before, 47.7-48.0 with the atomic plain form, 49.5-50.5 touch records or seen values
// streamed, 47.5-47.6 responses streamed (profiles/r06/nt_single_stores.txt).
template <typename T>
__device__ __forceinline__ void st_out(T* p, T v, bool plain) {
    if (plain) *p = v;
    else __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ void st_op(nrg_synth_op* p, const nrg_synth_op& o, bool plain) {
    if (plain) {
        *p = o;
        return;
    }
    const u64x2_t a = {o.tid, o.r1}, b = {o.r2, o.op};
    __builtin_nontemporal_store(a, (u64x2_t*)p);
    __builtin_nontemporal_store(b, (u64x2_t*)p + 1);
}
// Round 6: the sums' responses are streamed (compile-time, since st_out's hint is dropped): same box,
// three pairs, 45.40-45.66 -> 44.35-44.61 us per 1M-op round (profiles/r06/synth_resp_nt.txt).
// NRG_SY_RESP_NT=0 restores st_out (plain unless the A/B bit 9 asks, which compiles plain too).
#ifndef NRG_SY_RESP_NT
#define NRG_SY_RESP_NT 1
#endif
constexpr int MS_TPB = 256;
constexpr int MS_ITEMS = 8;
constexpr int MS_TILE = MS_TPB * MS_ITEMS;

__global__ void sy_init_kernel(u64* words, u64 n) {
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (u64)gridDim.x * 256ull) words[i] = i;
}

__global__ __launch_bounds__(256) void sy_expand_kernel(const nrg_synth_op* __restrict__ ring, u64 ring_mask, u64 lo,
                                                        u64 n, u64 N, u32 HR, u32 HW, u32 CW, u32 sentinel,
                                                        u32* __restrict__ sk, u32* __restrict__ sv) {
    const u32 T = HW + CW;
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (u64)gridDim.x * 256ull) {
        const nrg_synth_op o = ring[(lo + i) & ring_mask];
        const u32 set = o.op == NRG_SYNTH_WRITE_ONLY ? SETBIT : 0u;
        const u64 r2 = o.r2;
        const u64 end = r2 + HW;
        const bool hot_ok = end >= r2;  // `begin..end` is empty when the add wraps
        u64 pos = i * T;
        for (u32 j = 0; j < HW; j++, pos++) {
            sk[pos] = hot_ok ? (u32)((r2 + j) % HR) : sentinel;
            sv[pos] = (u32)pos | set;
        }
        u64 begin = o.r1 * o.tid;
        const u64 span = N - HR;
        for (u32 k = 0; k < CW; k++, pos++) {
            sk[pos] = (u32)(begin % span + HR);
            begin += r2;
            sv[pos] = (u32)pos | set;
        }
    }
}

constexpr u64 M_AGG = 1ull << 62;
constexpr u64 M_INC = 2ull << 62;
constexpr u64 M_MASK = 3ull << 62;

// M[p] = max{ q <= p : q heads its word's group, or touch q is a SET }
__global__ __launch_bounds__(MS_TPB) void sy_maxscan_kernel(const u32* __restrict__ sk, const u32* __restrict__ sv,
                                                            u64 n, u64* desc, u32* ticket, u32* __restrict__ M) {
    __shared__ u32 s_w[4];
    __shared__ u32 s_tile, s_base;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (t == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const u32 tile = s_tile;
    const u64 base = (u64)tile * MS_TILE + (u64)t * MS_ITEMS;
    // Branch-free marker computation: loads first, then selects. (A short-circuit
    // `p == 0 || sk[p-1] != sk[p]` form here was miscompiled by ROCm 7.2 clang for gfx950:
    // the first unrolled item's select body came out empty and its marker was lost.)
    u32 mk[MS_ITEMS];
    u32 run = 0;
    u32 kprev = (base > 0 && base - 1 < n) ? sk[base - 1] : 0u;
#pragma unroll
    for (int q = 0; q < MS_ITEMS; q++) {
        const u64 p = base + q;
        const bool in = p < n;
        const u32 k = in ? sk[p] : 0u;
        const u32 v = in ? sv[p] : 0u;
        const bool mark = in & ((p == 0) | (k != kprev) | ((v & SETBIT) != 0u));
        const u32 m = mark ? (u32)p : 0u;
        run = run > m ? run : m;
        mk[q] = run;
        kprev = k;
    }
    u32 inc = run;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u32 o = __shfl_up(inc, off, 64);
        if (lane >= off) inc = inc > o ? inc : o;
    }
    if (lane == 63) s_w[w] = inc;
    u32 ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = 0;
    __syncthreads();
    u32 wpre = 0, tagg = 0;
    for (int i = 0; i < 4; i++) {
        if (i < w) wpre = wpre > s_w[i] ? wpre : s_w[i];
        tagg = tagg > s_w[i] ? tagg : s_w[i];
    }
    if (w == 0) {
        // wave 0: lane l reads tile (tt - l)'s descriptor (64 predecessors per round trip)
        u32 pre = 0;
        if (tile == 0) {
            if (lane == 0) __hip_atomic_store(&desc[0], M_INC | tagg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(&desc[tile], M_AGG | tagg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int tt = (int)tile - 1;
            for (;;) {
                const int idx = tt - lane;
                const u64 v = idx >= 0 ? __hip_atomic_load(&desc[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                const u64 st = v & M_MASK;
                const u64 nr = __ballot(st == 0);
                const u64 ic = __ballot(st == M_INC);
                const int first_nr = nr ? __ffsll((unsigned long long)nr) - 1 : 64;
                const int first_ic = ic ? __ffsll((unsigned long long)ic) - 1 : 64;
                const bool found = first_ic < first_nr;
                const int use = found ? first_ic + 1 : first_nr;
                u32 x = lane < use ? (u32)v : 0u;
                for (int off = 32; off > 0; off >>= 1) {
                    const u32 y = __shfl_xor(x, off, 64);
                    x = x > y ? x : y;
                }
                pre = pre > x ? pre : x;
                if (found) break;
                tt -= use;
                if (use < 64) __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0) {
                const u32 ti = pre > tagg ? pre : tagg;
                __hip_atomic_store(&desc[tile], M_INC | ti, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (lane == 0) s_base = pre;
    }
    __syncthreads();
    u32 pre = s_base > wpre ? s_base : wpre;
    pre = pre > ex ? pre : ex;
#pragma unroll
    for (int q = 0; q < MS_ITEMS; q++) {
        const u64 p = base + q;
        if (p < n) M[p] = pre > mk[q] ? pre : mk[q];
    }
}

__device__ __forceinline__ u64 touch_tid(const nrg_synth_op* ring, u64 ring_mask, u64 lo, u32 v, u32 T) {
    return ring[(lo + (v & ~SETBIT) / T) & ring_mask].tid;
}

__global__ __launch_bounds__(256) void sy_resolve_kernel(const u32* __restrict__ sk, const u32* __restrict__ sv,
                                                         const u32* __restrict__ M, u64 n,
                                                         const nrg_synth_op* __restrict__ ring, u64 ring_mask, u64 lo,
                                                         const u64* __restrict__ words, u32 HW, u32 T, u32 sentinel,
                                                         u64 resp_lo, u64 resp_hi, u64* resp) {
    const u64 p = blockIdx.x * 256ull + threadIdx.x;
    if (p >= n) return;
    const u32 x = sk[p];
    const u32 v = sv[p];
    if (x == sentinel || (v & SETBIT)) return;
    const u32 order = v & ~SETBIT;
    if (order % T < HW) return;  // hot increments are not read
    const u64 g = lo + order / T;
    if (g < resp_lo || g >= resp_hi) return;
    const u32 m = M[p];
    const u32 mv = sv[m];
    u64 val;
    if (mv & SETBIT)
        val = touch_tid(ring, ring_mask, lo, mv, T) + (u64)(p - m - 1);
    else
        val = words[x] + (u64)(p - m);
    atomicAdd(&resp[g - resp_lo], val);
}

__global__ __launch_bounds__(256) void sy_commit_kernel(const u32* __restrict__ sk, const u32* __restrict__ sv,
                                                        const u32* __restrict__ M, u64 n,
                                                        const nrg_synth_op* __restrict__ ring, u64 ring_mask, u64 lo,
                                                        u64* __restrict__ words, u32 T, u32 sentinel) {
    const u64 p = blockIdx.x * 256ull + threadIdx.x;
    if (p >= n) return;
    const u32 x = sk[p];
    if (x == sentinel) return;
    if (p + 1 < n && sk[p + 1] == x) return;
    const u32 m = M[p];
    const u32 mv = sv[m];
    if (mv & SETBIT)
        words[x] = touch_tid(ring, ring_mask, lo, mv, T) + (u64)(p - m);
    else
        words[x] = words[x] + (u64)(p - m + 1);
}

__global__ __launch_bounds__(256) void sy_read_kernel(const nrg_synth_rd* __restrict__ ops, u64 n,
                                                      const u64* __restrict__ words, u64 N, u32 HR, u32 HW, u32 CR,
                                                      u64* __restrict__ sums) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    const nrg_synth_rd o = ops[i];
    u64 sum = 0;
    const u64 end = o.r2 + HW;
    if (end >= o.r2)
        for (u32 j = 0; j < HW; j++) sum += words[(o.r2 + j) % HR];
    u64 begin = o.r1 * o.tid;
    const u64 span = N - HR;
    for (u32 k = 0; k < CR; k++) {
        sum += words[begin % span + HR];
        begin += o.r2;
    }
    sums[i] = sum;
}

// ---- bucket replay: no global sort ------------------------------------------------------
// The default path for the reference's configurations (1 <= cold_writes <= 8, hot_reads <= 16,
// <= 1024 buckets of 512 cold words, rounds <= 8M ops). Hot and cold words are disjoint, so:
//   hot   words: each 2048-op tile folds its hot touches into a summary per hot word
//               {has SET, tid of the last SET, touches after it}; the summaries compose
//               associatively in log order (sy_sum_kernel's block 0 folds them).
//   cold  words: sy_part_kernel writes each tile's cold touches grouped by bucket
//               (word >> 9), in log order within a bucket (wave ballot ranking), plus a
//               [bucket][tile] count table; sy_bucket_kernel (one workgroup per bucket)
//               gathers the bucket's touches tile by tile — log order — and replays them
//               against the bucket's 512 words held in LDS, 1024 touches at a time (a
//               per-wave, per-word count table orders same-word touches across waves);
//               every touch's seen value goes back to its slot in the tile layout;
//               sy_sum_kernel adds them per op with LDS atomics (coalesced responses).
// Replaces expand + 3 radix passes + max-scan + scattered u64 atomics (620 us per 1M ops).
constexpr u32 SYB_SHIFT = 9;
constexpr u32 SYB_WORDS = 1u << SYB_SHIFT;  // LDS words per bucket (a bucket holds W <= 512 of them)
constexpr int SYA_TPB = 512, SYA_WAVES = SYA_TPB / 64, SYA_OROUNDS = 4;
constexpr u32 SYA_OPS = SYA_WAVES * SYA_OROUNDS * 64;  // ops per tile (11 bits)
constexpr u32 SY_MAX_NB = 512, SY_MAX_HOT = 16, SY_MAX_TILES = 4096, SY_MAX_CW = 8;
// Cold word 0 (bucket 0) is replayed by SY_B0_PARTS workgroups when the chunk holds no WriteOnly:
// its seen values are then its value plus the touch's rank, so each part takes a contiguous
// range of the touches. The bucket pass launches SY_MAX_NB workgroups in all (two per CU), so
// words 1.. go to SY_MAX_NB - SY_B0_PARTS buckets.
#ifndef NRG_SY_B0_PARTS
#define NRG_SY_B0_PARTS 4
#endif
constexpr u32 SY_B0_PARTS = NRG_SY_B0_PARTS;
#ifndef NRG_SYB_PER
#define NRG_SYB_PER 10  // 1M-op rounds: 8 -> 57.2 us, 10 -> 56.4 (two passes per bucket, not three; E positions
                        // recomputed, not kept per touch); 12 spills (profiles/r03_synth_pass_size.txt)
#endif
// Rankings: the partition and the bucket pass's SET-free passes rank a wave's touches with one
// returning LDS add per touch on a wave-private count. A returning LDS add hands the lanes of one
// instruction that hit the same count their old values in lane order (checked on the hardware:
// microbench/lds_add_order.hip, 2.1 G lanes; nrg_test_lds_add_order in the GPU suite), so the
// ranks follow log order. Round 4's peer masks (OR, read back, leader update: three LDS round
// trips per touch) ran 55.5 us per 1M-op round against 51.8 (profiles/r05_synth_lds_add.txt).
#ifndef NRG_SYP_PD
#define NRG_SYP_PD 1  // partition: wave rounds of op records in flight ahead of the one ranked
#endif
constexpr int SYP_PD = NRG_SYP_PD;
constexpr int SYB_TPB = 512, SYB_WAVES = SYB_TPB / 64, SYB_PER = NRG_SYB_PER;
constexpr int SYC_TPB = 512;
#ifndef NRG_SYS_T
// tiles per sum workgroup (A/B builds). With 1 the 489 sum workgroups of a 1M-op chunk queue
// behind the partition tiles for the launch's LDS slots (3 per CU) and end ~4 us after them;
// 2 puts every workgroup of the launch on the chip at once but doubles each sum workgroup's
// span: 58.3-58.6 vs 56.6-57.2 us per round (profiles/r03_synth_sum_tiles.txt)
#define NRG_SYS_T 1
#endif
#ifndef NRG_SYS_U
#define NRG_SYS_U 10  // touch entries per thread in flight before their LDS adds
#endif
constexpr int SYS_T = NRG_SYS_T, SYS_U = NRG_SYS_U;
constexpr u32 NOTOUCH = 0xFFFFFFFFu;

// Buckets of cold words (x relative to hot_reads). Cold word 0 has bucket 0 to itself: an op's
// cold touches start at r1 * tid, so every op of core tid 0 touches cold word 0
// (benches/synthetic.rs:165-171) -- 1/64 of all ops on one word, which as part of an ordinary
// bucket made it 2.5x the mean and the kernel's straggler. Words 1.. go to buckets 1.. of
// W = ceil((span - 1) / 511) words: 512 buckets, 2 workgroups per CU. The division is
// (x * ceil(2^40 / W)) >> 40, exact for x < 2^31 and W <= 512.
__device__ __forceinline__ u32 bucket_of(u32 x, u64 wm) { return x ? 1u + (u32)(((u64)(x - 1) * wm) >> 40) : 0u; }
__device__ __forceinline__ u32 word_in_bucket(u32 x, u32 b, u32 W) { return x ? (x - 1) - (b - 1) * W : 0u; }

// A cold touch in the tile layout, 4 bytes: word within its bucket (9 bits), SET (1), cold
// index k (3), op within its tile (11). The bucket and tile are implied by the position.
__device__ __forceinline__ u32 ent_make(u32 xl, bool set, u32 k, u32 opl) {
    return xl | (set ? 1u << 9 : 0u) | (k << 10) | (opl << 13);
}
__device__ __forceinline__ u32 ent_word(u32 e) { return e & (SYB_WORDS - 1); }
__device__ __forceinline__ bool ent_set(u32 e) { return (e >> 9) & 1u; }
__device__ __forceinline__ u32 ent_op(u32 e) { return e >> 13; }
// In HBM a touch is two 2-B records in parallel arrays: Ew {word in bucket, SET} for the bucket
// pass and Eo {op in tile} for the sums (and the bucket pass's SET passes): each pass reads only
// the half it needs (round 4 kept the 4-B entry: both passes read all 4 B).
__device__ __forceinline__ u16 ent_w(u32 e) { return (u16)(e & 0x3FFu); }
__device__ __forceinline__ u16 ent_o(u32 e) { return (u16)(e >> 13); }

// x mod d for d < 2^32 with m = floor((2^64 - 1) / d): the quotient estimate is at most two low
// (a software 64-bit division costs ~10x more: 10 us of a 1M-op partition pass)
__device__ __forceinline__ u64 mod_recip(u64 x, u64 d, u64 m) {
    u64 r = x - __umul64hi(x, m) * d;
    if (r >= d) r -= d;
    if (r >= d) r -= d;
    return r;
}

// Hot word summary of a run of touches: has ? value = base + cnt : value = before + cnt.
struct SyHot {
    u32 cnt;
    u32 has;
    u64 base;
};
__device__ __forceinline__ SyHot hot_compose(SyHot a, SyHot b) {
    if (b.has) return b;
    a.cnt += b.cnt;
    return a;
}

__device__ __forceinline__ u64 shfl_u64(u64 v, int src) {
    const u32 lo = (u32)__shfl((int)(u32)v, src, 64);
    const u32 hi = (u32)__shfl((int)(u32)(v >> 32), src, 64);
    return ((u64)hi << 32) | lo;
}

// orders a wave's own LDS accesses across lanes (the hardware keeps one wave's LDS
// instructions in order; this stops the compiler from moving them)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Stable ranking of one wave round in a (mask, count) table: every lane with a key ORs its bit
// into mask[key]; the mask read back is the set of lanes with that key. Returns count[key] + the
// number of lower lanes with the same key; the highest such lane advances count and clears mask
// (three LDS round trips; the bucket pass's passes with a WriteOnly, which need the peers).
template <typename CNT>
__device__ __forceinline__ u32 wave_rank_mask(bool on, u32 key, int lane, u64* mask, CNT* count, u64* peers_out) {
    if (on) atomicOr((unsigned long long*)&mask[key], 1ull << lane);
    wave_lds_sync();
    u64 peers = 0;
    u32 c0 = 0;
    if (on) {
        peers = mask[key];
        c0 = count[key];
    }
    wave_lds_sync();
    if (on && 63 - __clzll(peers) == lane) {
        mask[key] = 0;
        count[key] = (CNT)(c0 + (u32)__popcll(peers));
    }
    wave_lds_sync();
    *peers_out = peers;
    return c0 + (u32)__popcll(peers & ((1ull << lane) - 1));
}

// 32-bit seen values. Every cold touch's seen value is < 2^32 when, at the chunk's start, every
// word is < 2^31 and no WriteOnly of the chunk writes a tid >= 2^31 (a seen value is a word's or
// a SET's value plus fewer than 2^31 touches). The bucket pass then stores 4-B seen values (half
// the V traffic of the bucket pass and of the sums). Device-side, per chunk epoch e:
//   big[e & 1] = e   written by any bucket workgroup whose words end chunk e with a value >= 2^31
//   set_epoch[e & 1] = e   written by any partition tile holding such a WriteOnly
//   v32[slot]        the bucket pass's decision, read by the chunk's sums
// Every bucket workgroup decides alike: v32 = big[(e-1) & 1] != e-1 && set_epoch[e & 1] != e.
struct SyFlags {
    u32 big[2];
    u32 set_epoch[2];  // by epoch parity: chunk e's partition and chunk e-1's bucket pass may share a launch
    u32 v32[2];
    u32 wo_epoch[2];  // [e & 1] = e: chunk e holds a WriteOnly (bucket 0 then runs in one workgroup)
};

// Arguments of the partition pass of chunk e and of the sums of chunk e-1, which share a launch.
struct SyPartArgs {
    const nrg_synth_op* src;  // the chunk's ops in a caller buffer, or nullptr (ring)
    nrg_synth_op* ring;
    u64 ring_mask, lo, n, span, span_m;
    u32 w64;  // 2^64 mod span
    u32 HR;
    u64 hr_m;
    u32 HW, NB, W;
    u64 wm;
    u32 ntiles;
    u16* Ew;  // [tile][entry] {word, SET} records
    u16* Eo;  // [tile][entry] op-in-tile records
    u32* cnt_tb;
    SyHot* hot;
    SyFlags* fl;
    u32 epoch;
    u64* dbg;  // NRG_EXP & 2 (diagnostic): phase stamps of tile t in row SY_DBG_PART + t
    bool plain;    // plain stores for the log copy (default; st_out)
    bool plain_e;  // plain stores for the touch records (default)
};
// rows of the diagnostic stamp buffer: bucket b in row b, partition tile t in SY_DBG_PART + t,
// sum workgroup k in SY_DBG_SUM + k (tiles beyond 1024 are not stamped)
constexpr u32 SY_DBG_PART = 1024, SY_DBG_SUM = 2048, SY_DBG_ROWS = 3072;
struct SySumArgs {
    u32 blocks;  // workgroups of the sum role (0: none)
    const u16* Eo;
    const u64* V;
    u64 n, lo, resp_lo, resp_hi;
    u64* resp;
    uint8_t* some;
    u32 tile0, tile1, want;  // response tiles [tile0, tile1), SYS_T per workgroup
    const SyHot* hot;
    u32 ntiles, HR, CW;
    u64* words;
    const u32* v32;  // the chunk's seen-value width flag (SyFlags::v32[par]): 1 = 4-B seen values
    u64* dbg;
    bool plain;  // plain stores for the responses (default; st_out)
};

// LDS of a partition workgroup: ranking tables and staged words, then (same bytes) the tile's
// touches grouped by bucket; the sum role reuses the same bytes for its per-op sums
template <int CW>
struct SyPartLds {
    unsigned short wcnt[SYA_WAVES][SY_MAX_NB];
    union {
        struct {
            u32 words[SYA_WAVES][64 * CW];
        } r;
        u32 stage[SYA_OPS * CW];
        u64 sum[SYS_T * SYA_OPS];
    } u;
    SyHot hot[SYA_WAVES][SY_MAX_HOT];
    u32 part[SYA_WAVES];
};

// src: the chunk's ops in a caller buffer (nrg_synth_round_async); the role then writes the
// log copy itself (lane-contiguous). nullptr: the ops are in the ring.
template <int CW>
__device__ __forceinline__ void sy_part_role(const SyPartArgs& A, u32 tile, SyPartLds<CW>& L) {
    const nrg_synth_op* __restrict__ src = A.src;
    nrg_synth_op* ring = A.ring;
    const u64 ring_mask = A.ring_mask, lo = A.lo, n = A.n, span = A.span, span_m = A.span_m, hr_m = A.hr_m, wm = A.wm;
    const u32 w64 = A.w64;
    const u32 HR = A.HR, HW = A.HW, NB = A.NB, W = A.W;
    u16* __restrict__ Ew = A.Ew;
    u16* __restrict__ Eo = A.Eo;
    u32* __restrict__ cnt_tb = A.cnt_tb;
    SyHot* __restrict__ hot = A.hot;
    auto& s_wcnt = L.wcnt;
    auto& s_u = L.u;
    auto& s_hot = L.hot;
    auto& s_part = L.part;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const u64 op0 = (u64)tile * SYA_OPS;
    // [0] start [1] ops loaded and ranked [2] bucket offsets [3] staged in LDS [4] end, [9] HW_ID [10] XCC_ID
    u64* dbg = (A.dbg && tile < SY_DBG_SUM - SY_DBG_PART && threadIdx.x == 0) ? A.dbg + (u64)(SY_DBG_PART + tile) * 16 : nullptr;
#define SYP_MARK(K) \
    if (dbg) dbg[K] = wall_clock64()
    SYP_MARK(0);
    for (u32 i = tid; i < SYA_WAVES * SY_MAX_NB / 2; i += SYA_TPB) ((u32*)&s_wcnt[0][0])[i] = 0;
    if (lane < SY_MAX_HOT) s_hot[w][lane] = SyHot{0, 0, 0};
    __syncthreads();
    // a ranked cold touch: valid (bit 31), SET (29), word in bucket (20..28), bucket (11..19),
    // rank in the wave's count of its bucket (0..10; < 4 * 64 * CW <= 2048)
    u32 pk[SYA_OROUNDS * CW];
    const u32 opw = (u32)(w * SYA_OROUNDS) * 64 + lane;  // this lane's op in round 0, within the tile
    // the records of the next SYP_PD wave rounds are in flight
    nrg_synth_op nx[SYP_PD];
#pragma unroll
    for (int q = 0; q < SYP_PD; q++) {
        nx[q] = nrg_synth_op{0, 0, 0, 0};
        if (op0 + opw + q * 64 < n) nx[q] = src ? src[op0 + opw + q * 64] : ring[(lo + op0 + opw + q * 64) & ring_mask];
    }
#pragma unroll
    for (int orr = 0; orr < SYA_OROUNDS; orr++) {
        // 64 consecutive ops per wave round; lane = op
        const bool valid = op0 + opw + orr * 64 < n;
        const nrg_synth_op o = nx[orr % SYP_PD];
        if (orr + SYP_PD < SYA_OROUNDS && op0 + opw + (orr + SYP_PD) * 64 < n)
            nx[orr % SYP_PD] = src ? src[op0 + opw + (orr + SYP_PD) * 64]
                                   : ring[(lo + op0 + opw + (orr + SYP_PD) * 64) & ring_mask];
        if (src && valid) st_op(&ring[(lo + op0 + opw + orr * 64) & ring_mask], o, A.plain);
        const bool set = valid && o.op == NRG_SYNTH_WRITE_ONLY;
        if (set && (o.tid >> 31)) A.fl->set_epoch[A.epoch & 1] = A.epoch;  // this chunk's seen values may pass 2^32
        if (set) A.fl->wo_epoch[A.epoch & 1] = A.epoch;                    // this chunk holds a WriteOnly
        // hot touches (r2 + j) % HR, j < HW, skipped when r2 + HW wraps; ordered (lane, j)
        const bool hot_ok = valid && (o.r2 + HW >= o.r2);
        const u32 h0 = hot_ok ? (u32)mod_recip(o.r2, HR, hr_m) : 0u;
        for (u32 h = 0; h < HR; h++) {
            int ls = -1;
            u32 js = 0, tot = 0;
            // (h0 + j) % HR, stepped (no integer division per hot touch)
            for (u32 j = 0, hj = h0; j < HW; j++, hj = hj + 1 == HR ? 0u : hj + 1) {
                const bool on = hot_ok && hj == h;
                const u64 m = __ballot(on);
                const u64 sm = __ballot(on && set);
                tot += (u32)__popcll(m);
                if (sm) {
                    const int l = 63 - __clzll(sm);
                    if (l >= ls) {
                        ls = l;
                        js = j;
                    }
                }
            }
            if (tot == 0) continue;
            u32 after = tot;
            u64 base = 0;
            if (ls >= 0) {
                after = 0;
                const u64 gt = ls == 63 ? 0ull : (~0ull << (ls + 1));
                for (u32 j = 0, hj = h0; j < HW; j++, hj = hj + 1 == HR ? 0u : hj + 1) {
                    const u64 m = __ballot(hot_ok && hj == h);
                    after += (u32)__popcll(m & gt) + ((j > js && ((m >> ls) & 1ull)) ? 1u : 0u);
                }
                base = shfl_u64(o.tid, ls);
            }
            if (lane == 0) {
                SyHot cur = s_hot[w][h];
                s_hot[w][h] = ls >= 0 ? SyHot{after, 1u, base} : SyHot{cur.cnt + tot, cur.has, cur.base};
            }
        }
        // cold touches: this lane's CW words, then rank them in log order (op-major) per bucket
        // word k is (r1·tid + k·r2) mod 2^64 mod span: two reciprocal reductions per op, then
        // stepped in 32 bits -- x += r2 mod span, less 2^64 mod span when the u64 sum wraps
        u64 begin = o.r1 * o.tid;
        u32 xm = (u32)mod_recip(begin, span, span_m);
        const u32 r2m = (u32)mod_recip(o.r2, span, span_m), sp32 = (u32)span;
#pragma unroll
        for (int k = 0; k < CW; k++) {
            s_u.r.words[w][lane * CW + k] = valid ? ((xm + HR) | (set ? SETBIT : 0u)) : NOTOUCH;
            const u64 nb = begin + o.r2;
            const bool wrap = nb < begin;
            begin = nb;
            u32 t = xm + r2m;  // < 2 span < 2^32
            t = t >= sp32 ? t - sp32 : t;
            if (wrap) t = t >= w64 ? t - w64 : t + (sp32 - w64);
            xm = t;
        }
        wave_lds_sync();
        // all CW words read back (one LDS round trip) and bucketed before the rankings, which
        // then cost one round trip each
        u32 vw[CW], bw[CW];
#pragma unroll
        for (int r = 0; r < CW; r++) vw[r] = s_u.r.words[w][r * 64 + lane];
#pragma unroll
        for (int r = 0; r < CW; r++) bw[r] = vw[r] != NOTOUCH ? bucket_of((vw[r] & ~SETBIT) - HR, wm) : 0u;
#pragma unroll
        for (int r = 0; r < CW; r++) {
            // one returning LDS add per touch on the wave's packed u16 count pair
            u32 rank = 0;
            if (vw[r] != NOTOUCH) {
                const u32 sh = (bw[r] & 1u) * 16u;
                rank = (atomicAdd((u32*)&s_wcnt[w][bw[r] & ~1u], 1u << sh) >> sh) & 0xFFFFu;
            }
            const u32 xl = word_in_bucket((vw[r] & ~SETBIT) - HR, bw[r], W);
            pk[orr * CW + r] = vw[r] == NOTOUCH ? 0u
                                                : (1u << 31) | ((vw[r] & SETBIT) ? 1u << 29 : 0u) | (xl << 20) | (bw[r] << 11) | rank;
        }
    }
    __syncthreads();
    SYP_MARK(1);
    // bucket totals over the waves; wave prefixes; thread t owns bucket t
    const u32 bt = tid;
    u32 tot = 0;
    if (bt < NB)
        for (int ww = 0; ww < SYA_WAVES; ww++) {
            const u32 c = s_wcnt[ww][bt];
            s_wcnt[ww][bt] = (unsigned short)tot;
            tot += c;
        }
    u32 inc = tot;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u32 y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) s_part[w] = inc;
    __syncthreads();
    u32 toff = inc - tot;
    for (int ww = 0; ww < w; ww++) toff += s_part[ww];
    if (bt < NB) {
        for (int ww = 0; ww < SYA_WAVES; ww++) s_wcnt[ww][bt] = (unsigned short)(s_wcnt[ww][bt] + toff);
        cnt_tb[(u64)tile * NB + bt] = (toff << 16) | tot;  // [tile][bucket]: one coalesced row per tile
    }
    if ((u32)tid < HR) {
        SyHot a{0, 0, 0};
        for (int ww = 0; ww < SYA_WAVES; ww++) a = hot_compose(a, s_hot[ww][tid]);
        hot[(u64)tile * HR + tid] = a;
    }
    __syncthreads();
    SYP_MARK(2);
#pragma unroll
    for (int orr = 0; orr < SYA_OROUNDS; orr++) {
#pragma unroll
        for (int r = 0; r < CW; r++) {
            const u32 p = pk[orr * CW + r];
            if (!(p >> 31)) continue;
            const u32 t = r * 64 + lane;
            const u32 opl = (u32)(w * SYA_OROUNDS + orr) * 64 + t / CW;
            s_u.stage[s_wcnt[w][(p >> 11) & 511u] + (p & 2047u)] = ent_make((p >> 20) & 511u, (p >> 29) & 1u, t % CW, opl);
        }
    }
    __syncthreads();
    SYP_MARK(3);
    const u32 nops = (u32)(n - op0 < SYA_OPS ? n - op0 : SYA_OPS);
    // two records per thread: 4-B stores into each array
    u32* Ewt = (u32*)(Ew + (u64)tile * (SYA_OPS * CW));
    u32* Eot = (u32*)(Eo + (u64)tile * (SYA_OPS * CW));
    const u32 ne = nops * CW;
    for (u32 i = tid; 2 * i < ne; i += SYA_TPB) {
        const u32 a = s_u.stage[2 * i], b = 2 * i + 1 < ne ? s_u.stage[2 * i + 1] : 0u;
        st_out(&Ewt[i], (u32)ent_w(a) | ((u32)ent_w(b) << 16), A.plain_e);
        st_out(&Eot[i], (u32)ent_o(a) | ((u32)ent_o(b) << 16), A.plain_e);
    }
    if (dbg) {
        dbg[4] = wall_clock64();
        dbg[9] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        dbg[10] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    }
#undef SYP_MARK
}

// One workgroup per bucket. Passes of SYB_PASS touches in log order; wave w takes the pass's
// w-th contiguous SYB_PER rounds of 64: wave-private per-word counts rank the wave's
// touches without barriers, then per-word prefixes over the waves place them. A pass with a
// WriteOnly in it is applied wave by wave instead (values depend on the last SET).
// (<= 128 VGPRs: two 8-wave workgroups per CU)
#ifndef NRG_SYB_WPE
#define NRG_SYB_WPE 4  // waves per SIMD the bucket pass is compiled for (4: 128 VGPRs, two workgroups per CU)
#endif
// Arguments of the bucket pass of one chunk.
struct SyBucketArgs {
    const u16* Ew;
    const u16* Eo;
    const u32* cnt_tb;
    u32 NB, ntiles, tile_entries;
    u64* V;
    u64* words;
    u64 N;
    u32 HR, W;
    const nrg_synth_op* ring;
    u64 ring_mask, lo;
    SyFlags* fl;
    u32 epoch, vslot;  // the chunk's epoch; its seen values' slot (SyFlags::v32[vslot])
    u64* dbg;
    u32 stall;
    bool plain;
};
// LDS of a bucket workgroup; its dynamic part (s_pre[ntiles + 1], s_off[ntiles] u16) follows
template <int PER>
struct SyBucketLds {
    u64 cur[SYB_WORDS];
    u32 wc[SYB_WAVES][SYB_WORDS];
    u64 mk[SYB_WORDS];  // peer masks of the passes with a WriteOnly (one wave at a time)
    unsigned short tile[2][SYB_TPB * PER];  // tile of every touch of a pass (double buffered)
    u32 part[SYB_WAVES];
    u32 big;  // a word ends the chunk >= 2^31 (SyFlags)
};
__host__ __device__ constexpr size_t sy_bucket_dyn_bytes(u32 ntiles) { return (size_t)(ntiles + 1) * 4 + (size_t)ntiles * 2; }

// Workgroup `blk` of the pass's `nblk` (two per CU): its bucket, or a part of bucket 0.
template <int PER>
__device__ __forceinline__ void sy_bucket_role(const SyBucketArgs& B, u32 blk, u32 nblk, SyBucketLds<PER>& L, u32* s_dyn) {
    constexpr u32 SYB_PASS = SYB_TPB * PER;  // touches per pass
    constexpr int SYB_PER = PER;
    const u16* __restrict__ Ew = B.Ew;
    const u16* __restrict__ Eo = B.Eo;
    const u32* __restrict__ cnt_tb = B.cnt_tb;
    const u32 NB = B.NB, ntiles = B.ntiles, tile_entries = B.tile_entries, HR = B.HR, W = B.W, epoch = B.epoch;
    u64* __restrict__ V = B.V;
    u64* __restrict__ words = B.words;
    const u64 N = B.N, ring_mask = B.ring_mask, lo = B.lo;
    const nrg_synth_op* __restrict__ ring = B.ring;
    SyFlags* __restrict__ fl = B.fl;
    u64* __restrict__ dbg = B.dbg;
    const u32 stall = B.stall;
    const bool plain = B.plain;
    // dbg (NRG_EXP & 2, diagnostic): per block, thread 0's wall clock at the phase edges
    // [0] start [1] prologue loaded [2] scanned, then summed over passes [3] tile map [4] gather
    // [5] rank + place [6] stores, [7] end, [8] passes
    u64 tm_acc[4] = {0, 0, 0, 0}, tm_last = 0;
#define SY_MARK(K) \
    if (dbg && threadIdx.x == 0) dbg[(u64)blk * 16 + (K)] = tm_last = wall_clock64()
#define SY_ACC(K)                                  \
    if (dbg && threadIdx.x == 0) {                 \
        const u64 now_ = wall_clock64();           \
        tm_acc[K] += now_ - tm_last;               \
        tm_last = now_;                            \
    }
    SY_MARK(0);
    auto& s_cur = L.cur;
    auto& s_wc = L.wc;
    auto& s_mk = L.mk;
    auto& s_tile = L.tile;
    auto& s_part = L.part;
    auto& s_big = L.big;
    u32* s_pre = s_dyn;
    unsigned short* s_off = (unsigned short*)(s_dyn + ntiles + 1);
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    // buckets in contiguous runs per XCD (workgroups go to XCDs round-robin): neighbouring
    // buckets share the lines at their segments' edges in E and V, and those stay in one L2
    const u32 nxcd = 8, q = nblk / nxcd, rem = nblk % nxcd, xcd = blk % nxcd;
    const u32 v = xcd * q + (xcd < rem ? xcd : rem) + blk / nxcd;
    // v = 0..H: the parts of bucket 0 (H = nblk - NB helpers beside its own workgroup)
    const u32 H = nblk - NB;
    const u32 b = v <= H ? 0u : v - H, part = v <= H ? v : 0u;
    const bool split = b == 0 && H && fl->wo_epoch[epoch & 1] != epoch;
    if (b == 0 && part && !split) return;  // a WriteOnly in the chunk: bucket 0 in one workgroup
    const u64 w0 = b ? (u64)HR + 1 + (u64)(b - 1) * W : (u64)HR;  // bucket 0: cold word 0 alone
    const u32 nw = b ? W : 1u;
    // 4-B seen values this chunk (SyFlags): decided alike by every workgroup
    const bool v32 = fl->big[(epoch - 1) & 1] != epoch - 1 && fl->set_epoch[epoch & 1] != epoch;
    for (u32 t = tid; t < ntiles; t += SYB_TPB) {
        // [tile][bucket]: a tile's word for bucket b shares its line with the neighbouring buckets,
        // which run on this XCD (the contiguous runs above), so the line is fetched once per XCD
        const u32 p = cnt_tb[(u64)t * NB + b];
        s_off[t] = (unsigned short)(p >> 16);
        s_pre[t] = p & 0xFFFFu;
    }
    for (u32 i = tid; i < SYB_WORDS; i += SYB_TPB) s_cur[i] = i < nw && w0 + i < N ? words[w0 + i] : 0ull;
    if (tid == 0) s_big = 0;
    for (u32 i = tid; i < SYB_WORDS; i += SYB_TPB) s_mk[i] = 0;
    for (u32 i = tid; i < SYB_WAVES * SYB_WORDS; i += SYB_TPB) (&s_wc[0][0])[i] = 0;
    __syncthreads();
    SY_MARK(1);
    // exclusive scan of the per-tile counts: thread owns tiles [tid*K, tid*K + K)
    const u32 K = (ntiles + SYB_TPB - 1) / SYB_TPB;
    u32 loc = 0;
    for (u32 q = 0; q < K; q++) {
        const u32 t = tid * K + q;
        if (t < ntiles) loc += s_pre[t];
    }
    u32 inc = loc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u32 y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) s_part[w] = inc;
    __syncthreads();
    u32 run = inc - loc;
    for (int ww = 0; ww < w; ww++) run += s_part[ww];
    u32 total = 0;
    for (int ww = 0; ww < SYB_WAVES; ww++) total += s_part[ww];
    for (u32 q = 0; q < K; q++) {
        const u32 t = tid * K + q;
        if (t < ntiles) {
            const u32 c = s_pre[t];
            s_pre[t] = run;
            run += c;
        }
    }
    if (tid == 0) s_pre[ntiles] = total;
    // this workgroup's touches [start, end): all of its bucket's, or a part of bucket 0's, whose
    // word starts the part at its value plus the touches before it
    const u32 start = split ? (u32)((u64)total * part / (H + 1)) : 0u;
    const u32 end = split ? (u32)((u64)total * (part + 1) / (H + 1)) : total;
    if (split && tid == 0) s_cur[0] += start;
    __syncthreads();
    SY_MARK(2);
    // The pass starting at `base`: the tile of each of its touches, then this thread's entries.
    auto map_pass = [&](u32 base, unsigned short* map) {
        for (u32 t = tid; t < ntiles; t += SYB_TPB) {
            const u32 a = s_pre[t] > base ? s_pre[t] : base;
            const u32 z = s_pre[t + 1] < base + SYB_PASS ? s_pre[t + 1] : base + SYB_PASS;
            for (u32 j = a; j < z; j++) map[j - base] = (unsigned short)t;
        }
    };
    u32 nent[SYB_PER];
    // E position of touch i of the pass at `base` (its tile from the pass's map); recomputed
    // where needed rather than kept per touch (frees 2 * SYB_PER registers for larger passes)
    auto gpos_of = [&](u32 base, const unsigned short* map, u32 i) -> u32 {
        const u32 t = map[i - base];
        return t * tile_entries + s_off[t] + (i - s_pre[t]);
    };
    // (measured and dropped: seen values stored at their op's position in the tile, op * CW + k,
    // so the sums read V alone -- 89 vs 56.5 us per round: the scattered 4-B stores cost more
    // than the second read of E; profiles/r03_synth_opmajor_dropped.txt)
    auto load_pass = [&](u32 base, const unsigned short* map) {
#pragma unroll
        for (int q = 0; q < SYB_PER; q++) {
            const u32 i = base + (u32)w * (SYB_PER * 64) + q * 64 + lane;
            nent[q] = i < end ? (u32)Ew[gpos_of(base, map, i)] : 0u;
        }
    };
    if (start < end) {
        map_pass(start, s_tile[0]);
        __syncthreads();
        load_pass(start, s_tile[0]);
    }
    // Software pipelined: the next pass's entries are in flight while this pass is ranked.
    const u32 late = blk >= nblk / 2 ? 1u : 0u;  // the second workgroup on its CU
    for (u32 base = start, pb = 0; base < end; base += SYB_PASS, pb ^= 1) {
        // alternate which of a CU's two workgroups the SIMDs prefer, pass by pass: oldest-first
        // arbitration otherwise favours the first-dispatched one all the way through, and the
        // second ones ended 3.6 us later (profiles/r04_stack_synth_phases.txt; 55.97-56.83 vs
        // 56.53-57.18 us per round, profiles/r04_synth_setprio.txt)
        if ((pb ^ late) & 1u) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
        u32 ent[SYB_PER];
        const unsigned short* cmap = s_tile[pb];
        u64 sv[SYB_PER];
        bool myset = false;
#pragma unroll
        for (int q = 0; q < SYB_PER; q++) {
            ent[q] = nent[q];
            myset |= ent_set(ent[q]);
        }
        SY_ACC(1);
        const u32 nb = base + SYB_PASS;
        if (nb < end) map_pass(nb, s_tile[pb ^ 1]);
        const int anyset = __syncthreads_or(myset);  // also publishes the next pass's tile map
        if (nb < end) load_pass(nb, s_tile[pb ^ 1]);
        SY_ACC(0);
        if (!anyset) {
            if (b == 0) {  // one word: a touch's rank in its wave is its position there
                const u32 w0i = base + (u32)w * (SYB_PER * 64);
                u32 l = (u32)lane;
                asm volatile("" : "+v"(l));  // computed per pass: hoisted, these 8 constants spilled
#pragma unroll
                for (int q = 0; q < SYB_PER; q++) sv[q] = (u64)(q * 64 + l);
                if (lane == 0)
                    s_wc[w][0] = end > w0i ? (end - w0i < SYB_PER * 64 ? end - w0i : SYB_PER * 64) : 0u;
            } else {
#pragma unroll
                for (int q = 0; q < SYB_PER; q++) {
                    const u32 i = base + (u32)w * (SYB_PER * 64) + q * 64 + lane;
                    sv[q] = i < end ? atomicAdd(&s_wc[w][ent_word(ent[q])], 1u) : 0u;
                }
            }
            __syncthreads();
            u64 totw = 0;
            if (tid < (int)SYB_WORDS) {
                u32 acc = 0;
                for (int ww = 0; ww < SYB_WAVES; ww++) {
                    const u32 c = s_wc[ww][tid];
                    s_wc[ww][tid] = acc;
                    acc += c;
                }
                totw = acc;
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < SYB_PER; q++) {
                const u32 xl = ent_word(ent[q]);
                sv[q] += s_cur[xl] + s_wc[w][xl];
            }
            __syncthreads();
            if (tid < (int)SYB_WORDS) {
                s_cur[tid] += totw;
                for (int ww = 0; ww < SYB_WAVES; ww++) s_wc[ww][tid] = 0;
            }
        } else {
#pragma unroll
            for (int q = 0; q < SYB_PER; q++) {
                const bool isset = ent_set(ent[q]);  // 0 for touches past the end
                const u32 iq = base + (u32)w * (SYB_PER * 64) + q * 64 + lane;
                // (the op of a SET touch: its Eo record, read only in passes with a WriteOnly)
                const u64 op = isset && iq < end ? (u64)cmap[iq - base] * SYA_OPS + Eo[gpos_of(base, cmap, iq)] : 0ull;
                sv[q] = isset ? ring[(lo + op) & ring_mask].tid : 0ull;
            }
            for (int ww = 0; ww < SYB_WAVES; ww++) {
                if (ww == w) {
#pragma unroll
                    for (int q = 0; q < SYB_PER; q++) {
                        const u32 i = base + (u32)w * (SYB_PER * 64) + q * 64 + lane;
                        const bool valid = i < end;
                        const u32 xl = ent_word(ent[q]);
                        const bool isset = valid && ent_set(ent[q]);
                        u64 peers;
                        (void)wave_rank_mask(valid, xl, lane, s_mk, s_wc[w], &peers);
                        const u64 P = peers & ((1ull << lane) - 1);
                        const u64 S = __ballot(isset) & P;
                        const int sl = S ? 63 - __clzll(S) : lane;
                        const u64 stid = shfl_u64(sv[q], sl);
                        u64 seen = 0;
                        if (valid) {
                            if (S) seen = stid + (u64)__popcll(P & ~((2ull << sl) - 1));
                            else seen = s_cur[xl] + (u64)__popcll(P);
                        }
                        wave_lds_sync();
                        if (valid && 63 - __clzll(peers) == lane) s_cur[xl] = isset ? sv[q] : seen + 1;
                        wave_lds_sync();
                        sv[q] = isset ? 0ull : seen;
                    }
                    for (u32 k = lane; k < SYB_WORDS; k += 64) s_wc[w][k] = 0;
                }
                __syncthreads();
            }
        }
        SY_ACC(2);
        test_stall(stall & 1, w);  // (tests) slow waves still read cmap below
        // (stall & 2, diagnostic: a map overwritten under a slow wave gives a wild position; the
        // store is dropped instead of landing outside V)
        const u32 vcap = (stall & 2) ? ntiles * tile_entries : ~0u;
        if (v32) {
#pragma unroll
            for (int q = 0; q < SYB_PER; q++)
                if (base + (u32)w * (SYB_PER * 64) + q * 64 + lane < end) {
                    const u32 gp = gpos_of(base, cmap, base + (u32)w * (SYB_PER * 64) + q * 64 + lane);
                    if (gp < vcap) st_out(&((u32*)V)[gp], (u32)sv[q], plain);
                }
        } else {
#pragma unroll
            for (int q = 0; q < SYB_PER; q++)
                if (base + (u32)w * (SYB_PER * 64) + q * 64 + lane < end) {
                    const u32 gp = gpos_of(base, cmap, base + (u32)w * (SYB_PER * 64) + q * 64 + lane);
                    if (gp < vcap) st_out(&V[gp], sv[q], plain);
                }
        }
        // the stores above read this pass's tile map (cmap); the next pass's map is built into
        // the other buffer, but the pass after that overwrites this one: every wave must be done
        // with it before any wave starts the next iteration's map_pass
        if (!(stall & 2)) __syncthreads();  // (stall & 2: diagnostic only, results wrong)
        SY_ACC(3);
    }
    bool big = false;
    const bool owner = !split || part == H;  // bucket 0's last part ends at the word's value
    for (u32 i = tid; owner && i < nw; i += SYB_TPB)
        if (w0 + i < N) {
            words[w0 + i] = s_cur[i];
            big |= (s_cur[i] >> 31) != 0;
        }
    if (big) s_big = 1u;  // (an LDS flag: __syncthreads_or here kept the thread-id math live and spilled)
    __syncthreads();
    if (s_big && tid == 0) fl->big[epoch & 1] = epoch;
    if (blk == 0 && tid == 0) fl->v32[B.vslot] = v32 ? 1u : 0u;
    if (dbg && threadIdx.x == 0) {
        for (int k = 0; k < 4; k++) dbg[(u64)blk * 16 + 3 + k] = tm_acc[k];
        dbg[(u64)blk * 16 + 8] = (total + SYB_PASS - 1) / SYB_PASS;
        dbg[(u64)blk * 16 + 9] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        dbg[(u64)blk * 16 + 10] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
        dbg[(u64)blk * 16 + 11] = total;
    }
    SY_MARK(7);
#undef SY_MARK
#undef SY_ACC
}

__global__ __launch_bounds__(SYB_TPB) __attribute__((amdgpu_waves_per_eu(NRG_SYB_WPE))) void sy_bucket_kernel(SyBucketArgs B) {
    extern __shared__ u32 s_dyn[];  // s_pre[ntiles + 1], s_off[ntiles] (u16)
    __shared__ SyBucketLds<SYB_PER> L;
    sy_bucket_role<SYB_PER>(B, blockIdx.x, gridDim.x, L, s_dyn);
}

// Per-op sums of chunk S (one workgroup per 2048-op tile of the response window), then, in
// workgroup 0, the ordered fold of the tiles' hot-word summaries into the hot words.
__device__ __forceinline__ void sy_sum_role(const SySumArgs& S, u32 blk, u64* s_sum) {
    const u16* __restrict__ Eo = S.Eo;
    const u64* __restrict__ V = S.V;
    const u64 n = S.n, lo = S.lo, resp_lo = S.resp_lo, resp_hi = S.resp_hi;
    u64* __restrict__ resp = S.resp;
    uint8_t* __restrict__ some = S.some;
    const u32 tile0 = S.tile0, want = S.want, ntiles = S.ntiles, HR = S.HR, CW = S.CW;
    const SyHot* __restrict__ hot = S.hot;
    u64* __restrict__ words = S.words;
    const int tid = threadIdx.x;
    // [0] start [1] sums added [2] responses stored [3] hot fold done (workgroup 0)
    u64* dbg = (S.dbg && blk < SY_DBG_ROWS - SY_DBG_SUM && threadIdx.x == 0) ? S.dbg + (u64)(SY_DBG_SUM + blk) * 16 : nullptr;
    if (dbg) dbg[0] = wall_clock64();
    if (want) {
        // SYS_T consecutive tiles: their entries are contiguous (TE per tile; only the chunk's
        // last tile is partial), sums in s_sum[j * SYA_OPS + op]
        const u32 t0 = tile0 + blk * SYS_T;
        const u32 nt = S.tile1 - t0 < (u32)SYS_T ? S.tile1 - t0 : (u32)SYS_T;
        const u64 op0 = (u64)t0 * SYA_OPS;
        const u64 nops = n - op0 < (u64)nt * SYA_OPS ? n - op0 : (u64)nt * SYA_OPS;  // ops of the run
        for (u32 i = tid; i < SYS_T * SYA_OPS; i += SYC_TPB) s_sum[i] = 0;
        __syncthreads();
        const u32 TE = SYA_OPS * CW;
        const u16* Et = Eo + (u64)t0 * TE;
        // the run's entries: whole tiles of TE, then the last tile's nops % SYA_OPS ops
        const u32 ne = (u32)(nops / SYA_OPS) * TE + (u32)(nops % SYA_OPS) * CW;
        // SYS_U entries per thread in flight before their LDS adds (one at a time, every add
        // waited for its own two loads: 8-10 us per workgroup)
        auto add_all = [&](auto Vt) {
            for (u32 e0 = tid; e0 < ne; e0 += SYC_TPB * SYS_U) {
                u32 ee[SYS_U];
                u64 vv[SYS_U];
#pragma unroll
                for (int q = 0; q < SYS_U; q++) {
                    const u32 e = e0 + q * SYC_TPB;
                    ee[q] = e < ne ? Et[e] : 0u;
                    vv[q] = e < ne ? (u64)Vt[e] : 0ull;
                }
#pragma unroll
                for (int q = 0; q < SYS_U; q++) {
                    const u32 e = e0 + q * SYC_TPB;
                    const u32 j = SYS_T == 1 ? 0u : SYS_T == 2 ? (u32)(e >= TE) : e / TE;
                    if (e < ne) atomicAdd((unsigned long long*)&s_sum[j * SYA_OPS + ee[q]], (unsigned long long)vv[q]);
                }
            }
        };
        if (*S.v32) {
            add_all((const u32*)V + (u64)t0 * TE);  // 4-B seen values (SyFlags)
        } else {
            add_all(V + (u64)t0 * TE);
        }
        __syncthreads();
        if (dbg) dbg[1] = wall_clock64();
        for (u32 i = tid; i < nops; i += SYC_TPB) {
            const u64 g = lo + op0 + i;
            if (g >= resp_lo && g < resp_hi) {
#if NRG_SY_RESP_NT
                __builtin_nontemporal_store(s_sum[i], &resp[g - resp_lo]);
                if (some) __builtin_nontemporal_store((uint8_t)1, &some[g - resp_lo]);
#else
                st_out(&resp[g - resp_lo], s_sum[i], S.plain);
                if (some) st_out(&some[g - resp_lo], (uint8_t)1, S.plain);
#endif
            }
        }
    }
    if (dbg) {
        dbg[2] = wall_clock64();
        dbg[9] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        dbg[10] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
    if (blk != 0) return;
    // hot words: ordered fold of the tiles' summaries
    __syncthreads();
    SyHot* s_h = (SyHot*)s_sum;  // SYC_TPB entries
    const u32 K = (ntiles + SYC_TPB - 1) / SYC_TPB;
    for (u32 h = 0; h < HR; h++) {
        SyHot a{0, 0, 0};
        for (u32 q = 0; q < K; q++) {
            const u32 t = tid * K + q;
            if (t < ntiles) a = hot_compose(a, hot[(u64)t * HR + h]);
        }
        s_h[tid] = a;
        for (int st = 1; st < SYC_TPB; st <<= 1) {
            __syncthreads();
            if ((tid & (2 * st - 1)) == 0) s_h[tid] = hot_compose(s_h[tid], s_h[tid + st]);
        }
        __syncthreads();
        if (tid == 0) {
            const SyHot r = s_h[0];
            words[h] = r.has ? r.base + r.cnt : words[h] + r.cnt;
        }
        __syncthreads();
    }
    if (dbg) dbg[3] = wall_clock64();
}

// One launch: the partition of chunk e in workgroups [0, A.ntiles) (on the critical path: the
// bucket pass waits for it) and the sums of chunk e-1 in the workgroups behind them.
template <int CW>
__global__ __launch_bounds__(SYA_TPB) void sy_part_kernel(SyPartArgs A, SySumArgs S) {
    __shared__ SyPartLds<CW> L;
    if (blockIdx.x < A.ntiles)
        sy_part_role<CW>(A, blockIdx.x, L);
    else
        sy_sum_role(S, blockIdx.x - A.ntiles, L.u.sum);
}

// buckets: 0 = cold word 0, then W words each over at most SY_MAX_NB - SY_B0_PARTS buckets
static u64 sy_bucket_words(u64 span) {
    const u64 nbw = SY_MAX_NB - SY_B0_PARTS;
    return span > 1 ? (span - 1 + nbw - 1) / nbw : 1;
}
bool sy_bucket_eligible(const nrg_config& cf) {
    const u64 span = cf.synth_n - cf.synth_hot_reads;
    return cf.synth_cold_writes >= 1 && cf.synth_cold_writes <= SY_MAX_CW && cf.synth_hot_reads <= SY_MAX_HOT &&
           span <= 1 + (u64)(SY_MAX_NB - SY_B0_PARTS) * SYB_WORDS && cf.max_batch <= (u64)SY_MAX_TILES * SYA_OPS;
}

// Scratch: seen values V in two slots (chunk epoch & 1), touch records E in three (epoch % 3:
// Ew then Eo), [tile][bucket] counts in two (epoch & 1), hot summaries in three (epoch % 3).
// With one launch per round (NRG_KNOB_SY_FUSED) the partition of chunk e, the bucket pass of
// e-1 and the sums of e-2 share a launch: E and the hot summaries are live for three chunks,
// the counts and V for two. (The two-launch round needs two slots of E and one of counts and V.)
struct SyAux {
    u64 te;  // touch records per slot
    u64* V[2];  // u64 seen values, or u32 ones (SyFlags) in the same bytes
    u32* E[3];
    u32* cnt[2];
    SyHot* hot[3];
    SyFlags* fl;
};
static u64 sy_nb(const nrg_config& cf) {
    const u64 span = cf.synth_n - cf.synth_hot_reads;
    const u64 W = sy_bucket_words(span);
    return 1 + (span - 1 + W - 1) / W;
}
static SyAux sy_aux(void* base, const nrg_config& cf) {
    const u64 tiles = (cf.max_batch + SYA_OPS - 1) / SYA_OPS;
    const u64 te = tiles * SYA_OPS * cf.synth_cold_writes;
    const u64 nbt = sy_nb(cf) * tiles, ht = tiles * cf.synth_hot_reads;
    SyAux x;
    x.te = te;
    x.V[0] = (u64*)base;
    x.V[1] = x.V[0] + te;
    x.E[0] = (u32*)(x.V[1] + te);  // per slot: Ew (te u16) then Eo (te u16)
    x.E[1] = x.E[0] + te;
    x.E[2] = x.E[1] + te;
    x.cnt[0] = x.E[2] + te;
    x.cnt[1] = x.cnt[0] + nbt;
    x.hot[0] = (SyHot*)(((uintptr_t)(x.cnt[1] + nbt) + 15) & ~(uintptr_t)15);
    x.hot[1] = x.hot[0] + ht;
    x.hot[2] = x.hot[1] + ht;
    x.fl = (SyFlags*)(((uintptr_t)(x.hot[2] + ht) + 15) & ~(uintptr_t)15);
    return x;
}
static u16* sy_ew(const SyAux& x, u32 epoch) { return (u16*)x.E[epoch % 3]; }
static u16* sy_eo(const SyAux& x, u32 epoch) { return (u16*)x.E[epoch % 3] + x.te; }

u64 sy_bucket_aux_bytes(const nrg_config& cf) {
    const u64 tiles = (cf.max_batch + SYA_OPS - 1) / SYA_OPS;
    const u64 te = tiles * SYA_OPS * cf.synth_cold_writes;
    return te * (2 * 8 + 3 * 4) + 2 * sy_nb(cf) * tiles * 4 + 3 * tiles * cf.synth_hot_reads * sizeof(SyHot) + 256 +
           sizeof(SyFlags) + 32;
}

// Fresh scratch: the words may hold anything (sort-path chunks ran before), so the next chunk
// (epoch sy_round + 1) takes 8-B seen values: big[sy_round & 1] = sy_round.
hipError_t sy_aux_init(nrg_ctx* c) {
    SyAux x = sy_aux(c->d_sy_aux, c->cfg);
    SyFlags f{};
    f.big[0] = f.big[1] = c->sy_round;  // the other slot is compared with sy_round + 1 + 2k: never equal
    return hipMemcpy(x.fl, &f, sizeof f, hipMemcpyHostToDevice);
}

static SySumArgs sy_sum_args(nrg_ctx* c, const SyDeferred& d) {
    const nrg_config& cf = c->cfg;
    SyAux x = sy_aux(c->d_sy_aux, cf);
    SySumArgs S{};
    if (!d.valid) return S;
    S.blocks = (d.t1 - d.t0 + SYS_T - 1) / SYS_T;
    S.Eo = sy_eo(x, d.epoch);
    S.V = x.V[d.epoch & 1];
    S.n = d.n;
    S.lo = d.lo;
    S.resp_lo = d.rlo;
    S.resp_hi = d.rhi;
    S.resp = d.resp;
    S.some = d.some;
    S.tile0 = d.t0;
    S.tile1 = d.t1;
    S.want = d.want;
    S.hot = x.hot[d.epoch % 3];
    S.ntiles = d.ntiles;
    S.HR = cf.synth_hot_reads;
    S.CW = cf.synth_cold_writes;
    S.words = c->d_words;
    S.v32 = &x.fl->v32[d.epoch & 1];
    S.dbg = (c->exp & 2) ? c->d_dbg : nullptr;
    S.plain = !((c->exp >> 9) & 1);
    return S;
}

// bucket 0: cold word 0 alone; buckets 1..: W words each (<= 512, sy_bucket_eligible)
static u32 sy_W(const nrg_config& cf) { return (u32)sy_bucket_words(cf.synth_n - cf.synth_hot_reads); }
static u32 sy_NB(const nrg_config& cf) {
    const u64 span = cf.synth_n - cf.synth_hot_reads;
    const u32 W = sy_W(cf);
    return 1 + (u32)((span - 1 + W - 1) / W);
}

static SyBucketArgs sy_bucket_args(nrg_ctx* c, const SyDeferred& d) {
    const nrg_config& cf = c->cfg;
    SyAux x = sy_aux(c->d_sy_aux, cf);
    SyBucketArgs B{};
    B.Ew = sy_ew(x, d.epoch);
    B.Eo = sy_eo(x, d.epoch);
    B.cnt_tb = x.cnt[d.epoch & 1];
    B.NB = sy_NB(cf);
    B.ntiles = d.ntiles;
    B.tile_entries = SYA_OPS * cf.synth_cold_writes;
    B.V = x.V[d.epoch & 1];
    B.words = c->d_words;
    B.N = cf.synth_n;
    B.HR = cf.synth_hot_reads;
    B.W = sy_W(cf);
    B.ring = (const nrg_synth_op*)c->d_ring;
    B.ring_mask = c->log_size - 1;
    B.lo = d.lo;
    B.fl = x.fl;
    B.epoch = d.epoch;
    B.vslot = d.epoch & 1;
    B.dbg = (c->exp & 2) ? c->d_dbg : nullptr;
    B.stall = c->stall;
    B.plain = !((c->exp >> 8) & 1);
    return B;
}

static SyPartArgs sy_part_args(nrg_ctx* c, u64 lo, u64 n, const nrg_synth_op* src, u32 epoch) {
    const nrg_config& cf = c->cfg;
    const u32 HR = cf.synth_hot_reads;
    const u64 span = cf.synth_n - HR;
    SyAux x = sy_aux(c->d_sy_aux, cf);
    SyPartArgs A;
    A.src = src;
    A.ring = (nrg_synth_op*)c->d_ring;
    A.ring_mask = c->log_size - 1;
    A.lo = lo;
    A.n = n;
    A.span = span;
    A.span_m = ~0ull / span;
    A.w64 = (u32)((~0ull % span + 1) % span);
    A.HR = HR;
    A.hr_m = ~0ull / HR;
    A.HW = cf.synth_hot_writes;
    A.NB = sy_NB(cf);
    A.W = sy_W(cf);
    A.wm = ((1ull << 40) + A.W - 1) / A.W;
    A.ntiles = (u32)((n + SYA_OPS - 1) / SYA_OPS);
    A.Ew = sy_ew(x, epoch);
    A.Eo = sy_eo(x, epoch);
    A.cnt_tb = x.cnt[epoch & 1];
    A.hot = x.hot[epoch % 3];
    A.fl = x.fl;
    A.epoch = epoch;
    A.dbg = (c->exp & 2) ? c->d_dbg : nullptr;
    A.plain = !((c->exp >> 6) & 1);
    A.plain_e = !((c->exp >> 7) & 1);
    return A;
}

static hipError_t sy_launch_part(nrg_ctx* c, const SyPartArgs& A, const SySumArgs& S) {
    const unsigned grid = A.ntiles + S.blocks;
    hipStream_t st = c->stream;
#define SY_PART(CWV) \
    case CWV: sy_part_kernel<CWV><<<grid, SYA_TPB, 0, st>>>(A, S); break
    switch (c->cfg.synth_cold_writes) {
        SY_PART(1); SY_PART(2); SY_PART(3); SY_PART(4); SY_PART(5); SY_PART(6); SY_PART(7); SY_PART(8);
        default: return hipErrorInvalidValue;
    }
#undef SY_PART
    return hipGetLastError();
}

// One launch per round (NRG_KNOB_SY_FUSED): the partition of chunk e (A), the bucket pass of
// chunk e-1 (B, when bvalid) and the sums of chunk e-2 (S) in SY_FUSED_WG workgroups, two per CU,
// all resident at once. Workgroup w takes partition tile w, bucket workgroup w and sum workgroup
// w (and w + SY_FUSED_WG, ... for larger chunks); the first of a CU's two workgroups partitions
// first, the second replays its bucket first, so each CU runs one of each side by side (the
// partition streams records at memory bandwidth, the bucket pass is LDS- and latency-bound),
// and the sums follow. No role waits on another in the launch: the three chunks share no buffer.
constexpr u32 SY_FUSED_WG = SY_MAX_NB;  // = the bucket pass's workgroups: 2 per CU on 256 CUs
#ifndef NRG_SYF_PER
#define NRG_SYF_PER 10  // bucket-pass touches per thread per pass in the fused kernel
#endif
constexpr int SYF_PER = NRG_SYF_PER;
// The roles read their arguments through a laundered kernarg pointer at their point of use:
// the compiler cannot then keep the fields of the roles that run later live in registers across
// the roles that run first (kept live, they pushed the bucket role from 125 VGPRs into scratch).
// Kernarg layout of sy_round_kernel: A, B, S at their natural alignments, in order.
constexpr size_t sy_al(size_t x, size_t a) { return (x + a - 1) / a * a; }
constexpr size_t SY_KA_B = sy_al(sizeof(SyPartArgs), alignof(SyBucketArgs));
constexpr size_t SY_KA_S = sy_al(SY_KA_B + sizeof(SyBucketArgs), alignof(SySumArgs));
template <typename T>
__device__ __forceinline__ const T* sy_karg(size_t off) {
    const char __attribute__((address_space(4)))* k =
        (const char __attribute__((address_space(4)))*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k));
    return (const T*)(const T __attribute__((address_space(4)))*)(k + off);
}
template <int CW>
__device__ __forceinline__ void sy_round_part(u32 w, unsigned char* s_raw) {
    const SyPartArgs* a = sy_karg<SyPartArgs>(0);
    for (u32 t = w; t < a->ntiles; t += SY_FUSED_WG) {
        sy_part_role<CW>(*a, t, *reinterpret_cast<SyPartLds<CW>*>(s_raw));
        __syncthreads();
    }
}
template <int CW>
__global__ __launch_bounds__(SYB_TPB) __attribute__((amdgpu_waves_per_eu(NRG_SYB_WPE))) void sy_round_kernel(
    SyPartArgs A, SyBucketArgs B, SySumArgs S, u32 nblk_b, u32 part_first_below) {
    extern __shared__ __attribute__((aligned(16))) unsigned char s_raw[];
    const u32 w = blockIdx.x;
    (void)A;
    (void)B;
    (void)S;
    // the CU's first workgroup partitions, then replays its bucket; the second the other way
    // round (straight-line code: a loop over the two phases had the compiler hoist each role's
    // lane constants across the other role, and spill)
    if (w < part_first_below) sy_round_part<CW>(w, s_raw);
    {
        const SyBucketArgs* b = sy_karg<SyBucketArgs>(SY_KA_B);
        // (nblk_b <= SY_MAX_NB = SY_FUSED_WG: at most one bucket workgroup each)
        if (w < nblk_b) {
            sy_bucket_role<SYF_PER>(*b, w, nblk_b, *reinterpret_cast<SyBucketLds<SYF_PER>*>(s_raw),
                                    reinterpret_cast<u32*>(s_raw + ((sizeof(SyBucketLds<SYF_PER>) + 15) & ~(size_t)15)));
            __syncthreads();
        }
    }
    if (w >= part_first_below) sy_round_part<CW>(w, s_raw);
    const SySumArgs* sa = sy_karg<SySumArgs>(SY_KA_S);
    for (u32 k = w; k < sa->blocks; k += SY_FUSED_WG) {
        sy_sum_role(*sa, k, reinterpret_cast<SyPartLds<CW>*>(s_raw)->u.sum);
        __syncthreads();
    }
}

static hipError_t sy_launch_fused(nrg_ctx* c, const SyPartArgs& A, const SyDeferred& bd, const SySumArgs& S) {
    const nrg_config& cf = c->cfg;
    SyBucketArgs B{};
    u32 nblk_b = 0;
    size_t dyn_b = 0;
    if (bd.valid) {
        B = sy_bucket_args(c, bd);
        nblk_b = B.NB + SY_B0_PARTS - 1;
        dyn_b = ((sizeof(SyBucketLds<SYF_PER>) + 15) & ~(size_t)15) + sy_bucket_dyn_bytes(B.ntiles);
    }
    hipStream_t st = c->stream;
    // the first of each CU's two workgroups (0 .. 255, one per CU) partitions first (A/B, NRG_KNOB_EXP
    // bit 12: every workgroup partitions first; bit 13: every workgroup replays its bucket first)
    const u32 pfb = (c->exp & 0x1000) ? SY_FUSED_WG : (c->exp & 0x2000) ? 0u : SY_FUSED_WG / 2;
#define SY_FUSED(CWV)                                                                                      \
    case CWV: {                                                                                            \
        const size_t dyn = std::max(sizeof(SyPartLds<CWV>), dyn_b);                                        \
        if (dyn > 65536) {                                                                                 \
            hipError_t e_ = hipFuncSetAttribute((const void*)sy_round_kernel<CWV>,                         \
                                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);     \
            if (e_ != hipSuccess) return e_;                                                               \
        }                                                                                                  \
        sy_round_kernel<CWV><<<SY_FUSED_WG, SYB_TPB, dyn, st>>>(A, B, S, nblk_b, pfb);                     \
        break;                                                                                             \
    }
    switch (cf.synth_cold_writes) {
        SY_FUSED(1); SY_FUSED(2); SY_FUSED(3); SY_FUSED(4); SY_FUSED(5); SY_FUSED(6); SY_FUSED(7); SY_FUSED(8);
        default: return hipErrorInvalidValue;
    }
#undef SY_FUSED
    return hipGetLastError();
}

static hipError_t sy_launch_bucket(nrg_ctx* c, const SyDeferred& d) {
    const SyBucketArgs B = sy_bucket_args(c, d);
    sy_bucket_kernel<<<B.NB + SY_B0_PARTS - 1, SYB_TPB, sy_bucket_dyn_bytes(B.ntiles), c->stream>>>(B);
    return hipGetLastError();
}

// The deferred work of the last replayed chunks, if any: the sums (and hot-word fold) of the
// last chunk; with one launch per round also the bucket pass of the last chunk, then its sums.
hipError_t sy_flush(nrg_ctx* c) {
    if (c->sy_fused) {
        while (c->sy_pend_b.valid || c->sy_pend.valid) {
            const SySumArgs S = sy_sum_args(c, c->sy_pend);
            SyPartArgs A{};
            hipError_t e = sy_launch_fused(c, A, c->sy_pend_b, S);
            if (e != hipSuccess) return e;
            c->sy_pend = c->sy_pend_b;  // its sums next
            c->sy_pend_b.valid = false;
        }
        return hipSuccess;
    }
    if (!c->sy_pend.valid) return hipSuccess;
    const SySumArgs S = sy_sum_args(c, c->sy_pend);
    c->sy_pend.valid = false;
    SyPartArgs A{};
    return sy_launch_part(c, A, S);
}

static hipError_t sy_bucket_chunk(nrg_ctx* c, u64 lo, u64 n, u64 resp_lo, u64 resp_hi, u64* d_resp, uint8_t* d_some,
                                  const nrg_synth_op* src) {
    const u32 epoch = ++c->sy_round;
    const SyPartArgs A = sy_part_args(c, lo, n, src, epoch);
    SyDeferred d;
    d.valid = true;
    d.epoch = epoch;
    d.lo = lo;
    d.n = n;
    d.ntiles = A.ntiles;
    d.want = d_resp != nullptr && resp_lo < lo + n && resp_hi > lo;
    d.t0 = 0;
    d.t1 = 1;
    if (d.want) {
        const u64 a = resp_lo > lo ? resp_lo - lo : 0;
        const u64 z = resp_hi < lo + n ? resp_hi - lo : n;
        d.t0 = (u32)(a / SYA_OPS);
        d.t1 = (u32)((z + SYA_OPS - 1) / SYA_OPS);
    }
    d.rlo = resp_lo;
    d.rhi = resp_hi;
    d.resp = d.want ? d_resp : nullptr;
    d.some = d.want ? d_some : nullptr;
    const SySumArgs S = sy_sum_args(c, c->sy_pend);
    hipError_t e;
    timer_begin(c, "sy_replay");
    if (c->sy_fused) {
        // one launch: this chunk's partition, the last chunk's bucket pass, the one before's sums
        e = sy_launch_fused(c, A, c->sy_pend_b, S);
        timer_end(c, "sy_replay");
        if (e != hipSuccess) return e;
        c->sy_pend = c->sy_pend_b;
        c->sy_pend_b = d;
    } else {
        // two launches: this chunk's partition beside the last chunk's sums, then its bucket pass
        e = sy_launch_part(c, A, S);
        if (e == hipSuccess) e = sy_launch_bucket(c, d);
        timer_end(c, "sy_replay");
        if (e != hipSuccess) return e;
        c->sy_pend = d;
    }
    return c->pipeline ? hipSuccess : sy_flush(c);
}

// nrg_test_lds_add_order: the property the synthetic rankings rest on. Each wave, per trial, issues five
// returning adds over K packed u16 counts (as the partition does) with keys from a hash, and
// compares every lane's old value with the count before the instruction plus the lower lanes of
// the same key. out[0] += lanes checked, out[1] += lanes out of lane order.
__global__ __launch_bounds__(512) void sy_lds_add_order_kernel(u32 K, u32 trials, u64* out) {
    __shared__ unsigned short cnt[8][512];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    u64 nbad = 0, nchk = 0;
    for (u32 t = 0; t < trials; t++) {
        for (int i = lane; i < 512; i += 64) cnt[w][i] = 0;
        wave_lds_sync();
        for (int r = 0; r < 5; r++) {
            const u32 key = (u32)(mix64(((u64)blockIdx.x << 40) ^ ((u64)t << 20) ^ (u64)(r * 4096 + w * 64 + lane)) % K);
            u32 before = 0;
            for (int l = 0; l < 64; l++) {
                const u32 kl = (u32)__shfl((int)key, l, 64);  // every lane takes part (a source lane must be active)
                before += (l < lane && kl == key) ? 1u : 0u;
            }
            const u32 prior = cnt[w][key];
            wave_lds_sync();
            const u32 sh = (key & 1u) * 16u;
            const u32 old = (atomicAdd((u32*)&cnt[w][key & ~1u], 1u << sh) >> sh) & 0xFFFFu;
            wave_lds_sync();
            nbad += old != prior + before ? 1u : 0u;
            nchk++;
        }
    }
    atomicAdd((unsigned long long*)&out[0], (unsigned long long)nchk);
    atomicAdd((unsigned long long*)&out[1], (unsigned long long)nbad);
}

hipError_t sy_lds_add_order(nrg_ctx* c, u32 K, u32 trials, u32 blocks, u64* d_out) {
    if (K < 1 || K > 512) return hipErrorInvalidValue;
    sy_lds_add_order_kernel<<<blocks, 512, 0, c->stream>>>(K, trials, d_out);
    return hipGetLastError();
}

hipError_t sy_init(nrg_ctx* c) {
    sy_init_kernel<<<1024, 256, 0, c->stream>>>(c->d_words, c->cfg.synth_n);
    return hipGetLastError();
}


hipError_t sy_replay_chunk(nrg_ctx* c, u64 lo, u64 n, u64 resp_lo, u64 resp_hi, u64* d_resp, uint8_t* d_some,
                           const nrg_synth_op* src) {
    if (n == 0) return sy_flush(c);  // an empty round still completes the last round's deferred sums
    if (c->d_sy_aux) return sy_bucket_chunk(c, lo, n, resp_lo, resp_hi, d_resp, d_some, src);
    if (src) {  // the sort path replays from the ring: append the ops first (wrapping)
        const u64 mask = c->log_size - 1, first = std::min<u64>(n, c->log_size - (lo & mask));
        nrg_synth_op* ring = (nrg_synth_op*)c->d_ring;
        hipError_t e = hipMemcpyAsync(ring + (lo & mask), src, first * sizeof(nrg_synth_op), hipMemcpyDeviceToDevice,
                                      c->stream);
        if (e == hipSuccess && first < n)
            e = hipMemcpyAsync(ring, src + first, (n - first) * sizeof(nrg_synth_op), hipMemcpyDeviceToDevice,
                               c->stream);
        if (e != hipSuccess) return e;
    }
    hipStream_t st = c->stream;
    const nrg_config& cf = c->cfg;
    const u32 HW = cf.synth_hot_writes, CW = cf.synth_cold_writes, HR = cf.synth_hot_reads;
    const u32 T = HW + CW;
    const u64 nt = n * T;
    const u64 ring_mask = c->log_size - 1;
    const nrg_synth_op* ring = (const nrg_synth_op*)c->d_ring;
    const u32 sentinel = (u32)((1ull << c->synth_key_bits) - 1);
    u32* keys = (u32*)c->d_tmp_u64;
    u32* vals = keys + (u64)cf.max_batch * T;
    u32* M = (u32*)c->d_sort_aux;
    hipError_t e;
    const bool want = d_resp != nullptr && resp_lo < lo + n && resp_hi > lo;
    if (want) {
        const u64 a = resp_lo > lo ? resp_lo : lo;
        const u64 b = resp_hi < lo + n ? resp_hi : lo + n;
        if ((e = hipMemsetAsync(d_resp + (a - resp_lo), 0, (b - a) * sizeof(u64), st)) != hipSuccess) return e;
        if (d_some && (e = hipMemsetAsync(d_some + (a - resp_lo), 1, b - a, st)) != hipSuccess) return e;
    }
    timer_begin(c, "sy_replay");
    u64 g = (n + 255) / 256;
    if (g > 8192) g = 8192;
    sy_expand_kernel<<<(unsigned)g, 256, 0, st>>>(ring, ring_mask, lo, n, cf.synth_n, HR, HW, CW, sentinel, keys, vals);
    u32 *sk = nullptr, *sv = nullptr;
    if ((e = sort_pairs(c->sort, keys, vals, nt, (int)c->synth_key_bits, st, &sk, &sv)) != hipSuccess) return e;
    const u64 tiles = (nt + MS_TILE - 1) / MS_TILE;
    if ((e = hipMemsetAsync(c->d_scan_desc, 0, (32 + tiles) * sizeof(u64), st)) != hipSuccess) return e;
    sy_maxscan_kernel<<<(unsigned)tiles, MS_TPB, 0, st>>>(sk, sv, nt, (u64*)c->d_scan_desc + 32, c->d_scan_desc, M);
    const unsigned gb = (unsigned)((nt + 255) / 256);
    if (want)
        sy_resolve_kernel<<<gb, 256, 0, st>>>(sk, sv, M, nt, ring, ring_mask, lo, c->d_words, HW, T, sentinel, resp_lo,
                                             resp_hi, d_resp);
    sy_commit_kernel<<<gb, 256, 0, st>>>(sk, sv, M, nt, ring, ring_mask, lo, c->d_words, T, sentinel);
    timer_end(c, "sy_replay");
    return hipGetLastError();
}

hipError_t sy_maxscan(nrg_ctx* c, const u32* sk, const u32* sv, u64 n, u32* M) {
    const u64 tiles = (n + MS_TILE - 1) / MS_TILE;
    hipError_t e = hipMemsetAsync(c->d_scan_desc, 0, (32 + tiles) * sizeof(u64), c->stream);
    if (e != hipSuccess) return e;
    sy_maxscan_kernel<<<(unsigned)tiles, MS_TPB, 0, c->stream>>>(sk, sv, n, (u64*)c->d_scan_desc + 32,
                                                                c->d_scan_desc, M);
    return hipGetLastError();
}

hipError_t sy_read(nrg_ctx* c, const nrg_synth_rd* d_ops, u64 n, u64* d_sums) {
    if (n == 0) return hipSuccess;
    hipError_t e = sy_flush(c);  // reads see the hot words of every replayed chunk
    if (e != hipSuccess) return e;
    const nrg_config& cf = c->cfg;
    sy_read_kernel<<<(unsigned)((n + 255) / 256), 256, 0, c->stream>>>(
        d_ops, n, c->d_words, cf.synth_n, cf.synth_hot_reads, cf.synth_hot_writes, cf.synth_cold_reads, d_sums);
    return hipGetLastError();
}

}  // namespace nrg
