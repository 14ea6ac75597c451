// stack.hip — Stack replica replay on gfx950 (benches/stack.rs:36-84, nr/tests/stack.rs:31-96).
//
// Vec<u32>::push/pop in log order, with pop on an empty stack returning None and leaving
// the depth at 0. Each op is the function f(x) = max(a, x + b) of the depth before it
// (Push: b=+1, a=1; Pop: b=-1, a=0); these compose associatively
//      (f then g) = (b_f + b_g, max(a_g, a_f + b_g)),
// so the depth before every op is an exclusive scan (one pass, decoupled look-back).
//
// A Push at depth d writes slot d; a Pop at depth d > 0 reads slot d-1. Because the depth
// moves by ±1, the touches of one slot (crossings of the edge (s, s+1)) alternate Push/Pop in
// log order. No global sort is needed to pair them:
//   * inside a tile of 2048 ops, sorting the tile's touches by (slot, position) in LDS puts
//     every Pop right after the Push it returns, unless the Pop heads its slot's group;
//   * a Pop that heads its group started its tile above the slot, so its Push is the last
//     Push to that slot in the NEAREST EARLIER TILE WHOSE MINIMUM DEPTH IS <= the slot (every
//     tile in between stayed above the slot and so never touched it; that tile went at or below
//     the slot and ended above it, so its last op on the slot was a Push) — or, with no such
//     tile, the slot's content before the chunk.
// Each tile publishes its minimum depth and a table "last Push to slot tmin + r" (u16
// positions), so the cross-tile Pops (a few percent for random ops) walk back over tile minima
// only. The chunk's final content of a slot s below the final depth is its last Push, which
// lies in the LAST tile whose minimum depth is <= s (the walk never comes back down to s after
// it); that tile's table already holds it, so st_finish_kernel commits, per tile, the levels
// [tmin, min(tile end depth, minimum depth of every later tile)).
//
// Kernels: st_tile_kernel (scan + in-tile pairing + tables), st_finish_kernel (cross-tile
// Pops, last Pushes -> stack, depth update).
#include "internal.hpp"

namespace nrg {

constexpr int ST_TPB = 256;
constexpr int ST_ITEMS = 8;
constexpr int ST_TILE = ST_TPB * ST_ITEMS;  // 2048 ops: positions and relative slots fit 11 bits
constexpr uint16_t ST_NO_PUSH = 0xFFFFu;

struct Fn {
    long long b;
    long long a;
};
__device__ __forceinline__ Fn fn_then(Fn f, Fn g) {  // apply f, then g
    Fn r;
    r.b = f.b + g.b;
    const long long t = f.a + g.b;
    r.a = g.a > t ? g.a : t;
    return r;
}
__device__ __forceinline__ long long fn_apply(Fn f, long long x) {
    const long long t = x + f.b;
    return f.a > t ? f.a : t;
}

constexpr u64 D_AGG = 1ull << 62;
constexpr u64 D_MASK = 3ull << 62;

// identity of fn_then (a = -infinity for max(a, x + b))
constexpr Fn FN_ID = {0, -(1ll << 50)};

// Compose the 64 lanes' functions in tile order, oldest (highest lane) applied first:
// result = f_63 then f_62 ... then f_0, broadcast to every lane.
__device__ __forceinline__ Fn wave_compose(Fn f) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
        Fn o;
        o.b = __shfl_down(f.b, s, 64);
        o.a = __shfl_down(f.a, s, 64);
        if ((lane & (2 * s - 1)) == 0 && lane + s < 64) f = fn_then(o, f);
    }
    Fn r;
    r.b = __shfl(f.b, 0, 64);
    r.a = __shfl(f.a, 0, 64);
    return r;
}

__device__ __forceinline__ u64 pack_agg(Fn f) {
    return D_AGG | ((u64)(f.b + (1ll << 30)) << 31) | (u64)f.a;
}
__device__ __forceinline__ Fn unpack_agg(u64 v) {
    Fn f;
    f.a = (long long)(v & ((1ull << 31) - 1));
    f.b = (long long)((v >> 31) & ((1ull << 31) - 1)) - (1ll << 30);
    return f;
}

// Per-tile results of st_tile_kernel, read by st_cross_kernel.
struct StTiles {
    long long* tmin;   // [tiles] minimum depth reached in the tile (start and end included)
    u32* tend;         // [tiles] end depth of the tile - tmin
    u32* table;        // [tiles][ST_TILE] value of the tile's last Push to slot tmin + r, for the
                       // slots below the tile's end depth (the only ones ever looked up)
    u32* ucnt;         // [tiles] Pops whose Push is outside the tile
    u32* upop;         // [tiles][ST_TILE] those Pops: (slot - tmin) << 11 | position
    u32* uval;         // [tiles][ST_TILE] their slot's content before the chunk (if below it)
};

__device__ __forceinline__ long long block_min4(long long x, long long* s_w, int w, int lane) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const long long o = __shfl_xor(x, off, 64);
        x = o < x ? o : x;
    }
    if (lane == 0) s_w[w] = x;
    __syncthreads();
    long long m = s_w[0];
    for (int i = 1; i < 4; i++) m = s_w[i] < m ? s_w[i] : m;
    return m;
}

constexpr u32 ST_INF = 0xFFFFu;

// src: the chunk's records in a caller buffer (nrg_stack_round_async); the kernel then writes
// the log copy itself (Log::append fused into the replay). nullptr: records are in the ring.
__global__ __launch_bounds__(ST_TPB) void st_tile_kernel(const nrg_stack_op* __restrict__ src, nrg_stack_op* ring,
                                                         u64 ring_mask, u64 lo,
                                                         u64 n, DevCtl* ctl, u64* desc, u32* ticket, StTiles tl,
                                                         const u32* __restrict__ stack,
                                                         u64 cap, u64 resp_lo, u64 resp_hi, int push_resp,
                                                         u32* __restrict__ resp, uint8_t* __restrict__ some, u32 exp,
                                                         u64* __restrict__ dbg) {
#define ST_MARK(K) \
    if (dbg && threadIdx.x == 0) dbg[(u64)blockIdx.x * 16 + (K)] = wall_clock64()
    ST_MARK(0);
    __shared__ long long s_wb[4], s_wa[4], s_wmin[4];
    __shared__ u32 s_tile, s_ucnt, s_aend;
    __shared__ long long s_dbase;
    __shared__ u32 s_val[ST_TILE];             // op values by position
    __shared__ uint16_t s_A[ST_TILE + 1];      // depth after op i (- tmin) at [i + 1]; [0] = start
    // sparse min table over the threads' minima: s_sp[j][k] = min of threads (k - 2^j, k]
    __shared__ uint16_t s_sp[9][ST_TPB];
    __shared__ uint16_t s_sw[4];               // per wave: minimum of its threads
    __shared__ uint16_t s_tab[ST_TILE];        // last Push position per relative slot
    __shared__ u32 s_q[4][ST_ITEMS * 64];      // per wave: Pops answered beyond their thread
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (t == 0) {
        s_tile = (exp & 1) ? blockIdx.x : atomicAdd(ticket, 1u);  // exp 1: diagnostic only
        s_ucnt = 0;
    }
    __syncthreads();
    ST_MARK(1);
    const u32 tile = s_tile;
    const u64 tbase = (u64)tile * ST_TILE;
    const u64 base = tbase + (u64)t * ST_ITEMS;
    const long long d0 = ctl->depth;  // depth before the chunk (st_commit_kernel updates it)

    nrg_stack_op ops[ST_ITEMS];
    Fn agg = {0, 0};
#pragma unroll
    for (int q = 0; q < ST_ITEMS; q++) {
        const u64 i = base + q;
        if (i < n) {
            ops[q] = src ? src[i] : ring[(lo + i) & ring_mask];
            Fn f;
            f.b = ops[q].op ? 1 : -1;
            f.a = ops[q].op ? 1 : 0;
            agg = fn_then(agg, f);
        } else {
            ops[q].op = 2;  // padding
            ops[q].val = 0;
        }
    }
    if (src) {  // the log copy, lane-contiguous (the loads above are 8 records per thread)
        for (u32 k = t; k < ST_TILE; k += ST_TPB) {
            const u64 i = tbase + k;
            if (i < n) ring[(lo + i) & ring_mask] = src[i];
        }
    }
    // wave inclusive scan of thread aggregates (order matters)
    Fn inc = agg;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        Fn o;
        o.b = __shfl_up(inc.b, off, 64);
        o.a = __shfl_up(inc.a, off, 64);
        if (lane >= off) inc = fn_then(o, inc);
    }
    if (lane == 63) {
        s_wb[w] = inc.b;
        s_wa[w] = inc.a;
    }
    // exclusive within wave
    Fn ex;
    ex.b = __shfl_up(inc.b, 1, 64);
    ex.a = __shfl_up(inc.a, 1, 64);
    if (lane == 0) ex = Fn{0, 0};
    __syncthreads();
    Fn wpre = {0, 0};
    for (int i = 0; i < w; i++) wpre = fn_then(wpre, Fn{s_wb[i], s_wa[i]});
    ST_MARK(2);
    const Fn tpre = fn_then(wpre, ex);
    Fn tagg = {0, 0};
    for (int i = 0; i < 4; i++) tagg = fn_then(tagg, Fn{s_wb[i], s_wa[i]});
    if (t == 0) __hip_atomic_store(&desc[tile], pack_agg(tagg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // Pass 0 pairs the tile speculatively on the UNCLAMPED walk relative to the tile's start:
    // Push/Pop pairing depends only on relative depths, and it is the real pairing unless the
    // stack runs empty inside the tile (a Pop at depth 0 is a no-op). Whether it does needs the
    // tile's start depth, i.e. the look-back, which therefore runs after pass 0 and finds its
    // predecessors' aggregates already published. Pass 1 (a stack within 2048 of empty) redoes
    // the pairing on the clamped walk from the known start depth.
    long long dstart = tpre.b;
    bool clamp = false;
    long long tmin = 0;   // minimum of the walk, start and end included (pass 0: relative)
    u32 a[ST_ITEMS];      // depth after each of this thread's ops - tmin
    u32 astart = 0;       // depth before this thread's first op - tmin
    u32 rv[ST_ITEMS];     // response per op:
    uint8_t rk[ST_ITEMS]; //   0 none (padding, or queued below), 1 Some(rv), 2 None
    u32 qe[ST_ITEMS], qv[ST_ITEMS];  // queued Pops this lane resolved: entry and value,
    bool qx[ST_ITEMS];               //   or outside the tile (qx)
    u32 qn = 0;                      // wave-uniform queue length
    for (int pass = 0;; pass++) {
        long long dd = dstart, dmin = dd;
#pragma unroll
        for (int q = 0; q < ST_ITEMS; q++) {
            if (ops[q].op == 1) dd += 1;
            else if (ops[q].op == 0 && (!clamp || dd > 0)) dd -= 1;
            dmin = dd < dmin ? dd : dmin;
        }
        tmin = block_min4(dmin, s_wmin, w, lane);
        ST_MARK(3);
        u32 amin = ST_INF;
        dd = dstart;
#pragma unroll
        for (int q = 0; q < ST_ITEMS; q++) {
            if (ops[q].op == 1) dd += 1;
            else if (ops[q].op == 0 && (!clamp || dd > 0)) dd -= 1;
            a[q] = (u32)(dd - tmin);
            amin = a[q] < amin ? a[q] : amin;
            s_A[t * ST_ITEMS + q + 1] = (uint16_t)a[q];
            s_val[t * ST_ITEMS + q] = ops[q].val;
        }
        astart = (u32)(dstart - tmin);
        if (t == 0) s_A[0] = (uint16_t)astart;
        s_sp[0][t] = (uint16_t)amin;
        // suffix minimum over the threads after this one (exclusive), for the last-Push records
        u32 sfx = amin;  // inclusive suffix min within the wave
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const u32 o = __shfl_down(sfx, off, 64);
            if (lane + off < 64) sfx = o < sfx ? o : sfx;
        }
        if (lane == 0) s_sw[w] = (uint16_t)sfx;
        for (int r = t; r < ST_TILE; r += ST_TPB) s_tab[r] = ST_NO_PUSH;
        __syncthreads();
        {
            u32 m = amin;
#pragma unroll
            for (int j = 1; j < 9; j++) {
                const int h = 1 << (j - 1);
                if (t >= h) {
                    const u32 o = s_sp[j - 1][t - h];
                    m = o < m ? o : m;
                }
                s_sp[j][t] = (uint16_t)m;
                __syncthreads();
            }
        }
        ST_MARK(4);
        u32 after = __shfl_down(sfx, 1, 64);  // min over later threads in the wave
        if (lane == 63) after = ST_INF;
        for (int i = w + 1; i < 4; i++) after = s_sw[i] < after ? s_sw[i] : after;

        // Last Push to each slot below the tile's end depth: after the last time the walk is at
        // (or below) a level it pushes that level, i.e. at i + 1 for every suffix-record low i.
        {
            u32 cur = after;
            const bool lastthr = t == ST_TPB - 1;
#pragma unroll
            for (int q = ST_ITEMS - 1; q >= 0; q--) {
                const bool final = lastthr && q == ST_ITEMS - 1;  // nothing follows position 2047
                if (!final && a[q] < cur) s_tab[a[q]] = (uint16_t)(t * ST_ITEMS + q + 1);
                cur = a[q] < cur ? a[q] : cur;
            }
            if (t == 0 && astart < cur) s_tab[astart] = 0;
        }

        // Each Pop returns the Push right after the last earlier position whose depth is <= the
        // depth the Pop leaves (a previous-smaller-or-equal query over the tile). Pops that the
        // thread cannot answer from its own ops are queued per wave and answered with all lanes.
        u32 prv = astart;
        qn = 0;
#pragma unroll
        for (int q = 0; q < ST_ITEMS; q++) {
            const u32 pos = (u32)(t * ST_ITEMS + q);
            const bool pop = ops[q].op == 0 && prv > a[q];  // a non-empty Pop (empty: depth stays 0)
            rk[q] = 0;
            rv[q] = 0;
            if (ops[q].op == 0 && !pop) {
                rk[q] = 2;  // Pop on an empty stack: None
            } else if (ops[q].op == 1) {
                rk[q] = push_resp ? 1 : 2;
                rv[q] = ops[q].val;
            }
            bool need = false;
            if (pop) {
                const u32 s = a[q];
                int r = astart <= s ? t * ST_ITEMS - 1 : -2;
#pragma unroll
                for (int qq = 0; qq < ST_ITEMS; qq++)
                    if (qq < q && a[qq] <= s) r = t * ST_ITEMS + qq;
                if (r != -2) {
                    rk[q] = 1;
                    rv[q] = s_val[r + 1];
                } else {
                    need = true;
                }
            }
            const u64 m = __ballot(need);
            if (need) s_q[w][qn + __popcll(m & ((1ull << lane) - 1))] = (a[q] << 11) | pos;
            qn += (u32)__popcll(m);
            prv = a[q];
        }
        __syncthreads();
        ST_MARK(5);
#pragma unroll
        for (int j = 0; j < ST_ITEMS; j++) {
            const u32 i = (u32)lane + 64u * j;
            if (i >= qn) continue;
            const u32 e = s_q[w][i];
            const u32 s = e >> 11, pos = e & 2047u;
            // nearest earlier thread whose minimum is <= s: binary lifting, 9 steps
            int k = (int)(pos / ST_ITEMS) - 1;
            int r = -2;
#pragma unroll
            for (int jj = 8; jj >= 0; jj--)
                if (k >= 0 && s_sp[jj][k] > s) k -= 1 << jj;
            if (k >= 0) {
                u32 v[ST_ITEMS];
#pragma unroll
                for (int qq = 0; qq < ST_ITEMS; qq++) v[qq] = s_A[k * ST_ITEMS + qq + 1];
#pragma unroll
                for (int qq = 0; qq < ST_ITEMS; qq++)
                    if (v[qq] <= s) r = k * ST_ITEMS + qq;
            } else if (s_A[0] <= s) {
                r = -1;
            }
            qe[j] = e;
            qx[j] = r == -2;  // the Push is in an earlier tile or before the chunk
            qv[j] = r == -2 ? 0u : s_val[r + 1];
        }
        ST_MARK(6);
        if (pass == 1) break;

        if (w == 0) {
            // Wave 0 composes the aggregates of ALL earlier tiles itself (64 per wave
            // instruction, every load of a group in flight at once) instead of waiting for an
            // inclusive prefix to ripple down the chain of tiles. Lane l composes the run of
            // predecessors [r*G, r*G + G), r = 63 - l, in registers (older first); one wave
            // composition then joins the runs (the highest lane holds the oldest).
            const int np = (int)tile;
            const int G = (np + 63) / 64;
            const int r0 = (63 - lane) * G;
            Fn acc = FN_ID;
            constexpr int B = 8;  // descriptor loads in flight per lane
            for (int g0 = 0; g0 < G; g0 += B) {
                u64 v[B];
#pragma unroll
                for (int q = 0; q < B; q++) {
                    const int idx = r0 + g0 + q;
                    v[q] = (g0 + q < G && idx < np)
                               ? __hip_atomic_load(&desc[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : 0ull;
                }
#pragma unroll
                for (int q = 0; q < B; q++) {
                    const int idx = r0 + g0 + q;
                    if (g0 + q >= G || idx >= np) continue;
                    u32 spins = 0;
                    while (!(v[q] & D_MASK)) {  // not published yet (its tile is still loading)
                        __builtin_amdgcn_s_sleep(1);
                        v[q] = __hip_atomic_load(&desc[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (++spins == (1u << 26)) {  // bounded: never hang the device
                            atomicOr(&ctl->err, ERR_CAPACITY);
                            break;
                        }
                    }
                    acc = fn_then(acc, unpack_agg(v[q]));
                }
            }
            acc = np ? wave_compose(acc) : Fn{0, 0};
            const long long dbase = fn_apply(acc, d0);
            if (lane == 0) {
                const u64 ntiles = (n + ST_TILE - 1) / ST_TILE;
                if ((u64)tile == ntiles - 1) {
                    ctl->depth_next = fn_apply(tagg, dbase);
                    ctl->depth0 = d0;
                }
                s_dbase = dbase;
            }
        }
        __syncthreads();
        ST_MARK(7);
        const long long D = s_dbase;  // depth before the tile
        if (D + tmin >= 0) {          // the walk never reaches an empty stack: pass 0 holds
            tmin += D;
            break;
        }
        dstart = fn_apply(tpre, D);
        clamp = true;
    }

    // Responses, the capacity check, cross-tile Pops (with the slot's pre-chunk content: no
    // tile writes the stack before st_finish_kernel), then the last-Push table.
    {
        bool over = false;
        u32 prv = astart;
#pragma unroll
        for (int q = 0; q < ST_ITEMS; q++) {
            const u64 g = lo + tbase + (u64)(t * ST_ITEMS + q);
            over |= ops[q].op == 1 && (u64)(tmin + (long long)prv) >= cap;
            if (rk[q] && g >= resp_lo && g < resp_hi) {
                resp[g - resp_lo] = rk[q] == 1 ? rv[q] : 0u;
                some[g - resp_lo] = rk[q] == 1 ? 1 : 0;
            }
            prv = a[q];
        }
        if (over) atomicOr(&ctl->err, ERR_CAPACITY);
#pragma unroll
        for (int j = 0; j < ST_ITEMS; j++) {
            const u32 i = (u32)lane + 64u * j;
            if (i >= qn) continue;
            const u32 e = qe[j];
            const u64 g = lo + tbase + (e & 2047u);
            if (qx[j]) {
                const u32 h = atomicAdd(&s_ucnt, 1u);
                const long long slot = tmin + (long long)(e >> 11);
                tl.upop[(u64)tile * ST_TILE + h] = e;
                tl.uval[(u64)tile * ST_TILE + h] = slot < d0 && (u64)slot < cap ? stack[slot] : 0u;
            } else if (g >= resp_lo && g < resp_hi) {
                resp[g - resp_lo] = qv[j];
                some[g - resp_lo] = 1;
            }
        }
    }
    if (t == ST_TPB - 1) s_aend = a[ST_ITEMS - 1];
    __syncthreads();
    // Levels [tmin, end depth) each have a last Push (suffix records); no other level has one.
    u32* tab = tl.table + (u64)tile * ST_TILE;
    for (u32 r = t; r < s_aend; r += ST_TPB) tab[r] = s_val[s_tab[r]];
    if (t == 0) {
        tl.tmin[tile] = tmin;
        tl.tend[tile] = s_aend;
        tl.ucnt[tile] = s_ucnt;
    }
    ST_MARK(8);
#undef ST_MARK
}

// One block per tile after st_tile_kernel. Every block stages all tile minima in LDS (with the
// minimum of every 8- and 64-tile group) and then
//   * commits: the tile's levels [tmin, min(end depth, min of every later tile's minimum)) are
//     the slots whose last Push of the chunk is this tile's, held in its table;
//   * resolves the tile's Pops whose Push lies in an earlier tile: the nearest earlier tile
//     whose minimum is <= the slot (a walk that skips 8- and 64-tile groups whose minimum is
//     above the slot), or the pre-chunk content st_tile_kernel read.
// Block 0 publishes the new depth.
__global__ __launch_bounds__(256) void st_finish_kernel(u64 lo, u64 n, DevCtl* ctl, StTiles tl,
                                                        u32* __restrict__ stack, u64 cap, u64 resp_lo, u64 resp_hi,
                                                        u32* __restrict__ resp, uint8_t* __restrict__ some,
                                                        u64* desc, u32* ticket) {
    extern __shared__ long long s_tm[];  // [tiles] tile minima, [tiles/8 + 1] and [tiles/64 + 1] group minima
    __shared__ long long s_lo[4];
    const u32 tiles = gridDim.x;
    const u32 tile = blockIdx.x;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    // independent loads first: they overlap the staging below
    const u32 cnt = resp ? tl.ucnt[tile] : 0u;
    const u32 v0 = tl.upop[(u64)tile * ST_TILE + t];
    const u32 uv0 = tl.uval[(u64)tile * ST_TILE + t];
    const u32 tend = tl.tend[tile];
    if (t == 0) desc[tile] = 0;  // ready for the next chunk (the tile kernel is done)
    if (tile == 0 && t == 0) *ticket = 0;
    const u32 ngr = (tiles + 63) / 64;
    long long* s_g8 = s_tm + tiles;
    long long* s_gm = s_g8 + tiles / 8 + 1;
    long long later = 1ll << 62;  // minimum over the tiles after this one
    for (u32 k = t; k < ngr * 64; k += 256) {
        const long long v = k < tiles ? tl.tmin[k] : (1ll << 62);
        if (k < tiles) s_tm[k] = v;
        if (k > tile) later = v < later ? v : later;
        long long m = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const long long x = __shfl_xor(m, off, 64);
            m = x < m ? x : m;
            if (off == 4 && (lane & 7) == 0 && (k >> 3) <= tiles / 8) s_g8[k >> 3] = m;
        }
        if (lane == 0) s_gm[k >> 6] = m;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const long long x = __shfl_xor(later, off, 64);
        later = x < later ? x : later;
    }
    if (lane == 0) s_lo[w] = later;
    __syncthreads();
    if (tile == 0 && t == 0) ctl->depth = ctl->depth_next;
    {
        for (int i = 0; i < 4; i++) later = s_lo[i] < later ? s_lo[i] : later;
        const long long tm = s_tm[tile];
        long long hi = tm + (long long)tend;
        hi = hi < later ? hi : later;
        const u32* tab = tl.table + (u64)tile * ST_TILE;
        for (long long sl = tm + t; sl < hi; sl += 256)
            if ((u64)sl < cap) stack[sl] = tab[sl - tm];
    }
    const long long tmin = s_tm[tile];
    for (u32 j = t; j < cnt; j += 256) {
        const u32 v = j == (u32)t ? v0 : tl.upop[(u64)tile * ST_TILE + j];
        const u64 g = lo + (u64)tile * ST_TILE + (v & 2047u);
        if (g < resp_lo || g >= resp_hi) continue;
        const long long s = tmin + (v >> 11);
        int k = (int)tile - 1;
        while (k >= 0) {
            if ((k & 63) == 63 && s_gm[k >> 6] > s) {
                k -= 64;
                continue;
            }
            if ((k & 7) == 7 && s_g8[k >> 3] > s) {
                k -= 8;
                continue;
            }
            if (s_tm[k] <= s) break;
            k--;
        }
        u32 val;
        if (k >= 0)
            val = tl.table[(u64)k * ST_TILE + (u64)(s - s_tm[k])];
        else
            val = j == (u32)t ? uv0 : tl.uval[(u64)tile * ST_TILE + j];
        resp[g - resp_lo] = val;
        some[g - resp_lo] = 1;
    }
}

hipError_t st_replay_chunk(nrg_ctx* c, u64 lo, u64 n, u64 resp_lo, u64 resp_hi, uint32_t* d_resp, uint8_t* d_some,
                           const nrg_stack_op* src) {
    if (n == 0) return hipSuccess;
    hipStream_t st = c->stream;
    const u64 ring_mask = c->log_size - 1;
    nrg_stack_op* ring = (nrg_stack_op*)c->d_ring;
    const u64 tiles = (n + ST_TILE - 1) / ST_TILE;
    // descriptors: [ticket (64 words of u32 = 32 u64)] [tiles u64]; zero at open, and
    // st_finish_kernel clears what st_tile_kernel used (no memset launch per chunk)
    u64* desc = (u64*)c->d_scan_desc + 32;
    u32* ticket = c->d_scan_desc;
    const u64 mt = (c->cfg.max_batch + ST_TILE - 1) / ST_TILE;
    StTiles tl;
    tl.tmin = (long long*)c->d_st_aux;
    tl.ucnt = (u32*)(tl.tmin + mt);
    tl.tend = tl.ucnt + mt;
    tl.upop = tl.tend + mt;
    tl.uval = tl.upop + mt * ST_TILE;
    tl.table = tl.uval + mt * ST_TILE;
    const bool want = d_resp != nullptr && resp_lo < lo + n && resp_hi > lo;
    const u64 rlo = want ? resp_lo : 0, rhi = want ? resp_hi : 0;
    timer_begin(c, "st_replay");
    st_tile_kernel<<<(unsigned)tiles, ST_TPB, 0, st>>>(src, ring, ring_mask, lo, n, c->d_ctl, desc, ticket, tl,
                                                      c->d_stack, c->cfg.stack_capacity, rlo, rhi,
                                                      (int)c->cfg.stack_push_resp, d_resp, d_some, c->exp,
                                                      (c->exp & 2) ? c->d_dbg : nullptr);
    st_finish_kernel<<<(unsigned)tiles, 256, (tiles + tiles / 8 + tiles / 64 + 2) * 8, st>>>(
        lo, n, c->d_ctl, tl, c->d_stack, c->cfg.stack_capacity, rlo, rhi,
        want ? d_resp : nullptr, d_some, desc, ticket);
    timer_end(c, "st_replay");
    return hipGetLastError();
}

u64 st_aux_bytes(u64 max_batch) {
    const u64 mt = (max_batch + ST_TILE - 1) / ST_TILE;
    return mt * (8 + 4 + 4) + mt * ST_TILE * (4 + 4 + 4);
}

}  // namespace nrg
