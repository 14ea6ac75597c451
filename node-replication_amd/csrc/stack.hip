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
// only. The chunk's final content of a slot is its last Push, picked with one atomicMax per
// (tile, pushed slot) in a window of 2n slots around the chunk's starting depth.
//
// Kernels: st_tile_kernel (scan + LDS bitonic sort + in-tile pairing + tables),
// st_cross_kernel (cross-tile Pops; launched only when responses are wanted),
// st_commit_kernel (last Pushes -> stack, depth update).
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
constexpr u64 D_INC = 2ull << 62;
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
    uint16_t* table;   // [tiles][ST_TILE] position of the tile's last Push to slot tmin + r
    u32* ucnt;         // [tiles] Pops whose Push is outside the tile
    u32* upop;         // [tiles][ST_TILE] those Pops: (slot - tmin) << 11 | position
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

__global__ __launch_bounds__(ST_TPB) void st_tile_kernel(const nrg_stack_op* __restrict__ ring, u64 ring_mask, u64 lo,
                                                         u64 n, DevCtl* ctl, u64* desc, u32* ticket, StTiles tl,
                                                         u32* __restrict__ last, u64 cap, u64 resp_lo, u64 resp_hi,
                                                         int push_resp, u32* __restrict__ resp,
                                                         uint8_t* __restrict__ some) {
    __shared__ long long s_wb[4], s_wa[4], s_wmin[4];
    __shared__ u32 s_tile, s_ucnt;
    __shared__ long long s_dbase;
    __shared__ u32 s_val[ST_TILE];             // op values by position
    __shared__ uint16_t s_A[ST_TILE + 1];      // depth after op i (- tmin) at [i + 1]; [0] = start
    // sparse min table over the threads' minima: s_sp[j][k] = min of threads (k - 2^j, k]
    __shared__ uint16_t s_sp[9][ST_TPB];
    __shared__ uint16_t s_sw[4];               // per wave: minimum of its threads
    __shared__ uint16_t s_tab[ST_TILE];        // last Push position per relative slot
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (t == 0) {
        s_tile = atomicAdd(ticket, 1u);
        s_ucnt = 0;
    }
    __syncthreads();
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
            ops[q] = ring[(lo + i) & ring_mask];
            Fn f;
            f.b = ops[q].op ? 1 : -1;
            f.a = ops[q].op ? 1 : 0;
            agg = fn_then(agg, f);
        } else {
            ops[q].op = 2;  // padding
            ops[q].val = 0;
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
    const Fn tpre = fn_then(wpre, ex);
    if (w == 0) {
        // Wave 0 publishes the tile's aggregate and does the look-back with all 64 lanes:
        // lane l reads tile (tt - l)'s descriptor, so one memory round trip covers 64
        // predecessors.
        Fn tagg = {0, 0};
        for (int i = 0; i < 4; i++) tagg = fn_then(tagg, Fn{s_wb[i], s_wa[i]});
        long long dbase = d0;
        if (tile == 0) {
            if (lane == 0)
                __hip_atomic_store(&desc[0], D_INC | (u64)fn_apply(tagg, dbase), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(&desc[tile], pack_agg(tagg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            Fn acc = FN_ID;  // composition of the predecessors consumed so far (older ones apply first)
            int tt = (int)tile - 1;
            for (;;) {
                const int idx = tt - lane;
                const u64 v = idx >= 0 ? __hip_atomic_load(&desc[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                const u64 st = v & D_MASK;
                const u64 nr = __ballot(st == 0);
                const u64 ic = __ballot(st == D_INC);
                const int first_nr = nr ? __ffsll((unsigned long long)nr) - 1 : 64;
                const int first_ic = ic ? __ffsll((unsigned long long)ic) - 1 : 64;
                const int use = first_ic < first_nr ? first_ic : first_nr;  // aggregates usable now
                const Fn f = lane < use ? unpack_agg(v) : FN_ID;
                acc = fn_then(wave_compose(f), acc);
                if (first_ic < first_nr) {
                    const long long incv = (long long)(__shfl(v, first_ic, 64) & ~D_MASK);
                    dbase = fn_apply(acc, incv);
                    break;
                }
                tt -= use;
                if (use < 64) __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0)
                __hip_atomic_store(&desc[tile], D_INC | (u64)fn_apply(tagg, dbase), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
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

    // Depth after each op, relative to the tile's minimum (start and end included: <= 2048).
    const long long dbase = s_dbase;
    const long long dstart = fn_apply(tpre, dbase);
    long long dd = dstart, dmin = dd;
    bool over = false;
#pragma unroll
    for (int q = 0; q < ST_ITEMS; q++) {
        if (ops[q].op == 1) {
            over |= (u64)dd >= cap;
            dd += 1;
        } else if (ops[q].op == 0 && dd > 0) {
            dd -= 1;
        }
        dmin = dd < dmin ? dd : dmin;
    }
    if (over) atomicOr(&ctl->err, ERR_CAPACITY);
    const long long tmin = block_min4(dmin, s_wmin, w, lane);
    u32 a[ST_ITEMS];  // relative depth after each of this thread's ops
    u32 amin = ST_INF;
    dd = dstart;
#pragma unroll
    for (int q = 0; q < ST_ITEMS; q++) {
        if (ops[q].op == 1) dd += 1;
        else if (ops[q].op == 0 && dd > 0) dd -= 1;
        a[q] = (u32)(dd - tmin);
        amin = a[q] < amin ? a[q] : amin;
        s_A[t * ST_ITEMS + q + 1] = (uint16_t)a[q];
        s_val[t * ST_ITEMS + q] = ops[q].val;
    }
    const u32 astart = (u32)(dstart - tmin);  // relative depth before this thread's first op
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
    // depth the Pop leaves (a previous-smaller-or-equal query over the tile).
    u32 prv = astart;
#pragma unroll
    for (int q = 0; q < ST_ITEMS; q++) {
        const u32 pos = (u32)(t * ST_ITEMS + q);
        const u64 g = lo + tbase + pos;
        const bool inwin = g >= resp_lo && g < resp_hi;
        const bool pop = ops[q].op == 0 && prv > a[q];  // a non-empty Pop (empty: depth stays 0)
        if (ops[q].op == 0 && !pop && inwin) {            // Pop on an empty stack: None
            resp[g - resp_lo] = 0;
            some[g - resp_lo] = 0;
        } else if (ops[q].op == 1 && inwin) {
            resp[g - resp_lo] = push_resp ? ops[q].val : 0u;
            some[g - resp_lo] = push_resp ? 1 : 0;
        }
        if (pop) {
            const u32 s = a[q];
            int r = -2;
#pragma unroll
            for (int qq = 0; qq < ST_ITEMS; qq++)
                if (qq < q && a[qq] <= s) r = t * ST_ITEMS + qq;
            if (r == -2) {
                // nearest earlier thread whose minimum is <= s: binary lifting, 9 steps
                int k = t - 1;
#pragma unroll
                for (int j = 8; j >= 0; j--)
                    if (k >= 0 && s_sp[j][k] > s) k -= 1 << j;
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
            }
            if (r == -2) {  // the Push is in an earlier tile or before the chunk
                const u32 k = atomicAdd(&s_ucnt, 1u);
                tl.upop[(u64)tile * ST_TILE + k] = (s << 11) | pos;
            } else if (inwin) {
                resp[g - resp_lo] = s_val[r + 1];
                some[g - resp_lo] = 1;
            }
        }
        prv = a[q];
    }
    __syncthreads();
    uint16_t* tab = tl.table + (u64)tile * ST_TILE;
    for (int r = t; r < ST_TILE; r += ST_TPB) {
        const uint16_t p = s_tab[r];
        tab[r] = p;
        if (p != ST_NO_PUSH)
            atomicMax(&last[(u64)(tmin + r - d0 + (long long)n)], ((tile << 11) | p) + 1u);
    }
    if (t == 0) {
        tl.tmin[tile] = tmin;
        tl.ucnt[tile] = s_ucnt;
    }
}

// Pops whose Push lies in an earlier tile (or before the chunk). The block stages the minima
// of tiles [0, tile) in LDS with the minimum of every 64-tile group, so a walk back skips a
// group whose minimum is above the slot in one step.
__global__ __launch_bounds__(256) void st_cross_kernel(const nrg_stack_op* __restrict__ ring, u64 ring_mask, u64 lo,
                                                       StTiles tl, const u32* __restrict__ stack, u64 cap,
                                                       u64 resp_lo, u64 resp_hi, u32* __restrict__ resp,
                                                       uint8_t* __restrict__ some) {
    extern __shared__ long long s_tm[];  // [tiles] minima, then [tiles / 64 + 1] group minima
    const u32 tile = blockIdx.x;
    const u32 cnt = tl.ucnt[tile];
    if (cnt == 0) return;
    const int t = threadIdx.x, lane = t & 63;
    const u32 ngr = (tile + 63) / 64;
    long long* s_gm = s_tm + gridDim.x;
    for (u32 k = t; k < ngr * 64; k += 256) {
        long long m = k < tile ? tl.tmin[k] : (1ll << 62);
        if (k < tile) s_tm[k] = m;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const long long x = __shfl_xor(m, off, 64);
            m = x < m ? x : m;
        }
        if (lane == 0) s_gm[k >> 6] = m;
    }
    __syncthreads();
    const long long tmin = tl.tmin[tile];
    for (u32 j = t; j < cnt; j += 256) {
        const u32 v = tl.upop[(u64)tile * ST_TILE + j];
        const u64 g = lo + (u64)tile * ST_TILE + (v & 2047u);
        if (g < resp_lo || g >= resp_hi) continue;
        const long long s = tmin + (v >> 11);
        int k = (int)tile - 1;
        while (k >= 0) {
            if ((k & 63) == 63 && s_gm[k >> 6] > s) {
                k -= 64;
                continue;
            }
            if (s_tm[k] <= s) break;
            k--;
        }
        u32 val;
        if (k >= 0) {
            const u32 pos = tl.table[(u64)k * ST_TILE + (u64)(s - s_tm[k])];
            val = ring[(lo + (u64)k * ST_TILE + pos) & ring_mask].val;
        } else {
            val = (u64)s < cap ? stack[s] : 0u;
        }
        resp[g - resp_lo] = val;
        some[g - resp_lo] = 1;
    }
}

// Slot window [depth0 - n, depth0 + n): write each slot's last Push of the chunk, clear the
// window for the next chunk, and publish the new depth.
__global__ __launch_bounds__(256) void st_commit_kernel(const nrg_stack_op* __restrict__ ring, u64 ring_mask, u64 lo,
                                                        u64 n, DevCtl* ctl, u32* __restrict__ last,
                                                        u32* __restrict__ stack, u64 cap) {
    const long long d0 = ctl->depth0;
    if (blockIdx.x == 0 && threadIdx.x == 0) ctl->depth = ctl->depth_next;
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < 2 * n; i += (u64)gridDim.x * 256) {
        const u32 x = last[i];
        if (!x) continue;
        last[i] = 0;
        const long long slot = (long long)i + d0 - (long long)n;
        if ((u64)slot < cap) stack[slot] = ring[(lo + (u64)((x - 1) >> 11) * ST_TILE + ((x - 1) & 2047u)) & ring_mask].val;
    }
}

hipError_t st_replay_chunk(nrg_ctx* c, u64 lo, u64 n, u64 resp_lo, u64 resp_hi, uint32_t* d_resp, uint8_t* d_some) {
    if (n == 0) return hipSuccess;
    hipStream_t st = c->stream;
    const u64 ring_mask = c->log_size - 1;
    const nrg_stack_op* ring = (const nrg_stack_op*)c->d_ring;
    const u64 tiles = (n + ST_TILE - 1) / ST_TILE;
    // descriptors: [ticket (64 words of u32 = 32 u64)] [tiles u64]
    u64* desc = (u64*)c->d_scan_desc + 32;
    u32* ticket = c->d_scan_desc;
    hipError_t e = hipMemsetAsync(c->d_scan_desc, 0, (32 + tiles) * sizeof(u64), st);
    if (e != hipSuccess) return e;
    const u64 mt = (c->cfg.max_batch + ST_TILE - 1) / ST_TILE;
    StTiles tl;
    tl.tmin = (long long*)c->d_st_aux;
    tl.ucnt = (u32*)(tl.tmin + mt);
    tl.upop = tl.ucnt + mt;
    tl.table = (uint16_t*)(tl.upop + mt * ST_TILE);
    u32* last = (u32*)c->d_tmp_u64;  // 2 * max_batch u32, zero between chunks
    const bool want = d_resp != nullptr && resp_lo < lo + n && resp_hi > lo;
    const u64 rlo = want ? resp_lo : 0, rhi = want ? resp_hi : 0;
    timer_begin(c, "st_replay");
    st_tile_kernel<<<(unsigned)tiles, ST_TPB, 0, st>>>(ring, ring_mask, lo, n, c->d_ctl, desc, ticket, tl, last,
                                                      c->cfg.stack_capacity, rlo, rhi,
                                                      (int)c->cfg.stack_push_resp, d_resp, d_some);
    if (want)
        st_cross_kernel<<<(unsigned)tiles, 256, (tiles + tiles / 64 + 1) * 8, st>>>(ring, ring_mask, lo, tl, c->d_stack, c->cfg.stack_capacity,
                                                        rlo, rhi, d_resp, d_some);
    const u64 cg = (2 * n + 255) / 256;
    st_commit_kernel<<<(unsigned)(cg < 2048 ? cg : 2048), 256, 0, st>>>(ring, ring_mask, lo, n, c->d_ctl, last,
                                                                        c->d_stack, c->cfg.stack_capacity);
    timer_end(c, "st_replay");
    return hipGetLastError();
}

u64 st_aux_bytes(u64 max_batch) {
    const u64 mt = (max_batch + ST_TILE - 1) / ST_TILE;
    return mt * (8 + 4) + mt * ST_TILE * (4 + 2);
}

}  // namespace nrg
