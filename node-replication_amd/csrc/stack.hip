// stack.hip — Stack replica replay on gfx950 (benches/stack.rs:36-84, nr/tests/stack.rs:31-96).
//
// Vec<u32>::push/pop in log order, with pop on an empty stack returning None and leaving
// the depth at 0. Each op is the function f(x) = max(a, x + b) of the depth before it
// (Push: b=+1, a=1; Pop: b=-1, a=0); these compose associatively
//      (f then g) = (b_f + b_g, max(a_g, a_f + b_g)),
// so the depth before every op is an exclusive scan (one pass, decoupled look-back).
//
// A Push at depth d writes slot d; a Pop at depth d > 0 reads slot d-1. Because the depth
// moves by ±1, the crossings of the edge (t, t+1) alternate Push/Pop in log order, so after a
// stable sort of the touches by slot the value a Pop returns is exactly its predecessor in
// the slot's group (a Push of this batch) or, if it heads the group, the slot's pre-batch
// content. A slot's final content is its group's last Push (the group then ends with a Push).
#include "internal.hpp"

namespace nrg {

constexpr int ST_TPB = 256;
constexpr int ST_ITEMS = 8;
constexpr int ST_TILE = ST_TPB * ST_ITEMS;
constexpr u32 POPBIT = 0x80000000u;

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

__global__ __launch_bounds__(ST_TPB) void st_scan_kernel(const nrg_stack_op* __restrict__ ring, u64 ring_mask, u64 lo,
                                                         u64 n, DevCtl* ctl, u64* desc, u32* ticket,
                                                         u32* __restrict__ sk, u32* __restrict__ sv, u32 sentinel,
                                                         u64 cap, u64 resp_lo, u64 resp_hi, int push_resp,
                                                         u32* __restrict__ resp, uint8_t* __restrict__ some) {
    __shared__ long long s_wb[4], s_wa[4];
    __shared__ u32 s_tile;
    __shared__ long long s_dbase;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (t == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const u32 tile = s_tile;
    const u64 base = (u64)tile * ST_TILE + (u64)t * ST_ITEMS;

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
        // predecessors (a one-lane walk costs a round trip per predecessor tile, and all tiles
        // are in flight together, so each walks back to tile 0: 42 us for 1M ops).
        Fn tagg = {0, 0};
        for (int i = 0; i < 4; i++) tagg = fn_then(tagg, Fn{s_wb[i], s_wa[i]});
        long long dbase = 0;
        if (tile == 0) {
            dbase = ctl->depth;
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
            if ((u64)tile == ntiles - 1) ctl->depth = fn_apply(tagg, dbase);
            s_dbase = dbase;
        }
    }
    __syncthreads();
    long long d = fn_apply(tpre, s_dbase);
    bool over = false;
#pragma unroll
    for (int q = 0; q < ST_ITEMS; q++) {
        const u64 i = base + q;
        if (i >= n) break;
        const u64 g = lo + i;
        const bool inwin = g >= resp_lo && g < resp_hi;
        if (ops[q].op) {  // Push: writes slot d
            if ((u64)d >= cap) over = true;
            sk[i] = (u64)d >= cap ? sentinel : (u32)d;
            sv[i] = (u32)i;
            if (inwin) {
                resp[g - resp_lo] = push_resp ? ops[q].val : 0u;
                some[g - resp_lo] = push_resp ? 1 : 0;
            }
            d += 1;
        } else if (d > 0) {  // Pop: reads slot d-1 (resolved after the sort)
            sk[i] = (u32)(d - 1);
            sv[i] = (u32)i | POPBIT;
            d -= 1;
        } else {  // Pop on empty: None, depth stays 0
            sk[i] = sentinel;
            sv[i] = (u32)i | POPBIT;
            if (inwin) {
                resp[g - resp_lo] = 0;
                some[g - resp_lo] = 0;
            }
        }
    }
    if (over) atomicOr(&ctl->err, ERR_CAPACITY);
}

__global__ __launch_bounds__(256) void st_resolve_kernel(const u32* __restrict__ sk, const u32* __restrict__ sv, u64 n,
                                                         const nrg_stack_op* __restrict__ ring, u64 ring_mask, u64 lo,
                                                         const u32* __restrict__ stack, u32 sentinel, u64 resp_lo,
                                                         u64 resp_hi, u32* __restrict__ resp,
                                                         uint8_t* __restrict__ some) {
    const u64 p = blockIdx.x * 256ull + threadIdx.x;
    if (p >= n) return;
    const u32 slot = sk[p], v = sv[p];
    if (slot == sentinel || !(v & POPBIT)) return;
    const u64 g = lo + (v & ~POPBIT);
    if (g < resp_lo || g >= resp_hi) return;
    u32 val;
    if (p > 0 && sk[p - 1] == slot)
        val = ring[(lo + (sv[p - 1] & ~POPBIT)) & ring_mask].val;
    else
        val = stack[slot];
    resp[g - resp_lo] = val;
    some[g - resp_lo] = 1;
}

__global__ __launch_bounds__(256) void st_commit_kernel(const u32* __restrict__ sk, const u32* __restrict__ sv, u64 n,
                                                        const nrg_stack_op* __restrict__ ring, u64 ring_mask, u64 lo,
                                                        u32* __restrict__ stack, u32 sentinel) {
    const u64 p = blockIdx.x * 256ull + threadIdx.x;
    if (p >= n) return;
    const u32 slot = sk[p], v = sv[p];
    if (slot == sentinel || (v & POPBIT)) return;
    if (p + 1 < n && sk[p + 1] == slot) return;
    stack[slot] = ring[(lo + v) & ring_mask].val;
}

hipError_t st_replay_chunk(nrg_ctx* c, u64 lo, u64 n, u64 resp_lo, u64 resp_hi, uint32_t* d_resp, uint8_t* d_some) {
    if (n == 0) return hipSuccess;
    hipStream_t st = c->stream;
    const u64 ring_mask = c->log_size - 1;
    const nrg_stack_op* ring = (const nrg_stack_op*)c->d_ring;
    const u32 sentinel = (u32)((1ull << c->stack_key_bits) - 1);
    const u64 tiles = (n + ST_TILE - 1) / ST_TILE;
    // descriptors: [ticket (64 words of u32 = 32 u64)] [tiles u64]
    u64* desc = (u64*)c->d_scan_desc + 32;
    u32* ticket = c->d_scan_desc;
    hipError_t e = hipMemsetAsync(c->d_scan_desc, 0, (32 + tiles) * sizeof(u64), st);
    if (e != hipSuccess) return e;
    u32* keys = (u32*)c->d_tmp_u64;           // n u32
    u32* vals = keys + c->cfg.max_batch;      // n u32
    const bool want = d_resp != nullptr && resp_lo < lo + n && resp_hi > lo;
    timer_begin(c, "st_replay");
    st_scan_kernel<<<(unsigned)tiles, ST_TPB, 0, st>>>(ring, ring_mask, lo, n, c->d_ctl, desc, ticket, keys, vals,
                                                      sentinel, c->cfg.stack_capacity, want ? resp_lo : 0,
                                                      want ? resp_hi : 0, (int)c->cfg.stack_push_resp, d_resp, d_some);
    u32 *sk = nullptr, *sv = nullptr;
    e = sort_pairs(c->sort, keys, vals, n, (int)c->stack_key_bits, st, &sk, &sv);
    if (e != hipSuccess) return e;
    const unsigned g = (unsigned)((n + 255) / 256);
    if (want) st_resolve_kernel<<<g, 256, 0, st>>>(sk, sv, n, ring, ring_mask, lo, c->d_stack, sentinel, resp_lo,
                                                  resp_hi, d_resp, d_some);
    st_commit_kernel<<<g, 256, 0, st>>>(sk, sv, n, ring, ring_mask, lo, c->d_stack, sentinel);
    timer_end(c, "st_replay");
    return hipGetLastError();
}

}  // namespace nrg
