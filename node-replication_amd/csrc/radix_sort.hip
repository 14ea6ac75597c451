// radix_sort.hip — stable LSD radix sort of (u32 key, u32 value) pairs for gfx950.
//
// Used by the replay pipelines to group log records by target (BLT entry / stack slot /
// synthetic word) while preserving log order inside each group (SURVEY.md §2.2 K1/K3/K4;
// BASELINE.json north_star: "stable LDS/wavefront radix sort by key").
//
// Structure (one launch per 8-bit digit + one histogram launch):
//   rs_hist   : every block histograms its slice for all passes in LDS, then one global
//               atomicAdd per (pass, digit).
//   rs_pass   : tiles of 2048 keys taken in ticket order (forward progress for the
//               look-back); per-wave stable ranking with 8 ballots per key (64-lane
//               match, lanemask_lt popcount), per-wave digit counters in LDS; the tile's
//               per-digit counts are published as 32-bit {status:2, count:30} granules and
//               each digit thread looks back over predecessor tiles (decoupled look-back;
//               relaxed agent-scope atomics, the granule IS the flag, no fences needed);
//               keys are then reordered by digit in LDS and written out in runs.
#include "internal.hpp"

namespace nrg {

constexpr int RS_TPB = 256;
constexpr int RS_TILE_MIN = RS_TPB * 2;  // smallest tile (RS_ITEMS = 2): sizes the descriptor array
// Keys per thread. Measured on MI355X (100k keys): 2048-key tiles 10.3 us/pass, 512-key tiles
// slower (the look-back is bound by agent-scope atomic latency, not by per-tile work).
static inline int rs_items_for(u64 n) {
    (void)n;
    return 8;
}
constexpr u32 ST_AGG = 1u << 30;
constexpr u32 ST_INC = 2u << 30;
constexpr u32 ST_MASK = 3u << 30;
constexpr u32 CNT_MASK = (1u << 30) - 1;
constexpr int LB_WIN = 16;  // look-back window (descriptors loaded per step; 64 measured slower)
constexpr u64 RS_HIST_WORDS = 4 * 256;
constexpr u64 RS_TICKET_WORDS = 64;

__device__ __forceinline__ u32 wave_incl_scan(u32 x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        u32 y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

// exclusive scan over the 256 threads of a block; tmp holds 4 words
__device__ __forceinline__ u32 block_excl_scan256(u32 x, u32* tmp) {
    const u32 inc = wave_incl_scan(x);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) tmp[w] = inc;
    __syncthreads();
    u32 off = 0;
#pragma unroll
    for (int i = 0; i < 4; i++)
        if (i < w) off += tmp[i];
    __syncthreads();
    return off + inc - x;
}

__global__ __launch_bounds__(256) void rs_hist_kernel(const u32* __restrict__ keys, u64 n, int passes,
                                                      u32* __restrict__ hist) {
    __shared__ u32 sh[4 * 256];
    for (int i = threadIdx.x; i < 4 * 256; i += 256) sh[i] = 0;
    __syncthreads();
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (u64)gridDim.x * 256ull) {
        const u32 k = keys[i];
        for (int p = 0; p < passes; p++) atomicAdd(&sh[p * 256 + ((k >> (8 * p)) & 255)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < passes * 256; i += 256) {
        const u32 v = sh[i];
        if (v) atomicAdd(&hist[i], v);
    }
}

template <int RS_ITEMS>
__global__ __launch_bounds__(256) void rs_pass_kernel(const u32* __restrict__ kin, const u32* __restrict__ vin,
                                                      u32* __restrict__ kout, u32* __restrict__ vout, u64 n,
                                                      int shift, const u32* __restrict__ hist_p, u32* ticket,
                                                      u32* desc) {
    constexpr int RS_TILE = RS_TPB * RS_ITEMS;
    __shared__ u32 s_k[RS_TILE];
    __shared__ u32 s_v[RS_TILE];
    __shared__ u32 s_wh[4 * 256];
    __shared__ u32 s_texcl[256];
    __shared__ u32 s_gbase[256];
    __shared__ u32 s_tmp[4];
    __shared__ u32 s_tile;

    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (t == 0) s_tile = atomicAdd(ticket, 1u);
    for (int i = t; i < 4 * 256; i += 256) s_wh[i] = 0;
    __syncthreads();
    const u32 tile = s_tile;
    const u64 base = (u64)tile * RS_TILE;

    u32 key[RS_ITEMS], val[RS_ITEMS], rank[RS_ITEMS];
#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++) {
        const u64 e = base + (u64)w * (64 * RS_ITEMS) + j * 64 + lane;
        const bool valid = e < n;
        key[j] = valid ? kin[e] : 0u;
        val[j] = valid ? (vin ? vin[e] : (u32)e) : 0u;
    }

    // Stable rank within the wave: element order (wave, item, lane) is the input order.
    const u64 lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++) {
        const u64 e = base + (u64)w * (64 * RS_ITEMS) + j * 64 + lane;
        const bool valid = e < n;
        const u32 d = (key[j] >> shift) & 255u;
        u64 m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const bool bit = (d >> b) & 1u;
            const u64 bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
        u32 r = 0;
        if (valid) {
            const u32 cnt = (u32)__popcll(m);
            const int leader = __ffsll((unsigned long long)m) - 1;
            const u32 before = s_wh[w * 256 + d];
            r = before + (u32)__popcll(m & lt);
            if (lane == leader) s_wh[w * 256 + d] = before + cnt;
        }
        rank[j] = r;
    }
    __syncthreads();

    // Thread t owns digit t: wave prefixes, tile count, publish the aggregate.
    const u32 d = (u32)t;
    const u32 c0 = s_wh[d], c1 = s_wh[256 + d], c2 = s_wh[512 + d], c3 = s_wh[768 + d];
    const u32 tcnt = c0 + c1 + c2 + c3;
    u32* my = desc + (u64)tile * 256 + d;
    __hip_atomic_store(my, (tile == 0 ? ST_INC : ST_AGG) | tcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    s_wh[d] = 0;
    s_wh[256 + d] = c0;
    s_wh[512 + d] = c0 + c1;
    s_wh[768 + d] = c0 + c1 + c2;
    const u32 texcl = block_excl_scan256(tcnt, s_tmp);
    s_texcl[d] = texcl;
    const u32 gex = block_excl_scan256(hist_p[d], s_tmp);

    u32 excl = 0;
    if (tile > 0) {
        // Windowed look-back: LB_WIN predecessor descriptors are loaded together (independent
        // loads in flight), then consumed newest-first until an inclusive one. A serial walk
        // costs one memory round trip per predecessor tile; this costs one per LB_WIN.
        int tt = (int)tile - 1;
        for (;;) {
            u32 v[LB_WIN];
#pragma unroll
            for (int q = 0; q < LB_WIN; q++)
                v[q] = tt - q >= 0 ? __hip_atomic_load(desc + (u64)(tt - q) * 256 + d, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : ST_INC;  // before tile 0: an inclusive zero
            int used = 0;
            bool done = false;
#pragma unroll
            for (int q = 0; q < LB_WIN; q++) {
                if (done || used < q) continue;  // stopped earlier in the window
                const u32 st = v[q] & ST_MASK;
                if (st == 0) continue;  // not published yet: retry from here
                excl += v[q] & CNT_MASK;
                used = q + 1;
                if (st == ST_INC) done = true;
            }
            if (done) break;
            tt -= used;
            if (used < LB_WIN) __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(my, ST_INC | (excl + tcnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_gbase[d] = gex + excl;
    __syncthreads();

#pragma unroll
    for (int j = 0; j < RS_ITEMS; j++) {
        const u64 e = base + (u64)w * (64 * RS_ITEMS) + j * 64 + lane;
        if (e < n) {
            const u32 dj = (key[j] >> shift) & 255u;
            const u32 pos = s_texcl[dj] + s_wh[w * 256 + dj] + rank[j];
            s_k[pos] = key[j];
            s_v[pos] = val[j];
        }
    }
    __syncthreads();
    const u64 rem = n - base;
    const u32 tile_n = rem < (u64)RS_TILE ? (u32)rem : (u32)RS_TILE;
    for (u32 q = t; q < tile_n; q += RS_TPB) {
        const u32 k = s_k[q];
        const u32 dd = (k >> shift) & 255u;
        const u64 dst = (u64)s_gbase[dd] + (q - s_texcl[dd]);
        kout[dst] = k;
        vout[dst] = s_v[q];
    }
}

int sort_alloc(SortScratch& s, u64 cap) {
    if (cap == 0) cap = 1;
    s.cap = cap;
    s.max_tiles = (cap + RS_TILE_MIN - 1) / RS_TILE_MIN;
    s.ctl_words = RS_HIST_WORDS + RS_TICKET_WORDS + 4 * s.max_tiles * 256;
    for (int i = 0; i < 2; i++) {
        if (hipMalloc(&s.k[i], cap * 4) != hipSuccess) return NRG_E_NOMEM;
        if (hipMalloc(&s.v[i], cap * 4) != hipSuccess) return NRG_E_NOMEM;
    }
    if (hipMalloc(&s.ctlmem, s.ctl_words * 4) != hipSuccess) return NRG_E_NOMEM;
    return NRG_OK;
}

void sort_free(SortScratch& s) {
    for (int i = 0; i < 2; i++) {
        if (s.k[i]) (void)hipFree(s.k[i]);
        if (s.v[i]) (void)hipFree(s.v[i]);
        s.k[i] = s.v[i] = nullptr;
    }
    if (s.ctlmem) (void)hipFree(s.ctlmem);
    s.ctlmem = nullptr;
}

static int sort_passes(int key_bits) {
    int passes = (key_bits + 7) / 8;
    return passes < 1 ? 1 : passes > 4 ? 4 : passes;
}

hipError_t sort_prepare(SortScratch& s, u64 n, int key_bits, hipStream_t st, u32** hist) {
    if (n > s.cap || n >= (1ull << 30)) return hipErrorInvalidValue;
    const u64 tile_keys = (u64)RS_TPB * rs_items_for(n);
    const u64 tiles = (n + tile_keys - 1) / tile_keys;
    const u64 words = RS_HIST_WORDS + RS_TICKET_WORDS + (u64)sort_passes(key_bits) * tiles * 256;
    *hist = s.ctlmem;
    return hipMemsetAsync(s.ctlmem, 0, words * 4, st);
}

hipError_t sort_run(SortScratch& s, const u32* keys_in, const u32* vals_in, u64 n, int key_bits, hipStream_t st,
                    u32** out_k, u32** out_v) {
    const int passes = sort_passes(key_bits);
    const int items = rs_items_for(n);
    const u64 tile_keys = (u64)RS_TPB * items;
    const u64 tiles = (n + tile_keys - 1) / tile_keys;
    u32* hist = s.ctlmem;
    u32* tickets = s.ctlmem + RS_HIST_WORDS;
    u32* desc = s.ctlmem + RS_HIST_WORDS + RS_TICKET_WORDS;
    const u32* kin = keys_in;
    const u32* vin = vals_in;
    for (int p = 0; p < passes; p++) {
        u32* ko = s.k[p & 1];
        u32* vo = s.v[p & 1];
        u32* dsc = desc + (u64)p * tiles * 256;
        if (items == 2)
            rs_pass_kernel<2><<<(unsigned)tiles, RS_TPB, 0, st>>>(kin, vin, ko, vo, n, 8 * p, hist + 256 * p,
                                                                 tickets + p, dsc);
        else if (items == 4)
            rs_pass_kernel<4><<<(unsigned)tiles, RS_TPB, 0, st>>>(kin, vin, ko, vo, n, 8 * p, hist + 256 * p,
                                                                 tickets + p, dsc);
        else
            rs_pass_kernel<8><<<(unsigned)tiles, RS_TPB, 0, st>>>(kin, vin, ko, vo, n, 8 * p, hist + 256 * p,
                                                                 tickets + p, dsc);
        kin = ko;
        vin = vo;
    }
    *out_k = (u32*)kin;
    *out_v = (u32*)vin;
    return hipGetLastError();
}

hipError_t sort_pairs(SortScratch& s, const u32* keys_in, const u32* vals_in, u64 n, int key_bits,
                      hipStream_t st, u32** out_k, u32** out_v) {
    if (n == 0) {
        *out_k = s.k[0];
        *out_v = s.v[0];
        return hipSuccess;
    }
    u32* hist = nullptr;
    hipError_t e = sort_prepare(s, n, key_bits, st, &hist);
    if (e != hipSuccess) return e;
    // the histogram pass needs keys; with vals_in == nullptr the first pass generates 0..n-1
    u64 hb = (n + 256 * 8 - 1) / (256 * 8);  // 64 keys per thread measured 2.3x slower
    if (hb > 1024) hb = 1024;
    rs_hist_kernel<<<(unsigned)hb, 256, 0, st>>>(keys_in, n, sort_passes(key_bits), hist);
    return sort_run(s, keys_in, vals_in, n, key_bits, st, out_k, out_v);
}

}  // namespace nrg
