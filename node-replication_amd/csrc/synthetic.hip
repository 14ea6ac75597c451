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

hipError_t sy_init(nrg_ctx* c) {
    sy_init_kernel<<<1024, 256, 0, c->stream>>>(c->d_words, c->cfg.synth_n);
    return hipGetLastError();
}

hipError_t sy_replay_chunk(nrg_ctx* c, u64 lo, u64 n, u64 resp_lo, u64 resp_hi, u64* d_resp, uint8_t* d_some) {
    if (n == 0) return hipSuccess;
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
    const nrg_config& cf = c->cfg;
    sy_read_kernel<<<(unsigned)((n + 255) / 256), 256, 0, c->stream>>>(
        d_ops, n, c->d_words, cf.synth_n, cf.synth_hot_reads, cf.synth_hot_writes, cf.synth_cold_reads, d_sums);
    return hipGetLastError();
}

}  // namespace nrg
