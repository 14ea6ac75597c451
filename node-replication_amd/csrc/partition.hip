// partition.hip — cnr-style key partitioning of hashmap rounds across replicas.
//
// cnr (cnr/src/lib.rs:134-167) maps every operation to one of several logs with
// LogMapper::hash(); conflicting operations (the same key) share a log, so each log replays
// independently (cnr/src/replica.rs:430-445 hash -> log, :673-736 combine(hashidx)). Across GPUs
// the log of partition p lives on GPU p, which holds only the keys it owns: a round's Puts and
// Gets are routed to their owners, each owner replays the Puts it received in rank order (the
// global log order restricted to its keys, so every key sees its writes in the same order as an
// NR replay of W_0 || W_1 || ...), answers the Gets it received, and the answers travel back.
//
// Owner of a key: the low 32 bits of mix64(key) scaled to [0, parts). The table's home slot uses
// the top bits of the same mix (common.hpp table_home), so a partition's keys still spread over
// its whole table.
//
// Kernels (records of `words` u64 with the key in word 0: Puts 2, Get keys 1):
//   pt_count_kernel    per 2048-record tile: records per owner
//   pt_scan_kernel     per owner: exclusive scan of the tile counts, and the owner's total
//   pt_scatter_kernel  per tile: stable rank of each record among its owner's records of the
//                      tile (per wave, one ballot per distinct owner in a 64-record round; the
//                      per-owner counts of a wave live in lane `owner`), then out[dest] = record
//                      and pos[i] = dest, dest = owner start + tile offset + wave offset + rank
//   pt_gather_kernel   answers back to the caller's order: dst[i] = src[pos[i]]
#include "internal.hpp"

namespace nrg {

constexpr int PT_TPB = 256;
constexpr int PT_WAVES = PT_TPB / 64;
constexpr int PT_ROUNDS = 8;                             // 64-record rounds per wave
constexpr u32 PT_TILE = PT_TPB * PT_ROUNDS;              // 2048 records per tile

__global__ __launch_bounds__(PT_TPB) void pt_count_kernel(const u64* __restrict__ in, u64 n, u32 words, u32 parts,
                                                          u32* __restrict__ tcnt) {
    __shared__ u32 s_c[PT_MAX_PARTS];
    if (threadIdx.x < PT_MAX_PARTS) s_c[threadIdx.x] = 0;
    __syncthreads();
    const u64 t0 = (u64)blockIdx.x * PT_TILE;
    for (u32 k = threadIdx.x; k < PT_TILE; k += PT_TPB) {
        const u64 i = t0 + k;
        if (i < n) atomicAdd(&s_c[key_owner(in[i * words], parts)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < parts) tcnt[(u64)blockIdx.x * parts + threadIdx.x] = s_c[threadIdx.x];
}

// one block per owner p: toff[t][p] = sum of tcnt[t'][p], t' < t; total[p]
__global__ __launch_bounds__(PT_TPB) void pt_scan_kernel(const u32* __restrict__ tcnt, u32 ntiles, u32 parts,
                                                         u32* __restrict__ toff, u64* __restrict__ total) {
    __shared__ u32 s_w[PT_WAVES];
    const u32 p = blockIdx.x;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const u32 K = (ntiles + PT_TPB - 1) / PT_TPB;  // tiles [t*K, t*K + K) per thread
    u32 loc = 0;
    for (u32 q = 0; q < K; q++) {
        const u32 tile = t * K + q;
        if (tile < ntiles) loc += tcnt[(u64)tile * parts + p];
    }
    u32 inc = loc;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u32 y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    u32 run = inc - loc;
    for (int i = 0; i < w; i++) run += s_w[i];
    for (u32 q = 0; q < K; q++) {
        const u32 tile = t * K + q;
        if (tile < ntiles) {
            const u32 c = tcnt[(u64)tile * parts + p];
            toff[(u64)tile * parts + p] = run;
            run += c;
        }
    }
    if (t == PT_TPB - 1) {
        u32 all = 0;
        for (int i = 0; i < PT_WAVES; i++) all += s_w[i];
        total[p] = all;
    }
}

__global__ __launch_bounds__(PT_TPB) void pt_scatter_kernel(const u64* __restrict__ in, u64 n, u32 words, u32 parts,
                                                            const u32* __restrict__ toff, const u64* __restrict__ total,
                                                            u64* __restrict__ out, u32* __restrict__ pos) {
    __shared__ u32 s_base[PT_MAX_PARTS];          // owner start: exclusive prefix of the totals
    __shared__ u32 s_wc[PT_WAVES][PT_MAX_PARTS];  // per wave counts, then wave offsets
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    if (t == 0) {
        u32 acc = 0;
        for (u32 p = 0; p < parts; p++) {
            s_base[p] = acc;
            acc += (u32)total[p];
        }
    }
    const u64 t0 = (u64)blockIdx.x * PT_TILE + (u64)w * (PT_ROUNDS * 64);
    u32 own[PT_ROUNDS], rank[PT_ROUNDS];
    u32 cnt = 0;  // lane p: this wave's records of owner p so far
#pragma unroll
    for (int r = 0; r < PT_ROUNDS; r++) {
        const u64 i = t0 + (u64)r * 64 + lane;
        const bool valid = i < n;
        const u32 o = valid ? key_owner(in[i * words], parts) : 0u;
        own[r] = o;
        rank[r] = 0;
        u64 act = __ballot(valid);
        while (act) {  // one ballot per distinct owner among the 64 records (wave-uniform loop)
            const int leader = __ffsll((long long)act) - 1;
            const u32 ol = (u32)__shfl((int)o, leader, 64);
            const u64 m = __ballot(valid && o == ol);
            const u32 c0 = (u32)__shfl((int)cnt, (int)ol, 64);
            if (valid && o == ol) rank[r] = c0 + (u32)__popcll(m & ((1ull << lane) - 1));
            if ((u32)lane == ol) cnt += (u32)__popcll(m);
            act &= ~m;
        }
    }
    if ((u32)lane < parts) s_wc[w][lane] = cnt;
    __syncthreads();
    if (t < (int)parts) {
        u32 acc = 0;
        for (int i = 0; i < PT_WAVES; i++) {
            const u32 c = s_wc[i][t];
            s_wc[i][t] = acc;
            acc += c;
        }
    }
    __syncthreads();
    const u32* to = toff + (u64)blockIdx.x * parts;
#pragma unroll
    for (int r = 0; r < PT_ROUNDS; r++) {
        const u64 i = t0 + (u64)r * 64 + lane;
        if (i >= n) continue;
        const u32 o = own[r];
        const u32 dest = s_base[o] + to[o] + s_wc[w][o] + rank[r];
        for (u32 k = 0; k < words; k++) out[(u64)dest * words + k] = in[i * words + k];
        pos[i] = dest;
    }
}

__global__ __launch_bounds__(PT_TPB) void pt_gather_kernel(const u64* __restrict__ src, const uint8_t* __restrict__ src8,
                                                           const u32* __restrict__ pos, u64 n, u64* __restrict__ dst,
                                                           uint8_t* __restrict__ dst8) {
    for (u64 i = blockIdx.x * (u64)PT_TPB + threadIdx.x; i < n; i += (u64)gridDim.x * PT_TPB) {
        const u32 p = pos[i];
        if (dst) dst[i] = src[p];
        if (dst8) dst8[i] = src8[p];
    }
}

// ---- the replica group's fused partition (nrg_group_partitioned_round) -----------------------
// One launch partitions a round's Puts and Get keys together, in one pass: owner o's records go to
// a region of fixed capacity (out + o * cap, cap = the job's own record count, so any owner can
// take all of them), so no global scan of the owner totals is needed. Tiles are blockIdx-ordered
// (Puts first, then Gets); each publishes its per-owner counts as a look-back descriptor and takes
// its offsets from its predecessors' (decoupled look-back, relaxed agent-scope atomics; the
// descriptor word IS the flag, epoch-tagged so no reset pass runs between rounds). The last tile
// of a job writes the owner totals into the round's count-exchange words, and block 0 the
// member's host words (XW_*), so the exchange needs no host copy.
typedef u64 pt_u64x2 __attribute__((ext_vector_type(2)));
constexpr u64 PD_CNT = (1ull << 40) - 1, PD_AGG = 1ull << 40, PD_INC = 2ull << 40, PD_ST = 3ull << 40;
constexpr int PD_EP = 42, PD_WIN = 16;
// fused tiles: 16 waves x 8 rounds of 64 = 8192 records, so a 1M-op round has ~123 tiles and the
// look-back reaches an inclusive descriptor in a few windowed steps (2048-record tiles: 22 us per
// B1 round, the look-back chain of ~490 tiles)
constexpr int PF_TPB = 1024, PF_WAVES = PF_TPB / 64;
constexpr u32 PF_TILE = PF_TPB * PT_ROUNDS;

struct PtFJob {
    const u64* in;
    u64 n;
    u64 cap;      // owner o's records at out[(o * cap + j) * words]
    u64* out;
    u32* pos;     // pos[i] = o * cap + j: where record i went
    u64* desc;    // [tiles][parts] look-back descriptors
    u64* counts;  // [parts] the job's records per owner
    u32 tiles;
};
struct PtFWords {
    u64 w[PT_XW_MAX];
    u64* dst;
    u32 n;
};

template <int WORDS>
__device__ __forceinline__ void ptf_tile(const PtFJob& J, u32 tile, u32 parts, u64 ep, u32* s_wc_flat, u64* s_base) {
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    u32(*s_wc)[PT_MAX_PARTS] = (u32(*)[PT_MAX_PARTS])s_wc_flat;
    const u64 t0 = (u64)tile * PF_TILE + (u64)w * (PT_ROUNDS * 64);
    u64 rec[PT_ROUNDS][WORDS];
#pragma unroll
    for (int r = 0; r < PT_ROUNDS; r++) {
        const u64 i = t0 + (u64)r * 64 + lane;
        if (i < J.n) {
            if constexpr (WORDS == 2) {
                const pt_u64x2 v = ((const pt_u64x2*)J.in)[i];
                rec[r][0] = v.x;
                rec[r][1] = v.y;
            } else {
                rec[r][0] = J.in[i];
            }
        } else {
#pragma unroll
            for (int k = 0; k < WORDS; k++) rec[r][k] = 0;
        }
    }
    u32 own[PT_ROUNDS], rank[PT_ROUNDS];
    u32 cnt = 0;  // lane p: this wave's records of owner p so far
#pragma unroll
    for (int r = 0; r < PT_ROUNDS; r++) {
        const u64 i = t0 + (u64)r * 64 + lane;
        const bool valid = i < J.n;
        const u32 o = valid ? key_owner(rec[r][0], parts) : 0u;
        own[r] = o;
        rank[r] = 0;
        u64 act = __ballot(valid);
        while (act) {  // one ballot per distinct owner among the 64 records (wave-uniform loop)
            const int leader = __ffsll((long long)act) - 1;
            const u32 ol = (u32)__shfl((int)o, leader, 64);
            const u64 m = __ballot(valid && o == ol);
            const u32 c0 = (u32)__shfl((int)cnt, (int)ol, 64);
            if (valid && o == ol) rank[r] = c0 + (u32)__popcll(m & ((1ull << lane) - 1));
            if ((u32)lane == ol) cnt += (u32)__popcll(m);
            act &= ~m;
        }
    }
    if ((u32)lane < parts) s_wc[w][lane] = cnt;
    __syncthreads();
    if (t < (int)parts) {  // wave 0, lane = owner: tile count, wave offsets, look-back
        u32 tc = 0;
        for (int i = 0; i < PF_WAVES; i++) {
            const u32 c = s_wc[i][t];
            s_wc[i][t] = tc;
            tc += c;
        }
        u64* my = J.desc + (u64)tile * parts + t;
        __hip_atomic_store(my, ep | (tile == 0 ? PD_INC : PD_AGG) | tc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        u64 excl = 0;
        if (tile > 0) {
            // windowed: PD_WIN predecessor descriptors in flight per step, consumed newest-first
            // until an inclusive one (radix_sort.hip's look-back; stale epochs read as unpublished)
            int tt = (int)tile - 1;
            for (;;) {
                u64 v[PD_WIN];
#pragma unroll
                for (int q = 0; q < PD_WIN; q++)
                    v[q] = tt - q >= 0 ? __hip_atomic_load(J.desc + (u64)(tt - q) * parts + t, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT)
                                       : (ep | PD_INC);
                int used = 0;
                bool done = false;
#pragma unroll
                for (int q = 0; q < PD_WIN; q++) {
                    if (done || used < q) continue;
                    const u64 st = (v[q] >> PD_EP) == (ep >> PD_EP) ? (v[q] & PD_ST) : 0ull;
                    if (st == 0) continue;  // not published yet: retry from here
                    excl += v[q] & PD_CNT;
                    used = q + 1;
                    if (st == PD_INC) done = true;
                }
                if (done) break;
                tt -= used;
                if (used < PD_WIN) __builtin_amdgcn_s_sleep(1);
            }
            __hip_atomic_store(my, ep | PD_INC | (excl + tc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_base[t] = (u64)t * J.cap + excl;
        if (tile + 1 == J.tiles) J.counts[t] = excl + tc;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < PT_ROUNDS; r++) {
        const u64 i = t0 + (u64)r * 64 + lane;
        if (i >= J.n) continue;
        const u32 o = own[r];
        const u64 dest = s_base[o] + s_wc[w][o] + rank[r];
        if constexpr (WORDS == 2) {
            pt_u64x2 v;
            v.x = rec[r][0];
            v.y = rec[r][1];
            ((pt_u64x2*)J.out)[dest] = v;
        } else {
            J.out[dest] = rec[r][0];
        }
        J.pos[i] = (u32)dest;
    }
}

__global__ __launch_bounds__(PF_TPB) void pt_fused_kernel(PtFJob P, PtFJob K, u32 parts, u64 ep, PtFWords xw) {
    __shared__ u32 s_wc[PF_WAVES * PT_MAX_PARTS];
    __shared__ u64 s_base[PT_MAX_PARTS];
    const u32 b = blockIdx.x;
    if (b == 0) {
        if (threadIdx.x == 0) {  // (constant indices: a lane-indexed argument array goes to scratch)
#pragma unroll
            for (u32 k = 0; k < PT_XW_MAX; k++)
                if (k < xw.n) xw.dst[k] = xw.w[k];
        }
        if (threadIdx.x < parts) {  // a job without tiles has no owner records
            if (P.tiles == 0) P.counts[threadIdx.x] = 0;
            if (K.tiles == 0) K.counts[threadIdx.x] = 0;
        }
    }
    if (b < P.tiles) ptf_tile<2>(P, b, parts, ep, s_wc, s_base);
    else if (b - P.tiles < K.tiles) ptf_tile<1>(K, b - P.tiles, parts, ep, s_wc, s_base);
}

struct PtRoute {
    const u64* src;
    const uint8_t* src8;
    const u32* pos;
    u64 n;
    u64* dst;
    uint8_t* dst8;
};
// answers back to the caller's order, both routes of a round in one launch: dst[i] = src[pos[i]]
__global__ __launch_bounds__(PT_TPB) void pt_route2_kernel(PtRoute a, PtRoute b) {
    const u64 N = a.n + b.n;
    for (u64 i = blockIdx.x * (u64)PT_TPB + threadIdx.x; i < N; i += (u64)gridDim.x * PT_TPB) {
        const bool first = i < a.n;
        const PtRoute& r = first ? a : b;
        const u64 j = first ? i : i - a.n;
        const u32 p = r.pos[j];
        if (r.dst) r.dst[j] = r.src[p];
        if (r.dst8) r.dst8[j] = r.src8[p];
    }
}

// One owner: the stable partition is the identity (out = in, pos[i] = i, counts = n), a copy at
// streaming rate instead of a look-back over 8192-record tiles (a one-rank group: 28 -> ~5 us).
__global__ __launch_bounds__(PT_TPB) void pt_copy1_kernel(const u64* __restrict__ puts, u64 W, u64* __restrict__ pout,
                                                          u32* __restrict__ ppos, const u64* __restrict__ keys, u64 R,
                                                          u64* __restrict__ kout, u32* __restrict__ gpos, u64* counts,
                                                          PtFWords xw) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        counts[0] = W;
        counts[1] = R;
#pragma unroll
        for (u32 k = 0; k < PT_XW_MAX; k++)
            if (k < xw.n) xw.dst[k] = xw.w[k];
    }
    const u64 stride = (u64)gridDim.x * PT_TPB;
    for (u64 i = blockIdx.x * (u64)PT_TPB + threadIdx.x; i < W + R; i += stride) {
        if (i < W) {
            ((pt_u64x2*)pout)[i] = ((const pt_u64x2*)puts)[i];
            ppos[i] = (u32)i;
        } else {
            const u64 j = i - W;
            kout[j] = keys[j];
            gpos[j] = (u32)j;
        }
    }
}

hipError_t pt_fused(hipStream_t s, const u64* puts, u64 W, u64 cap_p, u64* pout, u32* ppos, const u64* keys, u64 R,
                    u64 cap_k, u64* kout, u32* gpos, u64* desc, u32 parts, u32 epoch, u64* counts, const u64* xw,
                    u32 nxw) {
    if (parts == 0 || parts > PT_MAX_PARTS || nxw > PT_XW_MAX) return hipErrorInvalidValue;
    if (W && (W > cap_p || (u64)parts * cap_p > 0xFFFFFFFFull)) return hipErrorInvalidValue;
    if (R && (R > cap_k || (u64)parts * cap_k > 0xFFFFFFFFull)) return hipErrorInvalidValue;
    PtFJob P{(const u64*)puts, W, cap_p, pout, ppos, desc, counts, (u32)((W + PF_TILE - 1) / PF_TILE)};
    PtFJob K{keys, R, cap_k, kout, gpos, desc + (u64)P.tiles * parts, counts + parts,
             (u32)((R + PF_TILE - 1) / PF_TILE)};
    PtFWords x{};
    for (u32 k = 0; k < nxw; k++) x.w[k] = xw[k];
    x.dst = counts + 2 * parts;
    x.n = nxw;
    if (parts == 1) {
        const u64 nb = (W + R + PT_TPB - 1) / PT_TPB;
        pt_copy1_kernel<<<(unsigned)(nb < 2048 ? (nb ? nb : 1) : 2048), PT_TPB, 0, s>>>(puts, W, pout, ppos, keys, R, kout,
                                                                                     gpos, counts, x);
        return hipGetLastError();
    }
    const u32 blocks = P.tiles + K.tiles;
    pt_fused_kernel<<<blocks ? blocks : 1u, PF_TPB, 0, s>>>(P, K, parts, (u64)(epoch & ((1u << 22) - 1)) << PD_EP, x);
    return hipGetLastError();
}

hipError_t pt_route2(hipStream_t s, const u64* src_a, const uint8_t* src8_a, const u32* pos_a, u64 n_a, u64* dst_a,
                     uint8_t* dst8_a, const u64* src_b, const uint8_t* src8_b, const u32* pos_b, u64 n_b, u64* dst_b,
                     uint8_t* dst8_b) {
    const u64 n = n_a + n_b;
    if (n == 0) return hipSuccess;
    const u64 blocks = (n + PT_TPB - 1) / PT_TPB;
    pt_route2_kernel<<<(unsigned)(blocks < 4096 ? blocks : 4096), PT_TPB, 0, s>>>(
        PtRoute{src_a, src8_a, pos_a, n_a, dst_a, dst8_a}, PtRoute{src_b, src8_b, pos_b, n_b, dst_b, dst8_b});
    return hipGetLastError();
}

u64 pt_desc_words(u64 W, u64 R, u32 parts) {
    return ((W + PF_TILE - 1) / PF_TILE + (R + PF_TILE - 1) / PF_TILE) * parts;
}

// Scratch for the tile counts and offsets, grown on demand (the replica's stream is drained
// before a reallocation).
static hipError_t pt_scratch(nrg_ctx* c, u64 words) {
    if (c->pt_words >= words) return hipSuccess;
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return e;
    if (c->d_pt) (void)hipFree(c->d_pt);
    c->d_pt = nullptr;
    c->pt_words = 0;
    if ((e = hipMalloc(&c->d_pt, words * sizeof(u32))) != hipSuccess) return e;
    c->pt_words = words;
    return hipSuccess;
}

hipError_t pt_partition(nrg_ctx* c, const u64* in, u64 n, u32 words, u32 parts, u64* out, u32* pos, u64* total) {
    if (parts == 0 || parts > PT_MAX_PARTS) return hipErrorInvalidValue;
    if (n == 0) return hipMemsetAsync(total, 0, parts * sizeof(u64), c->stream);
    const u64 ntiles = (n + PT_TILE - 1) / PT_TILE;
    if (ntiles > 0xFFFFFFFFull || n > 0xFFFFFFFFull) return hipErrorInvalidValue;
    hipError_t e = pt_scratch(c, 2 * ntiles * parts);
    if (e != hipSuccess) return e;
    u32* tcnt = (u32*)c->d_pt;
    u32* toff = tcnt + ntiles * parts;
    pt_count_kernel<<<(unsigned)ntiles, PT_TPB, 0, c->stream>>>(in, n, words, parts, tcnt);
    pt_scan_kernel<<<parts, PT_TPB, 0, c->stream>>>(tcnt, (u32)ntiles, parts, toff, total);
    pt_scatter_kernel<<<(unsigned)ntiles, PT_TPB, 0, c->stream>>>(in, n, words, parts, toff, total, out, pos);
    return hipGetLastError();
}

hipError_t pt_gather(nrg_ctx* c, const u64* src, const uint8_t* src8, const u32* pos, u64 n, u64* dst, uint8_t* dst8) {
    if (n == 0) return hipSuccess;
    const u64 blocks = (n + PT_TPB - 1) / PT_TPB;
    pt_gather_kernel<<<(unsigned)(blocks < 4096 ? blocks : 4096), PT_TPB, 0, c->stream>>>(src, src8, pos, n, dst, dst8);
    return hipGetLastError();
}

}  // namespace nrg
