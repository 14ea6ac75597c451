// stack.hip — Stack replica replay on gfx950 (benches/stack.rs:36-84, nr/tests/stack.rs:31-96).
//
// Vec<u32>::push/pop in log order, with pop on an empty stack returning None and leaving
// the depth at 0. A run of ops maps the depth x before it to max(x + e, e - m), where m <= 0 is
// the unclamped minimum of its ±1 walk and e its end; these compose associatively, so every
// lane's start depth is an exclusive scan (one pass, decoupled look-back over tiles).
//
// A Push at depth d writes slot d; a Pop at depth d > 0 reads slot d-1. Because the depth
// moves by ±1, the touches of one slot alternate Push/Pop in log order, so no sort is needed
// to pair them:
//   * each lane replays its own ops against a stack of its own in LDS;
//   * a Pop below the lane's start reads the level's last Push in the nearest earlier lane
//     whose lowest level is <= it (every lane in between stays above it);
//   * with no such lane in the tile, the nearest earlier TILE whose minimum depth is <= the
//     slot holds it (its table "last Push to slot tmin + r"), or else the slot's content
//     before the chunk;
//   * the chunk's final content of a slot s below the final depth is its last Push, in the
//     LAST tile whose minimum depth is <= s: that tile commits the levels
//     [tmin, min(tile end depth, minimum depth of every later tile)).
// One kernel, st_round_kernel: the tile pass of chunk e and the finish (cross-tile Pops,
// commit) of chunk e-1 in one launch.
#include "internal.hpp"

namespace nrg {

#ifndef NRG_ST_OPS
// ops per lane, measured at 1M-op rounds (bench.py --workload stack): 8 -> 17.4 us, 16 -> 18.8 us,
// 32 -> 21.2 us (session 7, before the branch-free query walk: 21.5 / 20.6 / 22.7 us); round 6:
// 4 (1024-op tiles, four per CU) 23.7 us against 8's 14.0 on one box (profiles/r06/stack_resp_policy.txt)
#define NRG_ST_OPS 8
#endif
constexpr int SW_OPS = NRG_ST_OPS;          // ops per lane, replayed in order by that lane (<= 32)
constexpr int ST_WAVES = 4;                 // a tile is one workgroup of 4 waves
constexpr int ST_LANES = 64 * ST_WAVES;     // 256 lanes
constexpr int ST_TILE = ST_LANES * SW_OPS;  // 2048 ops
constexpr int ST_PB = SW_OPS == 32 ? 13 : SW_OPS == 16 ? 12 : 11;  // bits of a position in the tile
constexpr u32 ST_PMASK = (1u << ST_PB) - 1;
static_assert(ST_TILE == 1 << ST_PB, "positions");
static_assert(SW_OPS == 8 || SW_OPS == 16 || SW_OPS == 32, "ops per lane");

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

// Per-tile results of the tile pass, read by the chunk's finish (st_round_kernel).
struct StTiles {
    long long* tmin;   // [tiles] minimum depth reached in the tile (start and end included)
    u32* tend;         // [tiles] end depth of the tile - tmin
    u32* table;        // [tiles][ST_TILE] value of the tile's last Push to slot tmin + r, for the
                       // slots below the tile's end depth (the only ones ever looked up)
    u32* ucnt;         // [tiles] Pops whose Push is outside the tile
    u32* upop;         // [tiles][ST_TILE] those Pops: (slot - tmin) << ST_PB | position
    u32* uval;         // [tiles][ST_TILE] their slot's content before the chunk (if below it)
};

// The nearest tile k <= from whose minimum is <= s (skipping 8- and 64-tile groups whose
// minimum is above s), or -1.
__device__ __forceinline__ int st_walk(const long long* s_tm, const long long* s_g8, const long long* s_gm, int k,
                                       long long s) {
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
    return k;
}

// The last tile of [0, tiles) whose minimum is <= s, or -1: the last 64-tile group with a
// minimum <= s, then its last such 8-tile group, then its last such tile, each level's eight
// reads in flight together (three or four LDS round trips instead of a walk's dependent steps).
__device__ __forceinline__ int st_find(const long long* s_tm, const long long* s_g8, const long long* s_gm, int tiles,
                                       long long s) {
    constexpr long long INF = 1ll << 62;
    int g = (tiles - 1) >> 6;
    for (;;) {  // 64-tile groups from the last, four at a time
        if (g < 0) return -1;
        long long m[4];
#pragma unroll
        for (int i = 0; i < 4; i++) m[i] = g - i >= 0 ? s_gm[g - i] : INF;
        int hit = -1;
#pragma unroll
        for (int i = 3; i >= 0; i--) hit = m[i] <= s ? i : hit;
        if (hit >= 0) {
            g -= hit;
            break;
        }
        g -= 4;
    }
    const int n8 = (tiles - 1) / 8;  // last valid 8-tile group
    long long m8[8];
#pragma unroll
    for (int i = 0; i < 8; i++) m8[i] = g * 8 + i <= n8 ? s_g8[g * 8 + i] : INF;
    int b = g * 8;
#pragma unroll
    for (int i = 0; i < 8; i++) b = m8[i] <= s ? g * 8 + i : b;
    long long m1[8];
#pragma unroll
    for (int i = 0; i < 8; i++) m1[i] = b * 8 + i < tiles ? s_tm[b * 8 + i] : INF;
    int k = -1;
#pragma unroll
    for (int i = 0; i < 8; i++) k = m1[i] <= s ? b * 8 + i : k;
    return k;
}

// Stage the tile minima of a chunk in LDS (256 threads): s_tm[tiles], then the minimum of
// every 8-tile group (s_g8) and 64-tile group (s_gm). Returns this thread's minimum over the
// tiles after `after` (pass ~0u for none).
__device__ __forceinline__ long long st_stage(const long long* __restrict__ tmin, u32 tiles, long long* s_tm,
                                              long long* s_g8, long long* s_gm, u32 after, bool in_lds = false) {
    const int t = threadIdx.x, lane = t & 63;
    const u32 ngr = (tiles + 63) / 64;
    long long later = 1ll << 62;
    for (u32 k = t; k < ngr * 64; k += 256) {
        // in_lds: s_tm[0, tiles) already holds the minima (st_copy_lds)
        const long long v = k < tiles ? (in_lds ? s_tm[k] : tmin[k]) : (1ll << 62);
        if (k < tiles) s_tm[k] = v;
        if (k > after) later = v < later ? v : later;
        long long m = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const long long x = __shfl_xor(m, off, 64);
            m = x < m ? x : m;
            if (off == 4 && (lane & 7) == 0 && (k >> 3) <= tiles / 8) s_g8[k >> 3] = m;
        }
        if (lane == 0) s_gm[k >> 6] = m;
    }
    return later;
}

// Copy the tile minima of a chunk (tiles x 8 B) into s_tm straight from global memory to LDS
// (global_load_lds: no VGPR holds them and no wait is due until the caller's next vmcnt wait,
// after which, with a barrier, the copy is visible to the workgroup). Called by one wave.
__device__ __forceinline__ void st_copy_lds(const long long* tmin, u32 tiles, long long* s_tm) {
    const u32 lane = threadIdx.x & 63, nd = 2 * tiles;
    const u32* src = reinterpret_cast<const u32*>(tmin);
    u32* dst = reinterpret_cast<u32*>(s_tm);
    for (u32 j0 = 0; j0 < nd; j0 += 64) {
        const u32 j = j0 + lane;
        if (j < nd)
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(src + j),
                                             (void __attribute__((address_space(3)))*)(dst + j0), 4, 0, 0);
    }
}

// A replay launch: the tile pass of chunk e (A) and, in the workgroups before it, the finish
// of chunk e-1 (P): its cross-tile Pops and its commit. Chunks alternate between two sets of
// per-tile buffers (parity), so the two never touch the same scratch.
struct StPass {
    const nrg_stack_op* src;  // chunk records in a caller buffer, or nullptr (ring)
    nrg_stack_op* ring;
    u64 ring_mask;
    u64 lo, n;                // log range
    u32 tiles, par;           // tiles; parity of the chunk's buffers and depth slot
    u64* desc;                // look-back descriptors (parity buffer)
    StTiles tl;
    u64 rlo, rhi;             // response window (log indices)
    u32* resp;
    uint8_t* some;
    u32 stall;  // NRG_KNOB_STALL (tests)
    u32 plain;  // (A/B, NRG_KNOB_EXP bit 6) plain stores instead of streaming ones for the tile outputs
};

// Streaming (nt) stores for outputs no later work of this launch reads (the log copy, the
// responses): with plain stores they stay dirty in the XCD's L2 until the kernel-end write-back,
// which then runs after the last workgroup (~13 MB per 1M-op round); streamed, they drain while
// the look-back waits. 15.35-15.50 -> 14.88-14.90 us per round on one box, 15.37-15.42 -> 15.14-15.24
// on another (profiles/r04_nt_stores.txt). NRG_KNOB_EXP bit 6 = plain stores (A/B).
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void nt_store4(uint4* p, uint4 v) {
    const u32x4_t t = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(t, (u32x4_t*)p);
}

// A tile's Pop responses: the lane's wide store and the later single-op stores (the answers to
// its unmatched Pops, from any wave of the tile, after a barrier) take the same cache policy, so
// no ordering between a streamed and a plain store to one word is relied on. The plain form is a
// relaxed wavefront-scope atomic store (the same plain store in the ISA): two plain-vs-streamed
// stores on either side of a branch are merged by the compiler into one plain store, the hint
// dropped (profiles/r06/stack_resp_policy.txt).
__device__ __forceinline__ void st_resp(u32* p, u32 v, u32 plain) {
    if (plain) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    else __builtin_nontemporal_store(v, p);
}

// Round 6: the `some` bytes (the lane's 8-B store and the patches, NRG_ST_SOME_NT) and the finish's
// stores (cross-tile answers and the commit, NRG_ST_FIN_NT) are streamed as well. Same box, two
// pairs: 13.87-13.96 -> 13.71-13.78 us per 1M-op round (finish alone 13.73-13.84, some alone no
// change; profiles/r06/stack_stream_some_finish.txt). Build with =0 for the plain A/B.
#ifndef NRG_ST_SOME_NT
#define NRG_ST_SOME_NT 1
#endif
#ifndef NRG_ST_FIN_NT
#define NRG_ST_FIN_NT 1
#endif
template <bool NT, typename T>
__device__ __forceinline__ void st_pol(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__device__ __forceinline__ void wave_sync() {  // LDS written by other lanes of this wave
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (m, e) of a clamped ±1 walk: unclamped minimum m <= 0 and end e; from start x it ends at
// max(x + e, e - m). Composition, f then g: (min(m_f, e_f + m_g), e_f + e_g).
__device__ __forceinline__ void me_then(int& m, int& e, int m2, int e2) {
    const int t = e + m2;
    m = m < t ? m : t;
    e += e2;
}

// One workgroup per tile of 256 * SW_OPS ops; lane t replays ops [SW_OPS t, SW_OPS (t + 1)) in order.
//   1. Local pass: every lane keeps its own stack in LDS (row = height, column = lane, so the
//      64 lanes of a wave never share a bank). A Pop with a non-empty local stack returns its
//      top; a Pop on an empty local stack is "unmatched" (it reaches below the lane's start).
//      Nothing here depends on the lane's start depth: the lane leaves `nun` unmatched Pops and
//      a residual stack of `top` Pushes, i.e. the map (m, e) = (-nun, top - nun).
//   2. Scan of the lanes' (m, e) (waves, then the 4 wave totals in LDS); the tile's aggregate
//      is published at once for later tiles' look-back.
//   3. Look-back (wave 0): lane l composes a run of earlier tiles' aggregates, one wave
//      composition joins the runs -> the tile's start depth D, hence each lane's start depth
//      D_t, its lowest level amin_t = max(D_t - nun, 0) and its end aend_t = amin_t + top. The
//      lane's residual Push i sits at level amin_t + i.
//   4. The k-th unmatched Pop of lane t (k < min(nun, D_t); the others find the stack empty)
//      reads level L = D_t - 1 - k, written last by the nearest earlier lane v with
//      amin_v <= L (every lane in between stays above L): residual entry L - amin_v of lane v.
//      Each wave lists its unmatched Pops and answers them one per lane per round by greedy
//      skips over a sparse table of lane minima (256 lanes: 8 levels). With no such lane the
//      Push is in an earlier tile (or before the chunk): the Pop goes to the finish's
//      list with the slot's pre-chunk content.
//   5. Table: level L of [tmin, tile end) is last pushed by the LAST lane with amin <= L, so
//      lane t writes the levels [amin_t, min(aend_t, min of later lanes' amin)) of its
//      residual stack -- exactly one writer per level.
// Tile order is blockIdx order: the look-back waits only on lower workgroups, which the
// in-order dispatcher has already placed (a bounded spin latches ERR_CAPACITY instead of
// hanging). src: the chunk's records in a caller buffer (nrg_stack_round_async); the kernel
// then writes the log copy itself (Log::append fused). nullptr: records are in the ring.
__device__ __forceinline__ void st_tile_role(const StPass& A, const StPass& P, u32 tile, DevCtl* ctl,
                                             const u32* __restrict__ stack, u64 cap, int push_resp,
                                             u64* __restrict__ dbg) {
    const nrg_stack_op* __restrict__ src = A.src;
    nrg_stack_op* ring = A.ring;
    const u64 ring_mask = A.ring_mask, lo = A.lo, n = A.n, resp_lo = A.rlo, resp_hi = A.rhi;
    u64* desc = A.desc;
    const StTiles& tl = A.tl;
    u32* __restrict__ resp = A.resp;
    uint8_t* __restrict__ some = A.some;
    const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
    const u64 tbase = (u64)tile * ST_TILE;
    const u64 wbase = tbase + (u64)wv * (64 * SW_OPS);  // the wave's ops
    const u64 base = tbase + (u64)t * SW_OPS;           // the lane's ops
    const bool full = base + SW_OPS <= n;
#define ST_MARK(K) \
    if (dbg && t == 0) dbg[(u64)tile * 16 + (K)] = wall_clock64()
    ST_MARK(0);
    if (dbg && t == 0)  // placement: HW_ID (CU, SH, SE) and XCC_ID
        dbg[(u64)tile * 16 + 11] = (u64)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                                   (u64)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32;
    // per wave: the lane stacks (rows of 64 lanes; row SW_OPS absorbs non-Push writes) followed
    // by the wave's query list; the first 16 KB also stage the wave's ops on their way in
    constexpr int W_STK = (SW_OPS + 1) * 64, W_UP = 64 * SW_OPS;
    static_assert(W_STK + W_UP >= 2 * 64 * SW_OPS, "staging fits");
    __shared__ __attribute__((aligned(16))) u32 s_wave[ST_WAVES][W_STK + W_UP];
    __shared__ int s_min[ST_LANES];     // lane minimum level - tile minimum
    // s_sp[j][v + 1] = min of s_min over lanes (v - 2^j, v]; column 0 (lane -1) holds 0, below
    // every level, so a walk that has left the tile stops there without a branch
    __shared__ unsigned short s_sp[8][ST_LANES + 1];
    __shared__ int s_suf[ST_LANES];     // inclusive suffix minimum of s_min inside the wave
    __shared__ int s_wm[ST_WAVES], s_we[ST_WAVES], s_wmin[ST_WAVES], s_tot[ST_WAVES];
    __shared__ long long s_D, s_d0;
    __shared__ u32 s_ucnt;
    constexpr u32 ST_XL = 1024;
    __shared__ u32 s_xl[ST_XL];         // the first cross-tile Pops (the rest re-read from upop)
    __shared__ u32 s_pre[ST_LANES];     // pre-chunk content of levels T0 .. T0 + 255
    u32 (*s_stk)[64] = reinterpret_cast<u32 (*)[64]>(s_wave[wv]);
    u32* s_up = s_wave[wv] + W_STK;
    if (t == 0) s_ucnt = 0;
    // the previous chunk's tile minima: a slot it wrote (>= its lowest level) is read from its
    // owner's table, because that chunk's commit runs in this same launch
    extern __shared__ long long s_ptm[];
    long long* s_pg8 = s_ptm + P.tiles;
    long long* s_pgm = s_pg8 + P.tiles / 8 + 1;

    // ---- load the lane's ops (and write the log copy when they come from the caller) ----
    u32 val[SW_OPS];
    u32 pm = 0, qm = 0;  // Push / Pop bit per op (padding past n is neither)
    // the wave's records as loaded (16-B unit 64 i + lane): with a caller buffer their log copy
    // is written after the tile's aggregate is published, so the copy's HBM writes do not slow
    // the loads every later tile's look-back waits on
    uint4 x[SW_OPS / 2];
    const u64 rw0 = (lo + wbase) & ring_mask;
    const bool ring_run = rw0 + 64 * SW_OPS <= ring_mask + 1 && !(rw0 & 1);  // contiguous, 16-B aligned
    bool copy_later = false;
    {
        const nrg_stack_op* wp = src ? src + wbase : ring + rw0;
        const bool vec = wbase + 64 * SW_OPS <= n && (src ? !((uintptr_t)wp & 15) : ring_run);  // wave-uniform
        if (vec) {
            // coalesced: 16-B unit u = 64 i + lane of the wave's ops (two ops), then through LDS
            // to the lane that replays it (row u / 16, column (u % 16) ^ (row % 16): no conflicts)
            const uint4* p4 = (const uint4*)wp;
#pragma unroll
            for (int i = 0; i < SW_OPS / 2; i++) x[i] = p4[64 * i + lane];
            copy_later = src != nullptr;
            uint4* s4 = reinterpret_cast<uint4*>(s_wave[wv]);
            constexpr int UPR = SW_OPS / 2;  // 16-B units per lane
#pragma unroll
            for (int i = 0; i < SW_OPS / 2; i++) {
                const int u = 64 * i + lane, r = u / UPR;
                s4[r * UPR + ((u % UPR) ^ (r % UPR))] = x[i];
            }
            wave_sync();
#pragma unroll
            for (int j = 0; j < SW_OPS / 2; j++) {
                const uint4 y = s4[lane * UPR + (j ^ (lane % UPR))];
                val[2 * j] = y.x;
                val[2 * j + 1] = y.z;
                pm |= (u32)(y.y != 0) << (2 * j) | (u32)(y.w != 0) << (2 * j + 1);
                qm |= (u32)(y.y == 0) << (2 * j) | (u32)(y.w == 0) << (2 * j + 1);
            }
            wave_sync();  // the staging rows become the lane stacks
        } else {
            // partial last wave, a ring wrap or an unaligned caller buffer: 8-B op loads, still
            // coalesced and all in flight (op u = 64 i + lane of the wave), then through LDS
            // (row u / 32, column (u % 32) ^ (row % 32)) to the lane that replays it
            const u64 nw = n > wbase ? (n - wbase < 64 * SW_OPS ? n - wbase : 64 * SW_OPS) : 0;
            uint2* s2 = reinterpret_cast<uint2*>(s_wave[wv]);
#pragma unroll 8
            for (int i = 0; i < SW_OPS; i++) {
                const u32 u = 64 * i + lane;
                nrg_stack_op o{0, 0};  // past the chunk: masked out below
                if (u < nw) {
                    const u64 r = (lo + wbase + u) & ring_mask;
                    o = src ? src[wbase + u] : ring[r];
                    if (src) ring[r] = o;
                }
                const u32 row = u / SW_OPS;
                s2[row * SW_OPS + ((u % SW_OPS) ^ (row % SW_OPS))] = uint2{o.val, o.op};
            }
            wave_sync();
#pragma unroll
            for (int q = 0; q < SW_OPS; q++) {
                const uint2 y = s2[lane * SW_OPS + (q ^ (lane % SW_OPS))];
                const bool in = (u32)(lane * SW_OPS + q) < nw;
                val[q] = y.x;
                pm |= (u32)(in && y.y != 0) << q;
                qm |= (u32)(in && y.y == 0) << q;
            }
            wave_sync();  // the staging rows become the lane stacks
        }
    }
    ST_MARK(1);

    // ---- 1. local pass (branch-free: no per-op lane masks held in SGPRs) ----
    u32 rt[SW_OPS];  // what each Pop read from the local stack (valid for matched Pops)
    u32 top = 0, nun = 0, umask = 0, topmax = 0;
    int hmax = 0;
#pragma unroll
    for (int q = 0; q < SW_OPS; q++) {
        const u32 pu = (pm >> q) & 1u, po = (qm >> q) & 1u;
        s_stk[SW_OPS + pu * (top - SW_OPS)][lane] = val[q];
        rt[q] = s_stk[min(top - 1u, (u32)SW_OPS)][lane];
        const u32 un = (u32)max((int)po - (int)top, 0);  // a Pop on the empty local stack
        umask |= un << q;
        nun += un;
        top = top + pu - po + un;
        topmax = max(topmax, top);
        hmax = max(hmax, (int)top - (int)nun);
    }
    // fold the known responses into rt[] (val[] dies here): Push -> its value if Push answers
    // Some, matched Pop -> what it read, everything else None (unmatched Pops are patched later)
    const u32 smask = (push_resp ? pm : 0u) | (qm & ~umask);
#pragma unroll
    for (int q = 0; q < SW_OPS; q++) {
        const u32 pq = (u32)__builtin_amdgcn_sbfe((int)pm, q, 1);
        rt[q] = ((val[q] & pq) | (rt[q] & ~pq)) & (u32)__builtin_amdgcn_sbfe((int)smask, q, 1);
    }
    ST_MARK(2);

    // ---- 2. scan of (m, e): inclusive over the wave, then the wave totals ----
    int im = -(int)nun, ie = (int)top - (int)nun;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int om = __shfl_up(im, off, 64), oe = __shfl_up(ie, off, 64);
        if (lane >= off) {
            int m = om, e = oe;
            me_then(m, e, im, ie);
            im = m;
            ie = e;
        }
    }
    if (lane == 63) {
        s_wm[wv] = im;
        s_we[wv] = ie;
    }
    int xm = __shfl_up(im, 1, 64), xe = __shfl_up(ie, 1, 64);  // exclusive within the wave
    if (lane == 0) xm = xe = 0;
    __syncthreads();
    int M = 0, E = 0, pmw = 0, pew = 0;  // tile aggregate; prefix of the earlier waves
#pragma unroll
    for (int w = 0; w < ST_WAVES; w++) {
        if (w == wv) {
            pmw = M;
            pew = E;
        }
        me_then(M, E, s_wm[w], s_we[w]);
    }
    me_then(pmw, pew, xm, xe);  // the lane's exclusive prefix within the tile
    xm = pmw;
    xe = pew;
    const Fn tagg = {E, E - M};  // max(a, x + b) form for the look-back
    if (t == 0) __hip_atomic_store(&desc[tile], pack_agg(tagg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ST_MARK(15);  // published
    if (copy_later) {  // Log::append's copy of the wave's records
        if (ring_run) {
            uint4* w4 = (uint4*)(ring + rw0);
            if (!A.plain) {
#pragma unroll
                for (int i = 0; i < SW_OPS / 2; i++) nt_store4(&w4[64 * i + lane], x[i]);
            } else {
#pragma unroll
                for (int i = 0; i < SW_OPS / 2; i++) w4[64 * i + lane] = x[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < SW_OPS / 2; i++) {
                const u64 o = lo + wbase + 2 * (64 * i + lane);
                ring[o & ring_mask] = nrg_stack_op{x[i].x, x[i].y};
                ring[(o + 1) & ring_mask] = nrg_stack_op{x[i].z, x[i].w};
            }
        }
    }

    // responses known now, lane-contiguous (unmatched Pops stay None until patched below)
    {
        const u64 g0 = lo + base;
        const bool in = full && g0 >= resp_lo && g0 + SW_OPS <= resp_hi;
        u32* rp = resp + (g0 - resp_lo);
        uint8_t* sp = some + (g0 - resp_lo);
        if (in && !((uintptr_t)rp & 15) && !((uintptr_t)sp & (SW_OPS >= 16 ? 15 : 7))) {
            if (!A.plain) {
#pragma unroll
                for (int j = 0; j < SW_OPS / 4; j++)
                    nt_store4(&((uint4*)rp)[j], uint4{rt[4 * j], rt[4 * j + 1], rt[4 * j + 2], rt[4 * j + 3]});
            } else {
#pragma unroll
                for (int j = 0; j < SW_OPS / 4; j++)
                    ((uint4*)rp)[j] = uint4{rt[4 * j], rt[4 * j + 1], rt[4 * j + 2], rt[4 * j + 3]};
            }
            if constexpr (SW_OPS >= 16) {
#pragma unroll
                for (int j = 0; j < SW_OPS / 16; j++) {
                    uint4 b;
                    u32* bb = (u32*)&b;
#pragma unroll
                    for (int k = 0; k < 4; k++) bb[k] = (((smask >> (16 * j + 4 * k)) & 15u) * 0x204081u) & 0x01010101u;
                    ((uint4*)sp)[j] = b;
                }
            } else {  // 8 ops per lane: one 8-B store
                const uint2 b = uint2{((smask & 15u) * 0x204081u) & 0x01010101u,
                                      (((smask >> 4) & 15u) * 0x204081u) & 0x01010101u};
                st_pol<NRG_ST_SOME_NT>((u64*)sp, (u64)b.x | ((u64)b.y << 32));
            }
        } else if (resp) {
#pragma unroll
            for (int q = 0; q < SW_OPS; q++) {
                const u64 g = g0 + q;
                if (base + q < n && g >= resp_lo && g < resp_hi) {
                    st_resp(&resp[g - resp_lo], rt[q], A.plain);
                    st_pol<NRG_ST_SOME_NT>(&some[g - resp_lo], (uint8_t)((smask >> q) & 1));
                }
            }
        }
    }
    ST_MARK(3);

    // ---- 3. look-back (wave 0): compose the aggregates of ALL earlier tiles (64 runs in
    // parallel, 8 loads in flight per lane; the highest lane holds the oldest run). The query
    // structures are built first: they need the tile's start depth only when the stack empties
    // inside the tile, so they are built for the unclamped walk and rebuilt in that (rare) case.
    // Round 6: no global load is waited on between the aggregate's publication and the
    // query-structure barrier (the look-back's first loads and the previous chunk's tile minima are
    // issued after it): 3.9 -> 2.3 us from publication to query structures, 14.83-14.95 -> 14.22-14.26
    // us per 1M-op round (profiles/r06/stack_lookback_after_build.txt). ----
    long long* sdepth = &ctl->depth0;             // depth after the chunk of each parity
    const int np = (int)tile;
    const int G = (np + 63) / 64;
    const int r0 = (63 - lane) * G;
    constexpr int B = 8;

    // Query structures for lane levels relative to the tile's lowest level: lane minimum amin_,
    // start dt_, and uq_ unmatched Pops that find an element. Outputs: s_min, the sparse table
    // s_sp, `later` (minimum over the later lanes) and the wave's query list s_up[0, total).
    int later = 0, total = 0;
    auto build = [&](int amin_, int dt_, int uq_) {
        s_min[t] = amin_;
        // sparse table: levels 0..6 inside the wave (windows clipped at the wave's first lane;
        // the part in earlier waves is added below), inclusive suffix minimum inside the wave
        int spw[7];
        spw[0] = amin_;
#pragma unroll
        for (int j = 1; j < 7; j++) {
            const int o = __shfl_up(spw[j - 1], 1 << (j - 1), 64);
            spw[j] = lane >= (1 << (j - 1)) && o < spw[j - 1] ? o : spw[j - 1];
        }
        int sf = amin_;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_down(sf, off, 64);
            if (lane + off < 64) sf = o < sf ? o : sf;
        }
        later = __shfl_down(sf, 1, 64);
        if (lane == 63) later = 1 << 30;
        s_suf[t] = sf;
        if (lane == 0) s_wmin[wv] = sf;
        // the wave's query list: lane t's unmatched Pops k < uq_
        int inc = uq_;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int o = __shfl_up(inc, off, 64);
            if (lane >= off) inc += o;
        }
        total = __shfl(inc, 63, 64);
        if (lane == 0) s_tot[wv] = total;
        {
            u32 um = umask;
            for (int k = 0, h = inc - uq_; k < uq_; k++, h++) {
                const int q = __builtin_ctz(um);
                um &= um - 1;
                s_up[h] = ((u32)(dt_ - 1 - k) << ST_PB) | ((u32)t * SW_OPS + (u32)q);
            }
        }
        __syncthreads();
        // complete the windows (t - 2^j, t] that reach into earlier waves: a suffix of the
        // previous wave (its inclusive suffix minimum) and, for level 7, whole waves before it
#pragma unroll
        for (int j = 0; j < 7; j++) {
            int m = spw[j];
            if (wv > 0 && lane < (1 << j) - 1) {
                const int o = s_suf[t - (1 << j) + 1];
                m = o < m ? o : m;
            }
            s_sp[j][t + 1] = (unsigned short)m;  // levels are < 2 * ST_TILE
        }
        int m7 = spw[6];
        if (wv > 0) m7 = s_wmin[wv - 1] < m7 ? s_wmin[wv - 1] : m7;
        if (wv > 1 && lane < 63) m7 = s_suf[t - 127] < m7 ? s_suf[t - 127] : m7;
        s_sp[7][t + 1] = (unsigned short)m7;
        if (t < 8) s_sp[t][0] = 0;
        for (int w = wv + 1; w < ST_WAVES; w++) later = s_wmin[w] < later ? s_wmin[w] : later;
    };
    // unclamped walk (D + M >= 0): amin = xe - nun - M, start xe - M, every unmatched Pop reads
    build(xe - (int)nun - M, xe - M, (int)nun);

    // ---- 4. unmatched Pops: QI queries per lane at a time, their table walks interleaved. The
    // queries of wave `lw`'s list, entries h = slot*64*QI + lane + k*64*QI*nslots (a wave answers
    // its own list, or a share of another wave's). Everything here is relative to the tile's
    // lowest level: with the unclamped structures nothing depends on the start depth D. ----
    constexpr int QI = 4;
    auto queries = [&](int lw, int slot, int nslots) {
        test_stall(A.stall & 1, wv);  // (tests) slow waves read the query structures below
        const u32* up = s_wave[lw] + W_STK;
        const int tot = s_tot[lw];
        for (int h0 = slot * 64 * QI + lane; h0 < tot; h0 += 64 * QI * nslots) {
            u32 e[QI];
            int v[QI];
#pragma unroll
            for (int i = 0; i < QI; i++) {
                const int h = h0 + 64 * i;
                e[i] = h < tot ? up[h] : 0u;
                v[i] = h < tot ? (int)((e[i] & ST_PMASK) / SW_OPS) - 1 : -1;
            }
            // the nearest earlier lane whose minimum is <= the level (greedy skips of 128, ..., 1);
            // branch-free, so each level's QI table reads are in flight together (predicated reads
            // compiled to one LDS round trip per query and level: 2.5 us for a 4096-op tile)
#pragma unroll
            for (int j = 7; j >= 0; j--) {
                int m[QI];
#pragma unroll
                for (int i = 0; i < QI; i++) m[i] = (int)s_sp[j][v[i] + 1];
#pragma unroll
                for (int i = 0; i < QI; i++) {
                    const int w = v[i] - (m[i] > (int)(e[i] >> ST_PB) ? 1 << j : 0);
                    v[i] = w > -1 ? w : -1;
                }
            }
            // the found lanes' residual entries, read together (lane 0's column for the others)
            int mn[QI];
            u32 rv[QI];
#pragma unroll
            for (int i = 0; i < QI; i++) mn[i] = s_min[v[i] > 0 ? v[i] : 0];
#pragma unroll
            for (int i = 0; i < QI; i++) {
                const int vv = v[i] > 0 ? v[i] : 0;
                rv[i] = s_wave[vv >> 6][v[i] >= 0 ? ((int)(e[i] >> ST_PB) - mn[i]) * 64 + (vv & 63) : 0];
            }
#pragma unroll
            for (int i = 0; i < QI; i++) {
                if (h0 + 64 * i >= tot) continue;
                const u32 pos = e[i] & ST_PMASK;
                if (v[i] >= 0) {
                    const u64 g = lo + tbase + pos;
                    if (resp && g >= resp_lo && g < resp_hi) {
                        st_resp(&resp[g - resp_lo], rv[i], A.plain);
                        st_pol<NRG_ST_SOME_NT>(&some[g - resp_lo], (uint8_t)1);
                    }
                } else {  // its Push is in an earlier tile or before the chunk
                    const u32 x = atomicAdd(&s_ucnt, 1u);
                    tl.upop[(u64)tile * ST_TILE + x] = e[i];
                    if (x < ST_XL) s_xl[x] = e[i];
                }
            }
        }
    };

    ST_MARK(12);  // query structures built (wave 0 starts its look-back wait)
    if (wv == 0) {
        // the previous chunk's tile minima (read only by the pre-chunk pass, after the queries):
        // copied into LDS beside the look-back's loads, whose waits cover the copy; the group minima
        // are staged from LDS after the look-back. (Loaded before the query structures, their
        // latency held that barrier.)
        if (P.tiles) st_copy_lds(P.tl.tmin, P.tiles, s_ptm);
        // the look-back's first loads: issued only now, so no wait before the query-structure
        // barrier covers them (agent-scope loads, served beyond the XCD's L2)
        const long long d0g = sdepth[A.par ^ 1];
        u64 v0[B];
#pragma unroll
        for (int q = 0; q < B; q++) {
            const int idx = r0 + q;
            v0[q] = (q < G && idx < np) ? __hip_atomic_load(&desc[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        }
        Fn acc = FN_ID;
        for (int g0 = 0; g0 < G; g0 += B) {
            u64 v[B];
#pragma unroll
            for (int q = 0; q < B; q++) {
                const int idx = r0 + g0 + q;
                v[q] = g0 == 0 ? v0[q]
                               : ((g0 + q < G && idx < np)
                                      ? __hip_atomic_load(&desc[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                      : 0ull);
            }
            // predecessors publish right after their local pass: re-poll only what is missing
            for (u32 spins = 0;; spins++) {
                bool ok = true;
#pragma unroll
                for (int q = 0; q < B; q++) ok &= g0 + q >= G || r0 + g0 + q >= np || (v[q] & D_MASK);
                if (ok) break;
                if (spins == (1u << 24)) {  // bounded: never hang the device
                    atomicOr(&ctl->err, ERR_CAPACITY);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
#pragma unroll
                for (int q = 0; q < B; q++) {
                    const int idx = r0 + g0 + q;
                    if (g0 + q < G && idx < np && !(v[q] & D_MASK))
                        v[q] = __hip_atomic_load(&desc[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
#pragma unroll
            for (int q = 0; q < B; q++)
                if (g0 + q < G && r0 + g0 + q < np) acc = fn_then(acc, unpack_agg(v[q]));
        }
        acc = np ? wave_compose(acc) : Fn{0, 0};
        ST_MARK(13);  // look-back resolved
        if (lane == 0) {
            s_D = fn_apply(acc, d0g);
            s_d0 = d0g;
        }
    } else {
        // while wave 0 waits on the look-back the other waves answer every wave's unmatched Pops
        // for the unclamped walk -- their own lists, then a share of wave 0's
        queries(wv, 0, 1);
        queries(0, wv - 1, ST_WAVES - 1);
        if (dbg && t == 64) dbg[(u64)tile * 16 + 14] = wall_clock64();  // wave 1's queries done
    }
    __syncthreads();
    ST_MARK(4);
    if (P.tiles) (void)st_stage(P.tl.tmin, P.tiles, s_ptm, s_pg8, s_pgm, ~0u, true);
    const long long D = s_D, d0 = s_d0;
    const long long T0 = D + M > 0 ? D + M : 0;              // the tile's lowest level
    const long long Dt = D + xe > xe - xm ? D + xe : xe - xm;  // the lane's start depth
    const long long aminl = Dt - (long long)nun > 0 ? Dt - (long long)nun : 0;
    const int amin = (int)(aminl - T0);  // levels relative to T0 from here on
    const int dt = (int)(Dt - T0);
    const int aend_r = amin + (int)top;  // the lane's end depth: max(Dt + e, top) - T0
    if (t == ST_LANES - 1 && tile == A.tiles - 1) sdepth[A.par] = T0 + aend_r;
    if (Dt + hmax > (long long)cap || (long long)topmax > (long long)cap) atomicOr(&ctl->err, ERR_CAPACITY);
    // the stack empties inside the tile (block-uniform, rare): Pops at depth 0 are no-ops and
    // levels shift, so the speculative answers are withdrawn -- every unmatched Pop back to None,
    // the cross-tile list emptied -- and the queries run again on the clamped structures
    const bool clamped = D + M < 0;
    if (clamped) {
        const u64 g0 = lo + base;
        for (u32 um = umask; um; um &= um - 1) {
            const u64 g = g0 + (u64)__builtin_ctz(um);
            if (resp && g >= resp_lo && g < resp_hi) {
                st_resp(&resp[g - resp_lo], 0u, A.plain);
                st_pol<NRG_ST_SOME_NT>(&some[g - resp_lo], (uint8_t)0);
            }
        }
        if (t == 0) s_ucnt = 0;
        __syncthreads();
        build(amin, dt, (int)(Dt < (long long)nun ? Dt : (long long)nun));
        queries(wv, 0, 1);
    }
    // The cross-tile Pops read exactly the levels [T0, D), each on the tile's first descent below
    // it. Their pre-chunk content: a slot the previous chunk wrote comes from its owner's table
    // (that chunk's commit runs in this launch), any other from the stack. Fetched now for the
    // first 256 levels, one per thread, so the loads land while the queries run.
    auto pre_content = [&](long long slot) -> u32 {
        if (slot >= d0 || (u64)slot >= cap) return 0u;
        const int k = P.tiles ? st_find(s_ptm, s_pg8, s_pgm, (int)P.tiles, slot) : -1;
        return k >= 0 ? P.tl.table[(u64)k * ST_TILE + (u64)(slot - s_ptm[k])] : stack[slot];
    };
    __syncthreads();
    ST_MARK(5);
    const u32 pre = t < D - T0 ? pre_content(T0 + t) : 0u;  // after the barrier: its fence would wait
    ST_MARK(9);

    if (dbg && t == 0) dbg[(u64)tile * 16 + 10] = (u64)total;
    s_pre[t] = pre;
    __syncthreads();
    // the cross-tile Pops' pre-chunk content (prefetched for the first 256 levels)
    ST_MARK(8);  // queries done (stored after the phases 0..7)
    const u32 ucnt = s_ucnt;
    for (u32 h = t; h < ucnt; h += ST_LANES) {
        const u32 e = h < ST_XL ? s_xl[h] : tl.upop[(u64)tile * ST_TILE + h];
        const u32 lr = e >> ST_PB;
        tl.uval[(u64)tile * ST_TILE + h] = lr < (u32)ST_LANES ? s_pre[lr] : pre_content(T0 + (long long)lr);
    }
    ST_MARK(6);

    // ---- 5. the tile's last-Push table for levels [T0, tile end) ----
    test_stall(A.stall & 1, wv);  // (tests) slow waves read their lane stacks below
    {
        u32* tab = tl.table + (u64)tile * ST_TILE;
        const int hi = aend_r < later ? aend_r : later;
        for (int L = amin; L < hi; L++) tab[L] = s_stk[L - amin][lane];
    }
    if (t == ST_LANES - 1) {
        tl.tmin[tile] = T0;
        tl.tend[tile] = (u32)aend_r;
        tl.ucnt[tile] = ucnt;
    }
    ST_MARK(7);
#undef ST_MARK
}

// The finish of chunk P, one workgroup per tile: with all tile minima staged in LDS it
//   * commits: the tile's levels [tmin, min(end depth, min of every later tile's minimum)) are
//     the slots whose last Push of the chunk is this tile's, held in its table;
//   * resolves the tile's Pops whose Push lies in an earlier tile: the nearest earlier tile
//     whose minimum is <= the slot (a walk that skips 8- and 64-tile groups whose minimum is
//     above the slot), or the pre-chunk content the tile pass read.
// Tile 0 publishes the chunk's end depth as the stack's length.
__device__ __forceinline__ void st_finish_role(const StPass& P, u32 tile, DevCtl* ctl, u32* __restrict__ stack,
                                               u64 cap) {
    extern __shared__ long long s_tm[];  // [tiles] tile minima, [tiles/8 + 1] and [tiles/64 + 1] group minima
    __shared__ long long s_lo[4];
    const u32 tiles = P.tiles;
    const StTiles& tl = P.tl;
    const u64 lo = P.lo, resp_lo = P.rlo, resp_hi = P.rhi;
    u32* __restrict__ resp = P.resp;
    uint8_t* __restrict__ some = P.some;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    // independent loads first: they overlap the staging below
    const u32 cnt = resp ? tl.ucnt[tile] : 0u;
    const u32 v0 = tl.upop[(u64)tile * ST_TILE + t];
    const u32 uv0 = tl.uval[(u64)tile * ST_TILE + t];
    const u32 tend = tl.tend[tile];
    if (t == 0) P.desc[tile] = 0;  // ready for the next chunk of this parity
    long long* s_g8 = s_tm + tiles;
    long long* s_gm = s_g8 + tiles / 8 + 1;
    long long later = st_stage(tl.tmin, tiles, s_tm, s_g8, s_gm, tile);  // minimum over the later tiles
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const long long x = __shfl_xor(later, off, 64);
        later = x < later ? x : later;
    }
    if (lane == 0) s_lo[w] = later;
    __syncthreads();
    if (tile == 0 && t == 0) ctl->depth = (&ctl->depth0)[P.par];
    for (int i = 0; i < 4; i++) later = s_lo[i] < later ? s_lo[i] : later;
    const long long tmin = s_tm[tile];
    // cross-tile Pops first (their table loads), then the commit, then the answers: the loads of
    // both are in flight together
    u32 pval = 0;
    u64 pg = ~0ull;
    const bool one = cnt <= 256;  // the common case: one Pop per thread
    if (one && (u32)t < cnt) {
        const u64 g = lo + (u64)tile * ST_TILE + (v0 & ST_PMASK);
        if (g >= resp_lo && g < resp_hi) {
            const long long s = tmin + (v0 >> ST_PB);
            const int k = st_walk(s_tm, s_g8, s_gm, (int)tile - 1, s);
            pval = k >= 0 ? tl.table[(u64)k * ST_TILE + (u64)(s - s_tm[k])] : uv0;
            pg = g;
        }
    }
    {
        long long hi = tmin + (long long)tend;
        hi = hi < later ? hi : later;
        const u32* tab = tl.table + (u64)tile * ST_TILE;
        for (long long sl = tmin + t; sl < hi; sl += 256)
            if ((u64)sl < cap) st_pol<NRG_ST_FIN_NT>(&stack[sl], tab[sl - tmin]);
    }
    if (pg != ~0ull) {
        st_pol<NRG_ST_FIN_NT>(&resp[pg - resp_lo], pval);
        st_pol<NRG_ST_FIN_NT>(&some[pg - resp_lo], (uint8_t)1);
    }
    if (!one) {
        for (u32 j = t; j < cnt; j += 256) {
            const u32 v = j == (u32)t ? v0 : tl.upop[(u64)tile * ST_TILE + j];
            const u64 g = lo + (u64)tile * ST_TILE + (v & ST_PMASK);
            if (g < resp_lo || g >= resp_hi) continue;
            const long long s = tmin + (v >> ST_PB);
            const int k = st_walk(s_tm, s_g8, s_gm, (int)tile - 1, s);
            st_pol<NRG_ST_FIN_NT>(&resp[g - resp_lo], k >= 0 ? tl.table[(u64)k * ST_TILE + (u64)(s - s_tm[k])]
                                                        : (j == (u32)t ? uv0 : tl.uval[(u64)tile * ST_TILE + j]));
            st_pol<NRG_ST_FIN_NT>(&some[g - resp_lo], (uint8_t)1);
        }
    }
}

__global__ __launch_bounds__(ST_LANES) void st_round_kernel(StPass A, StPass P, DevCtl* ctl, u32* __restrict__ stack,
                                                           u64 cap, int push_resp, u64* __restrict__ dbg) {
    // tile workgroups first: the dispatcher places workgroups in order, and the finish
    // workgroups (independent of this launch's tiles) fill in behind them
    if (blockIdx.x < A.tiles) {
        st_tile_role(A, P, blockIdx.x, ctl, stack, cap, push_resp, dbg);
    } else {
        const u32 f = blockIdx.x - A.tiles;
        // diagnostic (NRG_EXP & 2): finish workgroups' start/end at dbg[(128 + tile) * 16 + {0, 1}]
        if (dbg && threadIdx.x == 0 && f < 128) dbg[(128 + f) * 16] = wall_clock64();
        st_finish_role(P, f, ctl, stack, cap);
        if (dbg && threadIdx.x == 0 && f < 128) dbg[(128 + f) * 16 + 1] = wall_clock64();
    }
}

static u64 st_max_tiles(const nrg_ctx* c) { return (c->cfg.max_batch + ST_TILE - 1) / ST_TILE; }

static u64 st_parity_bytes(u64 mt) { return mt * (8 + 4 + 4) + mt * ST_TILE * (4 + 4 + 4); }

// the per-tile buffers and look-back descriptors of parity `par`
static StPass st_pass(nrg_ctx* c, u32 par) {
    const u64 mt = st_max_tiles(c);
    StPass s{};
    s.par = par;
    s.stall = c->stall;
    s.plain = (c->exp >> 6) & 1;
    s.ring = (nrg_stack_op*)c->d_ring;
    s.ring_mask = c->log_size - 1;
    // descriptors: [32 u64 unused] [parity][max tiles] u64; zero at open, and each chunk's finish
    // clears what its tile pass used (no memset launch per chunk)
    s.desc = (u64*)c->d_scan_desc + 32 + par * mt;
    char* base = (char*)c->d_st_aux + par * st_parity_bytes(mt);
    s.tl.tmin = (long long*)base;
    s.tl.ucnt = (u32*)(s.tl.tmin + mt);
    s.tl.tend = s.tl.ucnt + mt;
    s.tl.upop = s.tl.tend + mt;
    s.tl.uval = s.tl.upop + mt * ST_TILE;
    s.tl.table = s.tl.uval + mt * ST_TILE;
    return s;
}

static hipError_t st_launch(nrg_ctx* c, const StPass& A, const StPass& P) {
    const unsigned grid = A.tiles + P.tiles;
    const size_t dyn = P.tiles ? (size_t)(P.tiles + P.tiles / 8 + P.tiles / 64 + 2) * 8 : 0;
    st_round_kernel<<<grid, ST_LANES, dyn, c->stream>>>(A, P, c->d_ctl, c->d_stack, c->cfg.stack_capacity,
                                                         (int)c->cfg.stack_push_resp, (c->exp & 2) ? c->d_dbg : nullptr);
    return hipGetLastError();
}

// The finish of the last replayed chunk (its cross-tile Pops and its commit), if still pending.
hipError_t st_flush(nrg_ctx* c) {
    if (!c->st_pend.valid) return hipSuccess;
    StPass P = st_pass(c, c->st_pend.par);
    P.lo = c->st_pend.lo;
    P.n = c->st_pend.n;
    P.tiles = c->st_pend.tiles;
    P.rlo = c->st_pend.rlo;
    P.rhi = c->st_pend.rhi;
    P.resp = c->st_pend.resp;
    P.some = c->st_pend.some;
    c->st_pend.valid = false;
    StPass A{};
    return st_launch(c, A, P);
}

// One chunk: its tile pass, fused with the previous chunk's finish in one launch. The chunk's
// own finish runs in the next chunk's launch (config.pipeline = 1, until nrg_join or a sync)
// or right away.
hipError_t st_replay_chunk(nrg_ctx* c, u64 lo, u64 n, u64 resp_lo, u64 resp_hi, uint32_t* d_resp, uint8_t* d_some,
                           const nrg_stack_op* src) {
    if (n == 0) return st_flush(c);  // an empty round still completes the last round's deferred finish
    StPass A = st_pass(c, c->st_par);
    A.src = src;
    A.lo = lo;
    A.n = n;
    A.tiles = (u32)((n + ST_TILE - 1) / ST_TILE);
    const bool want = d_resp != nullptr && resp_lo < lo + n && resp_hi > lo;
    A.rlo = want ? resp_lo : 0;
    A.rhi = want ? resp_hi : 0;
    A.resp = want ? d_resp : nullptr;
    A.some = want ? d_some : nullptr;
    StPass P{};
    if (c->st_pend.valid) {
        P = st_pass(c, c->st_pend.par);
        P.lo = c->st_pend.lo;
        P.n = c->st_pend.n;
        P.tiles = c->st_pend.tiles;
        P.rlo = c->st_pend.rlo;
        P.rhi = c->st_pend.rhi;
        P.resp = c->st_pend.resp;
        P.some = c->st_pend.some;
    }
    timer_begin(c, "st_replay");
    hipError_t e = st_launch(c, A, P);
    timer_end(c, "st_replay");
    if (e != hipSuccess) return e;
    c->st_pend = StDeferred{true, lo, n, A.tiles, A.par, A.rlo, A.rhi, A.resp, A.some};
    c->st_par ^= 1;
    return c->pipeline ? hipSuccess : st_flush(c);
}

// [32 u64 unused] [parity][max tiles] u64 (st_pass)
u64 st_desc_words(u64 max_batch) { return 2 * (32 + 2 * ((max_batch + ST_TILE - 1) / ST_TILE)); }

u64 st_aux_bytes(u64 max_batch) { return 2 * st_parity_bytes((max_batch + ST_TILE - 1) / ST_TILE); }

}  // namespace nrg
