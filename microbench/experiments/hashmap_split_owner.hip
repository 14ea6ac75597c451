// hashmap.hip — NrHashMap replica replay on gfx950.
//
// Replaces the hot loop of Log::exec -> NrHashMap::dispatch_mut (nr/src/log.rs:494-518,
// benches/hashmap.rs:114-119, nr/examples/hashmap.rs:46-50) and the read path
// Replica::read_only -> dispatch (nr/src/replica.rs:483-497, benches/hashmap.rs:107-111).
//
// Table: 2^k open-addressing slots of 64 B (common.hpp), linear probing from
// mix64(key) >> (64 - k). A replay round covers the log records [lo, lo+n) and gets a fresh
// epoch e (never reused). A round goes through three stages:
//
//   split(e)   per Put: bin the Put by its key's slot range (bucket = top log2b bits of the
//              home slot) with a counting sort local to each tile of st Puts (LDS counters,
//              no global atomics); writes the log copy when the round was handed over in a
//              caller buffer. Output: items binned per (bucket, tile) + counts and offsets.
//   index(e)   one owner block per bucket gathers every Put of its slot range, finds the key's
//              slot or claims an empty one with a 64-bit CAS (created = e), and elects the
//              round's last writer of each key in LDS. As no other block holds Puts of those
//              keys, the election is exact: stamp[e&1] = e<<32 | i+1 is a plain store and the
//              winner is flagged in put_flag. A bucket with more Puts than one block takes
//              (Zipf hot keys) is shared by several blocks, which pre-combine in LDS and use
//              atomicMax; its winners are flagged "check the stamp".
//   apply(e)   flagged winners store their value (checked ones compare the stamp first).
//   reads(e)   per Get, against the state after round e: a key counts iff 0 < created <= e;
//              its value is the round's elected record when stamp[e&1] carries epoch e
//              (apply(e) may still be storing it), else the slot's value.
//
// All roles live in ONE kernel (hm_round_kernel, disjoint block ranges), launched as
// {index(e-1)} + {split(e)} + {apply(e-2) + reads(e-2)}: the latency-bound index pass overlaps
// the bandwidth-bound reads. Race-free because index(e-1) only claims empty slots (invisible to
// reads(e-2): created is 0 or e-1) and writes stamp[(e-1)&1], while apply/reads(e-2) look only
// at stamp[e&1] and at values that index never writes; split touches no table state.
// Scattered device-scope atomics run at ~20 G requests/s on MI355X; the previous design (one
// atomicMax per Put) spent 26 of 70 us of a 50 %-write round on them
// (profiles/r01_put_breakdown.txt). The result equals the sequential replay: last-writer-wins
// per key in log order, reads after the round's writes (SURVEY.md §8a round semantics).
#include "internal.hpp"

namespace nrg {

constexpr int TPB = 256;
constexpr u32 SIDE_SLOT = 0xFFFFFFFFu;  // put_slot value of the EMPTY_KEY key (side slot)
constexpr u32 FULL_SLOT = 0xFFFFFFFEu;  // put_slot value of a Put that found no slot
constexpr uint8_t FLAG_WIN = 1;         // the round's last writer of its key: store the value
constexpr uint8_t FLAG_CHECK = 2;       // may be the last writer: store iff the stamp is its own

// owner (index) role geometry
constexpr int OW_IPT = 4;                // Puts per thread per pass
constexpr int OW_PASS = TPB * OW_IPT;    // Puts per pass
constexpr int OW_LDS = 2 * OW_PASS;      // election table entries (load <= 1/2)
constexpr u32 OW_CHUNK = 4096;           // Puts one owner block takes before a bucket is shared
constexpr u32 OW_MMAX = HM_MAX_OWNERS_PER_BUCKET;  // most owner blocks per bucket
// LDS shared by all roles (one array, so the read role keeps its occupancy)
constexpr int SMEM_WORDS = 2 * OW_LDS + 3 * (int)HM_MAX_TILES + 16;

__device__ __forceinline__ u64 stamp_of(u32 epoch, u64 i) { return ((u64)epoch << 32) | (i + 1); }

// record i of a round: from a caller's buffer when given, else from the log ring
struct RecSrc {
    const nrg_put* src;
    const nrg_put* ring;
    u64 mask, lo;
    __device__ __forceinline__ nrg_put at(u64 i) const { return src ? src[i] : ring[(lo + i) & mask]; }
};

struct SplitJob {
    RecSrc rec;
    nrg_put* ring_out;  // log copy to write (nullptr: records already in the ring)
    u64 n;
    PutItem* items;
    u32* bin_cnt;  // [bucket][tile]
    u32* bin_off;
    uint8_t* put_flag;  // zeroed here (coalesced) for the round's owners to flag winners
    u32 st, ntiles, log2b;
    u32 nblocks;
};
struct OwnerJob {
    const PutItem* items;
    const u32* bin_cnt;
    const u32* bin_off;
    u32* put_slot;      // winners always; every Put when all_slots (previous-value responses)
    uint8_t* put_flag;  // zeroed by the split; winners flagged here
    u32 st, ntiles, log2b;
    u32 epoch;
    u32 nblocks;
    u32 all_slots;
    u64* created_acc;  // [HM_MAX_BUCKETS * OW_MMAX] keys created per owner block, summed by hm_count
    u32 exp;           // diagnostic knobs (NRG_EXP; results wrong): 1 stop after gather, 2 no probe, 4 no publish
};
struct ApplyJob {
    RecSrc rec;
    u64 n;
    const u32* put_slot;
    const uint8_t* put_flag;
    u32 epoch;
    u32 nblocks;
};
struct ReadJob {
    RecSrc rec;  // records of round `epoch` (used while its apply may be in flight); src=ring=0: none
    const u64* keys;
    u64 R;
    u64* vals;
    uint8_t* found;
    u32 epoch;
    u32 nblocks;
};

// What a read needs of a slot: two 16-B loads to the same 128-B line, {key, val} and
// {stamp1, created} (odd epochs) or {created, stamp0} (even epochs), issued together. The
// empty asm pins the values at this point: otherwise hipcc sinks the second load below the
// key compare of the probe loop, turning a Get into two dependent accesses.
struct View {
    u64 key, val, st;
    u32 created;
};
__device__ __forceinline__ View load_view(const Slot* p, u32 par) {
    typedef u64 u64x2 __attribute__((ext_vector_type(2)));
    const u64x2 a = *(const u64x2*)p;
    const u64x2 b = *(const u64x2*)((const char*)p + (par ? 16 : 24));
    u64 k = a.x, v = a.y;
    u64 st = par ? b.x : b.y;
    u32 cr = (u32)(par ? b.y : b.x);
    asm volatile("" : "+v"(k), "+v"(v), "+v"(st), "+v"(cr));
    View w;
    w.key = k;
    w.val = v;
    w.st = st;
    w.created = cr;
    return w;
}

// The value a read of epoch ep sees in a slot (or side slot) holding its key.
__device__ __forceinline__ bool resolve(View w, u32 ep, RecSrc rec, bool use_rec, u64* v) {
    if (w.created == 0 || w.created > ep) return false;  // inserted by a later round (or claiming)
    if (use_rec && (u32)(w.st >> 32) == ep)
        *v = rec.at((u64)(u32)w.st - 1).val;  // written in round ep; apply(ep) may be in flight
    else
        *v = w.val;
    return true;
}

// find-or-claim k from slot s (its key already loaded as key0); returns slot or -1 if full
__device__ __forceinline__ long long find_or_claim(Slot* table, u64 k, u64 s, u64 tmask, u64 key0, u32 epoch,
                                                   u32* created) {
    u64 key = key0;
    for (u64 pr = 0; pr <= tmask; pr++) {
        if (key == k) return (long long)s;
        if (key == EMPTY_KEY) {
            const u64 old = atomicCAS(&table[s].key, EMPTY_KEY, k);
            if (old == EMPTY_KEY) {
                table[s].created = epoch;
                *created += 1;
                return (long long)s;
            }
            if (old == k) return (long long)s;
        }
        s = (s + 1) & tmask;
        key = ld_relaxed(&table[s].key);
    }
    return -1;
}

// Exclusive scan of one value per thread over the 256 threads of a block (tmp: 4 words).
__device__ __forceinline__ u32 block_excl_scan(u32 x, u32* tmp, u32* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u32 inc = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u32 y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) tmp[w] = inc;
    __syncthreads();
    u32 pre = 0, all = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (q < w) pre += tmp[q];
        all += tmp[q];
    }
    __syncthreads();
    *total = all;
    return pre + inc - x;
}

__device__ __forceinline__ u32 bucket_of(u64 key, u32 log2b) {
    return key == EMPTY_KEY ? (1u << log2b) - 1 : (u32)(mix64(key) >> (64 - log2b));
}

// ---- role: split(e) ------------------------------------------------------------------------
// Tile t (this block) holds Puts [t*st, t*st + st). Counting sort by bucket inside the tile:
// items of bucket b land at items[t*st + bin_off[t][b] ...], bin_cnt[t][b] of them (tile-major:
// the split's writes are coalesced; owners read a column, which stays in L2).
__device__ __forceinline__ void split_role(SplitJob j, u32 t, u32* smem) {
    const u32 B = 1u << j.log2b;
    u32* cnt = smem;  // B <= HM_MAX_BUCKETS words
    u32* tmp = smem + HM_MAX_BUCKETS;
    for (u32 q = threadIdx.x; q < B; q += TPB) cnt[q] = 0;
    __syncthreads();
    const u64 base = (u64)t * j.st;
    const u64 end = base + j.st < j.n ? base + j.st : j.n;
    for (u64 i = base + threadIdx.x; i < end; i += TPB) {
        const nrg_put r = j.rec.at(i);
        if (j.ring_out) j.ring_out[(j.rec.lo + i) & j.rec.mask] = r;
        j.put_flag[i] = 0;
        atomicAdd(&cnt[bucket_of(r.key, j.log2b)], 1u);
    }
    __syncthreads();
    // exclusive scan of the B counters: thread q owns a contiguous run of per = B/TPB of them
    const u32 per = (B + TPB - 1) / TPB;
    const u32 q0 = threadIdx.x * per;
    u32 local = 0;
    for (u32 q = q0; q < q0 + per && q < B; q++) local += cnt[q];
    u32 total;
    u32 run = block_excl_scan(local, tmp, &total);
    for (u32 q = q0; q < q0 + per && q < B; q++) {
        const u32 c = cnt[q];
        j.bin_cnt[(u64)t * B + q] = c;
        j.bin_off[(u64)t * B + q] = run;
        cnt[q] = run;  // becomes the cursor
        run += c;
    }
    __syncthreads();
    for (u64 i = base + threadIdx.x; i < end; i += TPB) {
        const u64 k = j.rec.at(i).key;
        const u32 pos = atomicAdd(&cnt[bucket_of(k, j.log2b)], 1u);
        PutItem it;
        it.key = k;
        it.i = (u32)i;
        it.pad = 0;
        j.items[base + pos] = it;
    }
}

// ---- role: index(e) — owner blocks ----------------------------------------------------------
// Block (m, b): bucket b, share m of at most OW_MMAX. All Puts of bucket b's keys are in bucket
// b's runs, so when one block owns the bucket (the usual case) its LDS election is exact.
__device__ __forceinline__ void owner_role(OwnerJob j, u32 blk, Slot* table, u32 shift, u64 tmask, DevCtl* ctl,
                                           u32* smem) {
    const u32 B = 1u << j.log2b;
    const u32 b = blk % B, m = blk / B;
    u32* s_slot = smem;
    u32* s_max = smem + OW_LDS;
    u32* s_start = smem + 2 * OW_LDS;             // per tile: first index of its run in my list
    u32* s_off = s_start + HM_MAX_TILES;          // per tile: run offset inside the tile
    u32* s_cnt = s_off + HM_MAX_TILES;            // per tile: run length (0 if not mine)
    u32* s_misc = s_cnt + HM_MAX_TILES;           // [0..3] scan tmp, [4] created, [5] side max
    const u32 t = threadIdx.x;                     // one tile per thread (ntiles <= 256)
    const u32 c = t < j.ntiles ? j.bin_cnt[(u64)t * B + b] : 0;
    const u32 o = t < j.ntiles ? j.bin_off[(u64)t * B + b] : 0;
    u32 total;
    (void)block_excl_scan(c, s_misc, &total);
    u32 M = (total + OW_CHUNK - 1) / OW_CHUNK;
    if (M < 1) M = 1;
    if (M > OW_MMAX) M = OW_MMAX;
    if (m >= M || total == 0) return;  // uniform across the block
    const bool shared = M > 1;
    const u32 mine = (t % M == m) ? c : 0;
    u32 N;
    const u32 start = block_excl_scan(mine, s_misc, &N);
    s_start[t] = start;
    s_off[t] = o;
    s_cnt[t] = mine;
    if (t == 0) {
        s_misc[4] = 0;
        s_misc[5] = 0;
    }
    const u32 par = j.epoch & 1;
    u32 created = 0;
    for (u32 pb = 0; pb < N; pb += OW_PASS) {
        for (int q = threadIdx.x; q < OW_LDS; q += TPB) {
            s_slot[q] = 0xFFFFFFFFu;
            s_max[q] = 0;
        }
        __syncthreads();
        PutItem it[OW_IPT];
        u64 home[OW_IPT], key0[OW_IPT];
        bool ok[OW_IPT];
#pragma unroll
        for (int q = 0; q < OW_IPT; q++) {
            const u32 x = pb + (u32)q * TPB + threadIdx.x;
            ok[q] = x < N;
            it[q].key = EMPTY_KEY;
            it[q].i = 0;
            if (ok[q]) {
                // the run holding x: the last tile whose start is <= x (empty runs share starts)
                u32 lo = 0, hi = j.ntiles - 1;
                while (lo < hi) {
                    const u32 mid = (lo + hi + 1) >> 1;
                    if (s_start[mid] <= x) lo = mid; else hi = mid - 1;
                }
                it[q] = j.items[(u64)lo * j.st + s_off[lo] + (x - s_start[lo])];
            }
        }
        if (j.exp & 1) {
            u32 acc = 0;
#pragma unroll
            for (int q = 0; q < OW_IPT; q++) acc += it[q].i;
            if (acc == 0xFFFFFFFFu) j.put_flag[0] = 9;
            __syncthreads();
            continue;
        }
#pragma unroll
        for (int q = 0; q < OW_IPT; q++) {
            home[q] = table_home(it[q].key, shift);
            key0[q] = (ok[q] && it[q].key != EMPTY_KEY && !(j.exp & 2)) ? table[home[q]].key : it[q].key;
        }
#pragma unroll
        for (int q = 0; q < OW_IPT; q++) {
            if (!ok[q]) continue;
            const u32 i = it[q].i;
            if (it[q].key == EMPTY_KEY) {  // the side-slot key
                if (ld_relaxed32(&ctl->sp.created) == 0 && atomicCAS(&ctl->sp.created, 0u, j.epoch) == 0u) created++;
                atomicMax(&s_misc[5], i + 1);
                if (j.all_slots) j.put_slot[i] = SIDE_SLOT;
                continue;
            }
            const long long s = find_or_claim(table, it[q].key, home[q], tmask, key0[q], j.epoch, &created);
            if (s < 0) {
                atomicOr(&ctl->err, ERR_TABLE_FULL);
                if (j.all_slots) j.put_slot[i] = FULL_SLOT;
                continue;
            }
            if (j.all_slots) j.put_slot[i] = (u32)s;
            u32 h = (u32)(mix64((u64)s) & (OW_LDS - 1));
            for (;;) {
                const u32 old = atomicCAS(&s_slot[h], 0xFFFFFFFFu, (u32)s);
                if (old == 0xFFFFFFFFu || old == (u32)s) break;
                h = (h + 1) & (OW_LDS - 1);
            }
            atomicMax(&s_max[h], i + 1);
        }
        __syncthreads();
        // publish this pass's winners
        for (int q = threadIdx.x; q < OW_LDS && !(j.exp & 4); q += TPB) {
            const u32 s = s_slot[q];
            if (s == 0xFFFFFFFFu) continue;
            const u32 mx = s_max[q];
            u64* sp = slot_stamp(&table[s], par);
            if (shared) {
                atomicMax(sp, ((u64)j.epoch << 32) | mx);
                j.put_slot[mx - 1] = s;
                j.put_flag[mx - 1] = FLAG_CHECK;
                continue;
            }
            // sole owner: an earlier pass of this block may have elected a later Put already
            const u64 cur = pb ? ld_relaxed(sp) : 0;
            if ((u32)(cur >> 32) == j.epoch) {
                if ((u32)cur >= mx) continue;
                j.put_flag[(u32)cur - 1] = 0;
            }
            __hip_atomic_store(sp, ((u64)j.epoch << 32) | mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            j.put_slot[mx - 1] = s;
            j.put_flag[mx - 1] = FLAG_WIN;
        }
        __syncthreads();
    }
    if (created) atomicAdd(&s_misc[4], created);
    __syncthreads();
    if (threadIdx.x == 0) {
        // keys created by this block: a per-block counter (plain add, one writer per launch);
        // one same-address atomic per block would serialise at the memory side (~88/us)
        if (s_misc[4]) j.created_acc[blk] += s_misc[4];
        const u32 sm = s_misc[5];
        if (sm) {  // side key: rare, always elected with an atomic
            atomicMax(slot_stamp(&ctl->sp, par), ((u64)j.epoch << 32) | sm);
            j.put_slot[sm - 1] = SIDE_SLOT;
            j.put_flag[sm - 1] = FLAG_CHECK;
        }
    }
}

// ---- role: apply(e) -------------------------------------------------------------------------
__device__ __forceinline__ void apply_role(ApplyJob j, u32 blk, Slot* table, DevCtl* ctl) {
    const u64 i = (u64)blk * TPB + threadIdx.x;
    if (i >= j.n) return;
    const uint8_t f = j.put_flag[i];
    if (!f) return;
    const u32 s = j.put_slot[i];
    Slot* sl = s == SIDE_SLOT ? &ctl->sp : &table[s];
    if (f == FLAG_CHECK && *slot_stamp(sl, j.epoch & 1) != stamp_of(j.epoch, i)) return;
    sl->val = j.rec.at(i).val;
}

// ---- role: reads(e) -------------------------------------------------------------------------
template <int G>
__device__ __forceinline__ void read_role(ReadJob j, u32 blk, const Slot* table, u32 shift, u64 tmask,
                                          const DevCtl* ctl) {
    // G Gets per thread: all key loads, then all first-slot loads, are in flight together
    const u32 par = j.epoch & 1;
    const bool use_rec = j.rec.src != nullptr || j.rec.ring != nullptr;
    const u64 jb = (u64)blk * TPB * G + threadIdx.x;
    u64 k[G];
    View first[G];
#pragma unroll
    for (int g = 0; g < G; g++) {
        const u64 q = jb + (u64)g * TPB;
        k[g] = q < j.R ? j.keys[q] : EMPTY_KEY;
    }
#pragma unroll
    for (int g = 0; g < G; g++) first[g] = load_view(k[g] == EMPTY_KEY ? &ctl->sp : &table[table_home(k[g], shift)], par);
#pragma unroll
    for (int g = 0; g < G; g++) {
        const u64 q = jb + (u64)g * TPB;
        if (q >= j.R) break;
        u64 v = 0;
        bool f = false;
        if (k[g] == EMPTY_KEY) {
            f = resolve(first[g], j.epoch, j.rec, use_rec, &v);
        } else {
            u64 s = table_home(k[g], shift);
            View w = first[g];
            for (u64 pr = 0; pr <= tmask; pr++) {
                if (w.key == k[g]) {
                    f = resolve(w, j.epoch, j.rec, use_rec, &v);
                    break;
                }
                if (w.key == EMPTY_KEY) break;
                s = (s + 1) & tmask;
                w = load_view(&table[s], par);
            }
        }
        if (!f) v = 0;
        j.vals[q] = v;
        j.found[q] = f ? 1 : 0;
    }
}

// One launch = {index(e-1)} + {split(e)} + {apply(e-2)} + {reads(e-2)} over disjoint block
// ranges (any may be empty). Owner blocks come first so the latency-bound pass starts first.
template <int G>
__global__ __launch_bounds__(TPB) void hm_round_kernel(OwnerJob oj, SplitJob sj, ApplyJob aj, ReadJob rj,
                                                       Slot* table, u32 shift, u64 tmask, DevCtl* ctl) {
    __shared__ u32 smem[SMEM_WORDS];
    u32 b = blockIdx.x;
    if (b < oj.nblocks) {
        owner_role(oj, b, table, shift, tmask, ctl, smem);
        return;
    }
    b -= oj.nblocks;
    if (b < sj.nblocks) {
        split_role(sj, b, smem);
        return;
    }
    b -= sj.nblocks;
    if (b < aj.nblocks) {
        apply_role(aj, b, table, ctl);
        return;
    }
    b -= aj.nblocks;
    read_role<G>(rj, b, table, shift, tmask, ctl);
}

// Previous-value responses (HashMap::insert's return, nr/examples/hashmap.rs:46-50): with the
// round's Puts stably sorted by slot, a Put's previous value is its in-group predecessor's
// value, or the slot's value before the round (absent if the key was created in it). Runs
// after index(e) and before apply(e), so slot values are still the pre-round ones.
__global__ __launch_bounds__(TPB) void hm_prev_kernel(const u32* __restrict__ sk, const u32* __restrict__ sv, u64 n,
                                                      RecSrc rec, const Slot* __restrict__ table, const DevCtl* ctl,
                                                      u32 epoch, u64 resp_lo, u64 resp_hi, u64* __restrict__ prev,
                                                      uint8_t* __restrict__ prevf) {
    const u64 p = blockIdx.x * (u64)TPB + threadIdx.x;
    if (p >= n) return;
    const u32 s = sk[p];
    const u64 gidx = rec.lo + sv[p];
    if (gidx < resp_lo || gidx >= resp_hi) return;
    u64 v = 0;
    uint8_t f = 0;
    if (p > 0 && sk[p - 1] == s) {
        v = rec.at(sv[p - 1]).val;
        f = 1;
    } else if (s == SIDE_SLOT) {
        const u32 cr = ctl->sp.created;
        if (cr != 0 && cr != epoch) {
            v = ctl->sp.val;
            f = 1;
        }
    } else if (s != FULL_SLOT && table[s].created != epoch) {  // existed before the round
        v = table[s].val;
        f = 1;
    }
    prev[gidx - resp_lo] = v;
    prevf[gidx - resp_lo] = f;
}

__global__ __launch_bounds__(TPB) void hm_init_table_kernel(Slot* table, u64 slots) {
    for (u64 s = blockIdx.x * (u64)TPB + threadIdx.x; s < slots; s += (u64)gridDim.x * TPB) {
        Slot z = {};
        z.key = EMPTY_KEY;
        table[s] = z;
    }
}

// NrHashMap::default (benches/hashmap.rs:91-100): keys 0..n-1 -> k + off, inserted directly.
__global__ __launch_bounds__(TPB) void hm_prefill_range_kernel(Slot* table, u64 n, u64 off, u32 shift, u64 tmask,
                                                               DevCtl* ctl, u32 epoch) {
    __shared__ u32 s_ins;
    if (threadIdx.x == 0) s_ins = 0;
    __syncthreads();
    u32 inserted = 0;
    for (u64 k = blockIdx.x * (u64)TPB + threadIdx.x; k < n; k += (u64)gridDim.x * TPB) {
        u64 s = table_home(k, shift);
        bool done = false;
        for (u64 pr = 0; pr <= tmask && !done; pr++) {
            const u64 old = atomicCAS(&table[s].key, EMPTY_KEY, k);
            if (old == EMPTY_KEY || old == k) {
                table[s].val = k + off;
                if (old == EMPTY_KEY) table[s].created = epoch;
                inserted += old == EMPTY_KEY;
                done = true;
            }
            s = (s + 1) & tmask;
        }
        if (!done) atomicOr(&ctl->err, ERR_TABLE_FULL);
    }
    if (inserted) atomicAdd(&s_ins, inserted);
    __syncthreads();
    if (threadIdx.x == 0 && s_ins) atomicAdd(&ctl->nkeys, (u64)s_ins);
}

// number of keys = prefill/direct inserts (ctl->nkeys) + keys created by owner blocks
__global__ __launch_bounds__(TPB) void hm_count_kernel(const u64* __restrict__ acc, u64 n, DevCtl* ctl) {
    __shared__ u64 s_w[4];
    u64 x = 0;
    for (u64 q = threadIdx.x; q < n; q += TPB) x += acc[q];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) ctl->nkeys_total = ctl->nkeys + s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

__global__ __launch_bounds__(TPB) void hm_dump_kernel(const Slot* __restrict__ table, u64 slots, DevCtl* ctl,
                                                      u64* __restrict__ ok, u64* __restrict__ ov) {
    const u64 gid = blockIdx.x * (u64)TPB + threadIdx.x;
    if (gid == 0 && ctl->sp.created) {
        const u64 i = atomicAdd(&ctl->counter, 1ull);
        ok[i] = EMPTY_KEY;
        ov[i] = ctl->sp.val;
    }
    for (u64 s = gid; s < slots; s += (u64)gridDim.x * TPB) {
        const u64 k = table[s].key;
        if (k != EMPTY_KEY) {
            const u64 i = atomicAdd(&ctl->counter, 1ull);
            ok[i] = k;
            ov[i] = table[s].val;
        }
    }
}

__global__ __launch_bounds__(TPB) void hm_digest_kernel(const Slot* __restrict__ table, u64 slots,
                                                        const DevCtl* ctl, u64* out3) {
    __shared__ u64 s_c[4], s_s[4], s_x[4];
    const u64 gid = blockIdx.x * (u64)TPB + threadIdx.x;
    u64 c = 0, sm = 0, x = 0;
    if (gid == 0 && ctl->sp.created) {
        const u64 h = mix64(EMPTY_KEY ^ mix64(ctl->sp.val));
        c++;
        sm += h;
        x ^= h;
    }
    for (u64 s = gid; s < slots; s += (u64)gridDim.x * TPB) {
        const u64 k = table[s].key;
        if (k != EMPTY_KEY) {
            const u64 h = mix64(k ^ mix64(table[s].val));
            c++;
            sm += h;
            x ^= h;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        c += __shfl_xor(c, off, 64);
        sm += __shfl_xor(sm, off, 64);
        x ^= __shfl_xor(x, off, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_c[w] = c;
        s_s[w] = sm;
        s_x[w] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        c = s_c[0] + s_c[1] + s_c[2] + s_c[3];
        sm = s_s[0] + s_s[1] + s_s[2] + s_s[3];
        x = s_x[0] ^ s_x[1] ^ s_x[2] ^ s_x[3];
        atomicAdd(&out3[0], c);
        atomicAdd(&out3[1], sm);
        atomicXor(&out3[2], x);
    }
}

struct SegArgs {
    u64 start[64];  // exclusive prefix of lens (in records)
    u64 total;
    u32 nseg;
    u32 words;  // record size in u64 words
};

__global__ __launch_bounds__(TPB) void copy_segments_kernel(const u64* __restrict__ base, u64 seg_stride_words,
                                                            SegArgs a, u64* ring, u64 ring_mask, u64 dst_lo) {
    for (u64 r = blockIdx.x * (u64)TPB + threadIdx.x; r < a.total; r += (u64)gridDim.x * TPB) {
        u32 s = 0;
        while (s + 1 < a.nseg && a.start[s + 1] <= r) s++;
        const u64 j = r - a.start[s];
        const u64* srcp = base + s * seg_stride_words + j * a.words;
        u64* dst = ring + ((dst_lo + r) & ring_mask) * a.words;
        for (u32 q = 0; q < a.words; q++) dst[q] = srcp[q];
    }
}

static inline unsigned grid_for(u64 n, u64 cap = 4096) {
    u64 g = (n + TPB - 1) / TPB;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// ---- host side ----------------------------------------------------------------------------
static RecSrc ring_src(nrg_ctx* c, const nrg_put* src, u64 lo) {
    RecSrc r;
    r.src = src;
    r.ring = (const nrg_put*)c->d_ring;
    r.mask = c->log_size - 1;
    r.lo = lo;
    return r;
}

static u32 ilog2_floor(u64 x) {
    u32 b = 0;
    while ((2ull << b) <= x) b++;
    return b;
}

// Split geometry of a round of n Puts: ~256 Puts per bucket (one owner block, one Put per
// thread: the owner pass is latency-bound, so many small owners beat few large ones), at most
// HM_MAX_TILES tiles (one run per tile per owner thread), buckets no finer than the table.
static void round_geometry(nrg_ctx* c, HmRound& r) {
    u32 lb = r.n >= 2048 ? ilog2_floor(r.n / 256) : 3;
    if (lb < 3) lb = 3;
    if (lb > 11) lb = 11;  // HM_MAX_BUCKETS
    if (lb > c->cfg.log2_slots) lb = c->cfg.log2_slots;
    u64 st = 2048;
    while (st * HM_MAX_TILES < r.n) st <<= 1;
    r.log2b = lb;
    r.st = (u32)st;
    r.ntiles = (u32)((r.n + st - 1) / st);
    if (r.ntiles == 0) r.ntiles = 1;
}

template <int G>
static void launch_round(nrg_ctx* c, const OwnerJob& oj, const SplitJob& sj, const ApplyJob& aj, const ReadJob& rj) {
    const u32 blocks = oj.nblocks + sj.nblocks + aj.nblocks + rj.nblocks;
    NRG_LAUNCH(c, "hm_round", (hm_round_kernel<G>), blocks, TPB, 0, c->stream, oj, sj, aj, rj, c->d_table,
               c->slot_shift, (u64)(c->slots - 1), c->d_ctl);
}

// One launch: split `s` (records from split_src if given, else the ring; writing the ring copy
// if write_ring), index `x`, apply + read `a`; or, with all three null, R reads of the applied
// state at read_epoch.
static hipError_t launch(nrg_ctx* c, const HmRound* s, const nrg_put* split_src, bool write_ring, const HmRound* x,
                         const HmRound* a, const u64* keys = nullptr, u64 R = 0, u64* vals = nullptr,
                         uint8_t* found = nullptr, u32 read_epoch = 0) {
    SplitJob sj{};
    OwnerJob oj{};
    ApplyJob aj{};
    ReadJob rj{};
    if (s) {
        const u32 p = s->epoch & 1;
        sj.rec = ring_src(c, split_src, s->lo);
        sj.ring_out = write_ring ? (nrg_put*)c->d_ring : nullptr;
        sj.n = s->n;
        sj.items = c->d_items[p];
        sj.bin_cnt = c->d_bin_cnt[p];
        sj.bin_off = c->d_bin_off[p];
        sj.put_flag = c->d_put_flag[p];
        sj.st = s->st;
        sj.ntiles = s->ntiles;
        sj.log2b = s->log2b;
        sj.nblocks = s->ntiles;
    }
    if (x) {
        const u32 p = x->epoch & 1;
        oj.items = c->d_items[p];
        oj.bin_cnt = c->d_bin_cnt[p];
        oj.bin_off = c->d_bin_off[p];
        oj.put_slot = c->d_put_slot[p];
        oj.put_flag = c->d_put_flag[p];
        oj.st = x->st;
        oj.ntiles = x->ntiles;
        oj.log2b = x->log2b;
        oj.epoch = x->epoch;
        oj.nblocks = (1u << x->log2b) * OW_MMAX;
        oj.all_slots = c->all_slots ? 1 : 0;
        oj.created_acc = c->d_created;
        oj.exp = c->exp;
    }
    if (a) {
        const u32 p = a->epoch & 1;
        aj.rec = ring_src(c, a->src, a->lo);
        aj.n = a->n;
        aj.put_slot = c->d_put_slot[p];
        aj.put_flag = c->d_put_flag[p];
        aj.epoch = a->epoch;
        aj.nblocks = (u32)((a->n + TPB - 1) / TPB);
        rj.rec = aj.rec;
        rj.keys = a->keys;
        rj.R = a->R;
        rj.vals = a->vals;
        rj.found = a->found;
        rj.epoch = a->epoch;
    } else if (R) {  // reads only, every round applied: values come from the slots
        rj.keys = keys;
        rj.R = R;
        rj.vals = vals;
        rj.found = found;
        rj.epoch = read_epoch;
    }
    const u32 G = c->gets_per_thread >= 4 ? 4 : (c->gets_per_thread == 2 ? 2 : 1);
    rj.nblocks = (u32)((rj.R + TPB * G - 1) / (TPB * G));
    if (oj.nblocks + sj.nblocks + aj.nblocks + rj.nblocks == 0) return hipSuccess;
    if (G == 4)
        launch_round<4>(c, oj, sj, aj, rj);
    else if (G == 2)
        launch_round<2>(c, oj, sj, aj, rj);
    else
        launch_round<1>(c, oj, sj, aj, rj);
    return hipGetLastError();
}

// Advance the pipeline by one launch: index pend_i, apply + read pend_a.
static hipError_t advance(nrg_ctx* c) {
    hipError_t e = launch(c, nullptr, nullptr, false, c->pend_i.valid ? &c->pend_i : nullptr,
                          c->pend_a.valid ? &c->pend_a : nullptr);
    if (e != hipSuccess) return e;
    c->pend_a = c->pend_i;
    c->pend_i.valid = false;
    return hipSuccess;
}

hipError_t hm_flush(nrg_ctx* c) {
    while (c->pend_i.valid || c->pend_a.valid) {
        hipError_t e = advance(c);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Reads against the current state (no writes): attached to the newest round in flight if it has
// none, else launched after draining.
static hipError_t hm_reads(nrg_ctx* c, const u64* keys, u64 R, u64* vals, uint8_t* found) {
    if (R == 0) return hipSuccess;
    HmRound* newest = c->pend_i.valid ? &c->pend_i : (c->pend_a.valid ? &c->pend_a : nullptr);
    if (newest && newest->R == 0) {
        newest->keys = keys;
        newest->R = R;
        newest->vals = vals;
        newest->found = found;
        return hm_flush(c);
    }
    hipError_t e = hm_flush(c);
    if (e != hipSuccess) return e;
    return launch(c, nullptr, nullptr, false, nullptr, nullptr, keys, R, vals, found, c->epoch);
}

hipError_t hm_init(nrg_ctx* c) {
    hm_init_table_kernel<<<grid_for(c->slots, 16384), TPB, 0, c->stream>>>(c->d_table, c->slots);
    return hipGetLastError();
}

// Replay the records [lo, lo+n) (from `src_recs` if given, else from the ring; writing the
// ring copy if write_ring) and answer R reads against the state after them.
hipError_t hm_replay_chunk(nrg_ctx* c, const void* src_recs, u64 lo, u64 n, bool write_ring, const u64* d_get_keys,
                           u64 R, u64* d_get_vals, uint8_t* d_get_found, u64 resp_lo, u64 resp_hi, u64* d_prev,
                           uint8_t* d_prev_found, bool touch_log) {
    (void)touch_log;
    if (n == 0) return hm_reads(c, d_get_keys, R, d_get_vals, d_get_found);
    const nrg_put* src = (const nrg_put*)src_recs;
    HmRound r;
    r.valid = true;
    r.epoch = ++c->epoch;
    r.src = (src && !write_ring) ? src : nullptr;  // later stages: the ring copy if there is one
    r.lo = lo;
    r.n = n;
    r.keys = d_get_keys;
    r.R = R;
    r.vals = d_get_vals;
    r.found = d_get_found;
    round_geometry(c, r);
    hipError_t e;
    const bool want_prev = d_prev && resp_lo < lo + n && resp_hi > lo;
    if (want_prev || r.src) {
        // previous-value responses (or records in a private buffer): run this round's split and
        // index back to back, answer from the pre-apply state, then apply
        if ((e = hm_flush(c)) != hipSuccess) return e;
        if ((e = launch(c, &r, src, write_ring, nullptr, nullptr)) != hipSuccess) return e;
        c->all_slots = want_prev;
        e = launch(c, nullptr, nullptr, false, &r, nullptr);
        c->all_slots = false;
        if (e != hipSuccess) return e;
        if (want_prev) {
            u32 *sk = nullptr, *sv = nullptr;
            timer_begin(c, "hm_prev", c->stream);
            // slot ids < 2^30; the side-slot (0xFFFFFFFF) and full (0xFFFFFFFE) markers sort last
            e = sort_pairs(c->sort, c->d_put_slot[r.epoch & 1], nullptr, n, 32, c->stream, &sk, &sv);
            if (e != hipSuccess) return e;
            hm_prev_kernel<<<(unsigned)((n + TPB - 1) / TPB), TPB, 0, c->stream>>>(
                sk, sv, n, ring_src(c, r.src, lo), c->d_table, c->d_ctl, r.epoch, resp_lo, resp_hi, d_prev,
                d_prev_found);
            timer_end(c, "hm_prev", c->stream);
        }
        c->pend_a = r;
        c->pend_i.valid = false;
        if (!c->pipeline || r.src) return hm_flush(c);
        return hipGetLastError();
    }
    // one launch: split this round, index the previous one, apply + read the one before
    e = launch(c, &r, src, write_ring, c->pend_i.valid ? &c->pend_i : nullptr, c->pend_a.valid ? &c->pend_a : nullptr);
    if (e != hipSuccess) return e;
    c->pend_a = c->pend_i;
    c->pend_i = r;
    if (!c->pipeline) return hm_flush(c);
    return hipSuccess;
}

hipError_t hm_get_only(nrg_ctx* c, const u64* d_keys, u64 n, u64* d_vals, uint8_t* d_found) {
    return hm_reads(c, d_keys, n, d_vals, d_found);
}

hipError_t hm_prefill_range(nrg_ctx* c, u64 n, u64 off) {
    hipError_t e = hm_flush(c);
    if (e != hipSuccess) return e;
    // a fresh epoch: later reads see these values in the slots, not an older round's record
    const u32 epoch = ++c->epoch;
    hm_prefill_range_kernel<<<grid_for(n, 8192), TPB, 0, c->stream>>>(c->d_table, n, off, c->slot_shift,
                                                                      c->slots - 1, c->d_ctl, epoch);
    return hipGetLastError();
}

hipError_t hm_count(nrg_ctx* c) {
    hipError_t e = hm_flush(c);
    if (e != hipSuccess) return e;
    hm_count_kernel<<<1, TPB, 0, c->stream>>>(c->d_created, HM_MAX_BUCKETS * OW_MMAX, c->d_ctl);
    return hipGetLastError();
}

hipError_t hm_dump(nrg_ctx* c, u64* d_keys, u64* d_vals) {
    hipError_t e = hm_flush(c);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(&c->d_ctl->counter, 0, sizeof(u64), c->stream);
    if (e != hipSuccess) return e;
    hm_dump_kernel<<<grid_for(c->slots, 8192), TPB, 0, c->stream>>>(c->d_table, c->slots, c->d_ctl, d_keys, d_vals);
    return hipGetLastError();
}

hipError_t hm_digest(nrg_ctx* c, u64* d_out3) {
    hipError_t e = hm_flush(c);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(d_out3, 0, 3 * sizeof(u64), c->stream);
    if (e != hipSuccess) return e;
    hm_digest_kernel<<<grid_for(c->slots, 8192), TPB, 0, c->stream>>>(c->d_table, c->slots, c->d_ctl, d_out3);
    return hipGetLastError();
}

hipError_t copy_segments(nrg_ctx* c, const void* d_base, u32 nseg, u64 seg_stride, const u64* lens, u64 dst_lo) {
    SegArgs a;
    if (nseg > 64) return hipErrorInvalidValue;
    a.nseg = nseg;
    a.words = c->rec_bytes / 8;
    u64 acc = 0;
    for (u32 s = 0; s < nseg; s++) {
        a.start[s] = acc;
        acc += lens[s];
    }
    a.total = acc;
    if (acc == 0) return hipSuccess;
    copy_segments_kernel<<<grid_for(acc, 8192), TPB, 0, c->stream>>>(
        (const u64*)d_base, seg_stride * a.words, a, (u64*)c->d_ring, c->log_size - 1, dst_lo);
    return hipGetLastError();
}

}  // namespace nrg
