// hashmap.hip — NrHashMap replica replay on gfx950.
//
// Replaces the hot loop of Log::exec -> NrHashMap::dispatch_mut (nr/src/log.rs:494-518,
// benches/hashmap.rs:114-119, nr/examples/hashmap.rs:46-50) and the read path
// Replica::read_only -> dispatch (nr/src/replica.rs:483-497, benches/hashmap.rs:107-111).
//
// Table: 2^k open-addressing slots of 64 B (common.hpp), linear probing from
// mix64(key) >> (64 - k). A replay round covers the log records [lo, lo+n) and gets a fresh
// epoch e (never reused). Its work splits into two halves:
//
//   index(e)   per Put: find the key's slot, or claim an empty one with a 64-bit CAS
//              (created = e); elect the round's last writer of every key with
//              atomicMax(slot.stamp[e&1], e<<32 | i+1), pre-combined per block in LDS so a
//              hot key costs one global atomic per block (Zipf streams). Writes put_slot[i]
//              and, when the round is appended here, the log copy.
//   apply(e)   per Put: the elected writer (stamp[e&1] == (e, i+1)) stores its value.
//   reads(e)   per Get, against the state after round e: a key counts iff 0 < created <= e;
//              its value is the round's elected record when stamp[e&1] carries epoch e
//              (apply(e) may still be storing it), else the slot's value.
//
// All three roles live in ONE kernel (hm_round_kernel, disjoint block ranges), launched as
// {index(e) | apply(e-1) + reads(e-1)}: the latency-bound index pass of a round overlaps the
// bandwidth-bound reads of the previous one. This is race-free because index(e) only claims
// empty slots (invisible to reads(e-1): created is 0 or e) and raises stamp[e&1], while
// apply(e-1)/reads(e-1) only look at stamp[(e-1)&1] and at values that index never writes.
// The result equals the sequential replay: last-writer-wins per key in log order, and reads
// after the round's writes (SURVEY.md §8a round semantics).
#include "internal.hpp"

namespace nrg {

typedef u64 u64x2 __attribute__((ext_vector_type(2)));

constexpr int TPB = 256;  // B1: 36.6 us/round; 128: 36.4 (noise); 512: 37.6 (profiles/r01_variants/tpb_sweep.txt)
constexpr u32 SIDE_SLOT = 0xFFFFFFFFu;   // put_slot value of the EMPTY_KEY key (side slot)
constexpr u32 FULL_SLOT = 0xFFFFFFFEu;   // put_slot value of a Put that found no slot

__device__ __forceinline__ u64 stamp_of(u32 epoch, u64 i) { return ((u64)epoch << 32) | (i + 1); }

// record i of a round: from a caller's buffer when given, else from the log ring
struct RecSrc {
    const nrg_put* src;
    const nrg_put* ring;
    u64 mask, lo;
    __device__ __forceinline__ nrg_put at(u64 i) const { return src ? src[i] : ring[(lo + i) & mask]; }
};

struct IndexJob {
    RecSrc rec;
    nrg_put* ring_out;  // log copy to write (nullptr: records already in the ring)
    u64 n;
    u32* put_slot;
    u32 epoch;
    u32 nblocks;
    u64* created_acc;  // [HM_CREATED_SLOTS] keys created by index blocks
    u64x2* bk_ent;  // bucket election (hm_elect_kernel): per index block, its distinct {slot, i+1; value}
    u32* bk_cnt;  // entries grouped by slot bucket; [bucket][block] = offset << 16 | count
    u32 bk_shift;  // bucket of slot s = s >> bk_shift
    u32 bk_nb;     // buckets (power of two, <= HM_BK_MAX)
    u32 exp;  // diagnostic knobs (NRG_EXP; results are wrong when set): 1 no stamp atomics,
              // 2 no LDS combining (one atomic per Put), 4 no apply role, 8 no index role
};
struct ApplyJob {
    RecSrc rec;
    u64 n;
    const u32* put_slot;
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
    // plain loads: the second hits the line the first brought in (non-temporal loads measured
    // 37.0 -> 44.6 us per B1 round, both going to memory)
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

// Block-wide exclusive prefix sum of one u32 per thread (TPB threads); *total gets the sum.
__device__ __forceinline__ u32 block_scan_excl(u32 v, u32* total) {
    __shared__ u32 s_w[TPB / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u32 inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u32 y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) s_w[w] = inc;
    __syncthreads();
    u32 pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < TPB / 64; i++) {
        pre += i < w ? s_w[i] : 0u;
        tot += s_w[i];
    }
    __syncthreads();
    if (total) *total = tot;
    return pre + inc - v;
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

// ---- role: index(e) -------------------------------------------------------------------------
template <int K1_ITEMS, bool BK>
__device__ __forceinline__ void index_role(IndexJob j, u32 blk, Slot* table, u32 shift, u64 tmask,
                                           DevCtl* ctl) {
    constexpr int K1_TILE = TPB * K1_ITEMS;
    constexpr int K1_LDS = 2 * K1_TILE;
    __shared__ u32 s_slot[K1_LDS];
    __shared__ u32 s_max[K1_LDS];
    __shared__ u32 s_created;
    __shared__ u32 s_bk[BK ? HM_BK_MAX : 1];
    for (int q = threadIdx.x; q < K1_LDS; q += TPB) {
        s_slot[q] = 0xFFFFFFFFu;
        s_max[q] = 0;
    }
    if constexpr (BK)
        for (int q = threadIdx.x; q < (int)j.bk_nb; q += TPB) s_bk[q] = 0;
    if (threadIdx.x == 0) s_created = 0;
    __syncthreads();
    const u32 par = j.epoch & 1;
    const u64 base = (u64)blk * K1_TILE;
    u32 created = 0;
    u64 sl_idx[K1_ITEMS];
    u64 key0[K1_ITEMS];
    nrg_put rec[K1_ITEMS];
    u32 hq[K1_ITEMS];  // LDS combine entry of each record (bucket election), ~0u: none
#pragma unroll
    for (int q = 0; q < K1_ITEMS; q++) hq[q] = ~0u;
    // issue every record load and every first probe before waiting on any of them
#pragma unroll
    for (int q = 0; q < K1_ITEMS; q++) {
        const u64 i = base + (u64)q * TPB + threadIdx.x;
        rec[q] = i < j.n ? j.rec.at(i) : nrg_put{EMPTY_KEY, 0};
    }
#pragma unroll
    for (int q = 0; q < K1_ITEMS; q++) {
        const u64 i = base + (u64)q * TPB + threadIdx.x;
        if (i < j.n && j.ring_out) j.ring_out[(j.rec.lo + i) & j.rec.mask] = rec[q];
        sl_idx[q] = table_home(rec[q].key, shift);
        key0[q] = rec[q].key != EMPTY_KEY ? table[sl_idx[q]].key : EMPTY_KEY;
    }
#pragma unroll
    for (int q = 0; q < K1_ITEMS; q++) {
        const u64 i = base + (u64)q * TPB + threadIdx.x;
        if (i >= j.n) continue;
        const u64 k = rec[q].key;
        if (k == EMPTY_KEY) {  // the side-slot key
            if (ld_relaxed32(&ctl->sp.created) == 0 && atomicCAS(&ctl->sp.created, 0u, j.epoch) == 0u) created++;
            atomicMax(slot_stamp(&ctl->sp, par), stamp_of(j.epoch, i));
            j.put_slot[i] = SIDE_SLOT;
            continue;
        }
        const long long s = find_or_claim(table, k, sl_idx[q], tmask, key0[q], j.epoch, &created);
        if (s < 0) {
            atomicOr(&ctl->err, ERR_TABLE_FULL);
            j.put_slot[i] = FULL_SLOT;
            continue;
        }
        j.put_slot[i] = (u32)s;
        if (j.exp & 2) {
            if (!(j.exp & 1)) atomicMax(slot_stamp(&table[s], par), stamp_of(j.epoch, i));
            continue;
        }
        // combine in LDS: max (i+1) per slot within the block
        u32 h = (u32)(mix64((u64)s) & (K1_LDS - 1));
        for (;;) {
            const u32 old = atomicCAS(&s_slot[h], 0xFFFFFFFFu, (u32)s);
            if (old == 0xFFFFFFFFu || old == (u32)s) break;
            h = (h + 1) & (K1_LDS - 1);
        }
        atomicMax(&s_max[h], (u32)(i + 1));
        hq[q] = h;
        sl_idx[q] = (u64)s;
    }
    // one key-count atomic per block: a same-address atomic per thread serialises at the
    // memory side (16k new keys cost ~16 us that way)
    if (created) atomicAdd(&s_created, created);
    __syncthreads();
    if constexpr (BK) {
        // Bucket election: no stamp atomics. The block's distinct (slot, last i+1) pairs go to
        // its tile of bk_ent grouped by slot bucket (order inside a bucket is irrelevant: the
        // elector takes the maximum); bk_cnt[bucket][block] says where.
        // the block's last record per slot is the one whose i+1 won the LDS combine; its
        // thread holds the value, so entries carry it and the elector gathers no records
        bool win[K1_ITEMS];
#pragma unroll
        for (int q = 0; q < K1_ITEMS; q++) {
            const u64 i = base + (u64)q * TPB + threadIdx.x;
            win[q] = hq[q] != ~0u && s_max[hq[q]] == (u32)(i + 1);
            if (win[q]) atomicAdd(&s_bk[(u32)sl_idx[q] >> j.bk_shift], 1u);
        }
        __syncthreads();
        constexpr int PER = HM_BK_MAX / TPB;  // buckets per thread (bk_nb <= HM_BK_MAX)
        u32 c[PER], loc = 0;
#pragma unroll
        for (int r = 0; r < PER; r++) {
            const u32 b = threadIdx.x * PER + r;
            c[r] = b < j.bk_nb ? s_bk[b] : 0u;
            loc += c[r];
        }
        const u32 run = block_scan_excl(loc, nullptr);
        __syncthreads();
        u32 off = run;
#pragma unroll
        for (int r = 0; r < PER; r++) {
            const u32 b = threadIdx.x * PER + r;
            if (b < j.bk_nb) {
                j.bk_cnt[(u64)b * j.nblocks + blk] = (off << 16) | c[r];
                s_bk[b] = off;
            }
            off += c[r];
        }
        __syncthreads();
        u64x2* ent = j.bk_ent + (u64)blk * K1_TILE;
#pragma unroll
        for (int q = 0; q < K1_ITEMS; q++) {
            if (!win[q]) continue;
            const u64 i = base + (u64)q * TPB + threadIdx.x;
            u64x2 e;
            e.x = (sl_idx[q] << 32) | (u64)(i + 1);
            e.y = rec[q].val;
            ent[atomicAdd(&s_bk[(u32)sl_idx[q] >> j.bk_shift], 1u)] = e;
        }
    } else {
        for (int q = threadIdx.x; q < K1_LDS; q += TPB) {
            const u32 s = s_slot[q];
            if (s != 0xFFFFFFFFu && !(j.exp & 1))
                atomicMax(slot_stamp(&table[s], par), ((u64)j.epoch << 32) | s_max[q]);
        }
    }
    // keys created by this block: spread over HM_CREATED_SLOTS counters (summed by hm_count);
    // one same-address atomic per block would serialise at the memory side (~88 per us)
    if (threadIdx.x == 0 && s_created) atomicAdd(&j.created_acc[blk % HM_CREATED_SLOTS], (u64)s_created);
}

// ---- role: apply(e) -------------------------------------------------------------------------
__device__ __forceinline__ void apply_role(ApplyJob j, u32 blk, Slot* table, DevCtl* ctl) {
    const u64 i = (u64)blk * TPB + threadIdx.x;
    if (i >= j.n) return;
    const u32 par = j.epoch & 1;
    const u32 s = j.put_slot[i];
    const u64 want = stamp_of(j.epoch, i);
    if (s == SIDE_SLOT) {
        if (*slot_stamp(&ctl->sp, par) == want) ctl->sp.val = j.rec.at(i).val;
    } else if (s != FULL_SLOT) {
        if (*slot_stamp(&table[s], par) == want) table[s].val = j.rec.at(i).val;
    }
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

// One launch = {index(e)} + {apply(p)} + {reads(p)} over disjoint block ranges (any may be
// empty). Index blocks come first so the latency-bound pass is dispatched first (reads first:
// B1 37.0 -> 40.5 us, 50 % writes 66.6 -> 75.8 us; profiles/r01_variants/block_order.txt).
template <int K1_ITEMS, int G, bool BK>
__global__ __launch_bounds__(TPB) void hm_round_kernel(IndexJob ij, ApplyJob aj, ReadJob rj, Slot* table, u32 shift,
                                                       u64 tmask, DevCtl* ctl) {
    u32 b = blockIdx.x;
    if (b < ij.nblocks) {
        index_role<K1_ITEMS, BK>(ij, b, table, shift, tmask, ctl);
        return;
    }
    b -= ij.nblocks;
    if (b < aj.nblocks) {
        apply_role(aj, b, table, ctl);
        return;
    }
    b -= aj.nblocks;
    read_role<G>(rj, b, table, shift, tmask, ctl);
}

// Bucket election + apply of one round (the large-round alternative to the stamp atomics):
// one block per slot bucket gathers the bucket's (slot, i+1) entries from every index block's
// tile, keeps the maximum i+1 per slot in an LDS hash table (the last writer in log order) and
// stores that record's value into the slot: one plain store per distinct key instead of a
// scattered device atomic per Put (25.6 G/s) and a stamp re-read per Put in apply (plain
// scattered 8-B stores run at 69 G/s, profiles/r01_get_floor.txt). A bucket whose distinct
// slots overflow the table is redone in 2, 4, ... slot sub-ranges (the stores are idempotent).
// The side slot (key u64::MAX) keeps its stamp; block 0 applies it.
constexpr int HM_EL_HT = 2048;
constexpr int HM_EL_CH = 2048;  // entries gathered per pass (one u16 tile id each in LDS)
constexpr int HM_EL_PER = HM_EL_CH / TPB;
__global__ __launch_bounds__(TPB) void hm_elect_kernel(const u64x2* __restrict__ ent, const u32* __restrict__ cnt,
                                                       u32 nblocks, u32 tile, u32 bk_shift, RecSrc rec, Slot* table,
                                                       DevCtl* ctl, u32 epoch) {
    const u32 K1_TILE = tile;  // entries per index block (TPB x its Puts per thread)
    extern __shared__ u32 s_dyn[];    // s_pre[nblocks + 1] entry prefix, s_off[nblocks] (u16)
    __shared__ u32 s_hk[HM_EL_HT];
    __shared__ u32 s_hv[HM_EL_HT];
    __shared__ uint16_t s_tile[HM_EL_CH];
    u32* s_pre = s_dyn;
    uint16_t* s_off = (uint16_t*)(s_dyn + nblocks + 1);
    const u32 b = blockIdx.x;
    // this bucket's (offset, count) in every index tile; thread owns tiles [tid*K, tid*K + K)
    const u32 K = (nblocks + TPB - 1) / TPB;
    u32 loc = 0;
    for (u32 q = 0; q < K; q++) {
        const u32 t = threadIdx.x * K + q;
        if (t < nblocks) {
            const u32 v = cnt[(u64)b * nblocks + t];
            s_off[t] = (uint16_t)(v >> 16);
            s_pre[t] = v & 0xFFFFu;
            loc += v & 0xFFFFu;
        }
    }
    u32 total;
    u32 run = block_scan_excl(loc, &total);
    for (u32 q = 0; q < K; q++) {
        const u32 t = threadIdx.x * K + q;
        if (t < nblocks) {
            const u32 c = s_pre[t];
            s_pre[t] = run;
            run += c;
        }
    }
    if (threadIdx.x == 0) s_pre[nblocks] = total;
    u32 lp = 0;  // parts = 2^lp slot sub-ranges of the bucket, about <= HT/2 entries each
    while ((total >> lp) > HM_EL_HT / 2 && lp < bk_shift) lp++;
    __syncthreads();
    u64x2 x[HM_EL_PER];
    // the chunk [base, base + CH) of this bucket's entries into registers, all loads in flight
    auto load_chunk = [&](u32 base) {
        for (u32 q = 0; q < K; q++) {
            const u32 t = threadIdx.x * K + q;
            if (t >= nblocks) break;
            const u32 lo_ = s_pre[t] > base ? s_pre[t] : base;
            const u32 hi_ = s_pre[t + 1] < base + HM_EL_CH ? s_pre[t + 1] : base + HM_EL_CH;
            for (u32 i = lo_; i < hi_; i++) s_tile[i - base] = (uint16_t)t;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < HM_EL_PER; r++) {
            const u32 i = base + r * TPB + threadIdx.x;
            x[r].x = ~0ull;
            if (i < total) {
                const u32 t = s_tile[i - base];
                x[r] = ent[(u64)t * K1_TILE + s_off[t] + (i - s_pre[t])];
            }
        }
        __syncthreads();  // s_tile is reused by the next chunk
    };
    auto in_part = [&](u32 sl, u32 p) { return !lp || ((sl >> (bk_shift - lp)) & ((1u << lp) - 1)) == p; };
    const bool one_chunk = total <= (u32)HM_EL_CH;
    for (u32 p = 0; p < (1u << lp);) {
        for (int q = threadIdx.x; q < HM_EL_HT; q += TPB) {
            s_hk[q] = 0xFFFFFFFFu;
            s_hv[q] = 0;
        }
        bool ovf = false;
        for (u32 base = 0; base < total; base += HM_EL_CH) {  // 1: latest i+1 per slot
            load_chunk(base);
#pragma unroll
            for (int r = 0; r < HM_EL_PER; r++) {
                if (x[r].x == ~0ull) continue;
                const u32 sl = (u32)(x[r].x >> 32);
                if (!in_part(sl, p)) continue;
                u32 h = (u32)(mix64(sl) & (HM_EL_HT - 1));
                int pr = 0;
                for (; pr < HM_EL_HT; pr++) {
                    const u32 old = atomicCAS(&s_hk[h], 0xFFFFFFFFu, sl);
                    if (old == 0xFFFFFFFFu || old == sl) break;
                    h = (h + 1) & (HM_EL_HT - 1);
                }
                if (pr == HM_EL_HT) ovf = true;
                else atomicMax(&s_hv[h], (u32)x[r].x);
            }
        }
        if (__syncthreads_or(ovf)) {  // more distinct slots than the table holds: finer parts
            lp++;
            p = 0;
            continue;
        }
        for (u32 base = 0; base < total; base += HM_EL_CH) {  // 2: the winners store their values
            if (!one_chunk) load_chunk(base);
#pragma unroll
            for (int r = 0; r < HM_EL_PER; r++) {
                if (x[r].x == ~0ull) continue;
                const u32 sl = (u32)(x[r].x >> 32);
                if (!in_part(sl, p)) continue;
                u32 h = (u32)(mix64(sl) & (HM_EL_HT - 1));
                while (s_hk[h] != sl) h = (h + 1) & (HM_EL_HT - 1);
                if (s_hv[h] == (u32)x[r].x) table[sl].val = x[r].y;
            }
        }
        __syncthreads();
        p++;
    }
    if (b == 0 && threadIdx.x == 0) {
        const u64 st = *slot_stamp(&ctl->sp, epoch & 1);
        if ((u32)(st >> 32) == epoch) ctl->sp.val = rec.at((u64)(u32)st - 1).val;
    }
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

// number of keys = direct inserts (ctl->nkeys) + keys created by replay rounds
__global__ __launch_bounds__(TPB) void hm_count_kernel(const u64* __restrict__ acc, u64 n, DevCtl* ctl) {
    __shared__ u64 s_w[TPB / 64];
    u64 x = 0;
    for (u64 q = threadIdx.x; q < n; q += TPB) x += acc[q];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 t = ctl->nkeys;
        for (int w = 0; w < TPB / 64; w++) t += s_w[w];
        ctl->nkeys_total = t;
    }
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
    __shared__ u64 s_c[TPB / 64], s_s[TPB / 64], s_x[TPB / 64];
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
        c = sm = x = 0;
        for (int v = 0; v < TPB / 64; v++) {
            c += s_c[v];
            sm += s_s[v];
            x ^= s_x[v];
        }
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

// ---- owner path: partitioned replay of large rounds (no election atomics, no apply pass) -----
//
// A round's Puts are split by the top 8 bits of mix64(key) (the home slot's top bits) into
// 256 buckets; every key belongs to exactly one bucket, and one block of hm_own_kernel owns
// each (bucket, sub-bucket). That block picks every key's last writer in LDS and stores the
// value into the slot itself, so no global atomicMax elects writers and no apply pass runs:
//
//   hm_part_kernel  tiles of 1024 Puts in ticket order: dedup by key in LDS (the tile's last
//                   writer and its value), count per bucket, decoupled look-back over the
//                   tiles' per-bucket counts (the rs_pass scheme), scatter (key, value) into
//                   fixed-capacity bucket regions. Look-back offsets keep tile order inside a
//                   region, so a key's last writer is its LAST entry in the region. Entries past
//                   a region's capacity go to an overflow list with their would-be position.
//   hm_own_kernel   per (bucket, sub-bucket): the max region position per key in LDS, then
//                   find-or-claim the slot and store the value; the side-slot key rides the
//                   usual stamp (one atomicMax per Put of key u64::MAX, applied by block 0).
//
// Reads of the round run after hm_own_kernel (next launch) and see the values in the slots.
//
// Status: opt-in (NRG_OWNER_MIN), parity-green, SLOWER than the stamp path on MI355X
// (profiles/r01_variants/owner_path.txt): at 800k Puts + 900k Gets per round 135 us vs 110 us
// (part 40 us, own 65 us); at B1 65 us vs 37 us. The part pass alone has a ~10 us latency
// floor (load, LDS count, look-back, scatter) plus 7 us of LDS dedup at 100k Puts, so the
// global atomics it removes (45 us at 800k) are not recovered. Kept for the next round's work
// on the write path.
constexpr int PT_KP = 8;
constexpr int PT_TILE = TPB * PT_KP;  // 2048 Puts per part tile
constexpr int PT_LDS = 2 * PT_TILE;   // dedup table entries
constexpr int NBKT = 256;             // buckets (one look-back digit per thread)
constexpr int OW_LDS = 2048;          // per-block key table of hm_own_kernel
constexpr u32 OW_CLASS = 1024;        // region entries per class (table load <= 1/2)
constexpr int OW_K = OW_LDS / TPB;    // elected keys per thread, loads issued together
constexpr u32 PT_AGG = 1u << 30, PT_INC = 2u << 30, PT_MASK = 3u << 30, PT_CNT = (1u << 30) - 1;
constexpr int PT_WIN = 32;

__device__ __forceinline__ u32 bucket_of(u64 x) { return (u32)(x >> 56); }  // x = mix64(key)

struct PartBufs {
    u32* ticket;   // [1]
    u32* ovf_cnt;  // [1]
    u32* desc;     // [tiles][NBKT] look-back granules {status:2, count:30}
    u64* bkey;     // [NBKT][cap]
    u64* bval;     // [NBKT][cap]
    u64* okey;     // overflow entries
    u64* oval;
    u32* opos;     // would-be region position
    u32* obkt;     // bucket
    u64 cap;
};

__global__ __launch_bounds__(TPB) void hm_part_kernel(RecSrc rec, nrg_put* ring_out, u64 n, u32 epoch, PartBufs pb,
                                                      DevCtl* ctl) {
    __shared__ u64 s_key[PT_LDS];
    __shared__ u32 s_max[PT_LDS];  // 1 + the tile offset of the key's last writer
    __shared__ u32 s_cnt[NBKT];
    __shared__ u32 s_excl[NBKT];
    __shared__ u32 s_tile;
    const int t = threadIdx.x;
    if (t == 0) s_tile = atomicAdd(pb.ticket, 1u);
    for (int q = t; q < PT_LDS; q += TPB) {
        s_key[q] = EMPTY_KEY;
        s_max[q] = 0;
    }
    s_cnt[t] = 0;
    __syncthreads();
    const u32 tile = s_tile;
    const u64 base = (u64)tile * PT_TILE;
    const u32 par = epoch & 1;
    nrg_put r[PT_KP];
#pragma unroll
    for (int q = 0; q < PT_KP; q++) {
        const u64 i = base + (u64)q * TPB + t;
        r[q] = i < n ? rec.at(i) : nrg_put{EMPTY_KEY, 0};
    }
    u32 hh[PT_KP];
#pragma unroll
    for (int q = 0; q < PT_KP; q++) {
        const u64 i = base + (u64)q * TPB + t;
        hh[q] = 0xFFFFFFFFu;
        if (i >= n) continue;
        if (ring_out) ring_out[(rec.lo + i) & rec.mask] = r[q];
        const u64 k = r[q].key;
        if (k == EMPTY_KEY) {  // the side-slot key keeps the stamp election (hm_own_kernel applies it)
            atomicMax(slot_stamp(&ctl->sp, par), stamp_of(epoch, i));
            continue;
        }
        u32 h = (u32)(mix64(k) >> 20) & (PT_LDS - 1);
        for (;;) {
            const u64 old = atomicCAS(&s_key[h], EMPTY_KEY, k);
            if (old == EMPTY_KEY || old == k) break;
            h = (h + 1) & (PT_LDS - 1);
        }
        atomicMax(&s_max[h], (u32)(i - base) + 1u);
        hh[q] = h;
    }
    __syncthreads();
    // per-bucket counts (the order inside a tile's run does not matter: one entry per key)
    u32 rk[PT_LDS / TPB];
#pragma unroll
    for (int e = 0; e < PT_LDS / TPB; e++) {
        const u64 k = s_key[e * TPB + t];
        rk[e] = k != EMPTY_KEY ? atomicAdd(&s_cnt[bucket_of(mix64(k))], 1u) : 0u;
    }
    __syncthreads();
    // thread t owns bucket t: publish the count, look back over earlier tiles
    const u32 tcnt = s_cnt[t];
    u32* my = pb.desc + (u64)tile * NBKT + t;
    __hip_atomic_store(my, (tile == 0 ? PT_INC : PT_AGG) | tcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    u32 excl = 0;
    if (tile > 0) {
        int tt = (int)tile - 1;
        for (;;) {
            u32 v[PT_WIN];
#pragma unroll
            for (int q = 0; q < PT_WIN; q++)
                v[q] = tt - q >= 0 ? __hip_atomic_load(pb.desc + (u64)(tt - q) * NBKT + t, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : PT_INC;
            int used = 0;
            bool done = false;
#pragma unroll
            for (int q = 0; q < PT_WIN; q++) {
                if (done || used < q) continue;
                const u32 st = v[q] & PT_MASK;
                if (st == 0) continue;
                excl += v[q] & PT_CNT;
                used = q + 1;
                if (st == PT_INC) done = true;
            }
            if (done) break;
            tt -= used;
            if (used < PT_WIN) __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store(my, PT_INC | (excl + tcnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    s_excl[t] = excl;
    __syncthreads();
#pragma unroll
    for (int e = 0; e < PT_LDS / TPB; e++) {
        const u64 k = s_key[e * TPB + t];
        if (k == EMPTY_KEY) continue;
        const u32 b = bucket_of(mix64(k));
        const u32 pos = s_excl[b] + rk[e];
        const u64 v = rec.at(base + s_max[e * TPB + t] - 1).val;  // the tile's records are still cached
        if (pos < pb.cap) {
            pb.bkey[(u64)b * pb.cap + pos] = k;
            pb.bval[(u64)b * pb.cap + pos] = v;
        } else {
            const u32 o = atomicAdd(pb.ovf_cnt, 1u);
            pb.okey[o] = k;
            pb.oval[o] = v;
            pb.opos[o] = pos;
            pb.obkt[o] = b;
        }
    }
}

__global__ __launch_bounds__(TPB) void hm_own_kernel(RecSrc rec, u32 epoch, u32 ntiles, PartBufs pb, u32 split,
                                                     Slot* table, u32 shift, u64 tmask, DevCtl* ctl,
                                                     u64* created_acc, u32* clear_desc, u64 clear_words,
                                                     u32* clear_ctl) {
    __shared__ u64 s_k[OW_LDS];
    __shared__ u64 s_w[OW_LDS];  // max of ((region position + 1) << 32 | overflow index)
    __shared__ uint16_t s_list[OW_LDS];
    __shared__ u32 s_created, s_full, s_n;
    const int t = threadIdx.x;
    const u32 o = blockIdx.x;
    const u32 b = o / split, sub = o % split;
    // the other parity's buffers (used two owner rounds ago) are cleared for the next round
    for (u64 q = (u64)o * TPB + t; q < clear_words; q += (u64)gridDim.x * TPB) clear_desc[q] = 0;
    if (o == 0 && t < 2) clear_ctl[t] = 0;
    const u32 total = pb.desc[(u64)(ntiles - 1) * NBKT + b] & PT_CNT;  // last tile's inclusive count
    const u32 nin = total < pb.cap ? total : (u32)pb.cap;
    const u32 novf = total > pb.cap ? *pb.ovf_cnt : 0u;
    const u32 mine = (total + split - 1) / split;  // region entries of this sub-bucket, about
    const u32 classes = mine > OW_CLASS ? (mine + OW_CLASS - 1) / OW_CLASS : 1u;
    if (t == 0) {
        s_created = 0;
        s_full = 0;
    }
    u32 created = 0;
    for (u32 c = 0; c < classes; c++) {
        for (int q = t; q < OW_LDS; q += TPB) {
            s_k[q] = EMPTY_KEY;
            s_w[q] = 0;
        }
        __syncthreads();
        for (u32 p = t; p < nin + novf; p += TPB) {
            u64 k, w;
            if (p < nin) {
                k = pb.bkey[(u64)b * pb.cap + p];
                w = ((u64)(p + 1) << 32);
            } else {
                const u32 q = p - nin;
                if (pb.obkt[q] != b) continue;
                k = pb.okey[q];
                w = ((u64)(pb.opos[q] + 1) << 32) | q;
            }
            const u64 x = mix64(k);
            if (((x >> 40) & (split - 1)) != sub) continue;
            if (classes > 1 && (u32)((x >> 8) % classes) != c) continue;
            u32 h = (u32)(x >> 20) & (OW_LDS - 1);
            u32 tries = 0;
            for (;;) {
                const u64 old = atomicCAS(&s_k[h], EMPTY_KEY, k);
                if (old == EMPTY_KEY || old == k) break;
                h = (h + 1) & (OW_LDS - 1);
                if (++tries == OW_LDS) {
                    s_full = 1;
                    break;
                }
            }
            if (tries < OW_LDS) atomicMax(&s_w[h], w);
        }
        __syncthreads();
        // compact the elected keys, then give each thread up to OW_K of them with every value
        // load and first probe in flight together
        if (t == 0) s_n = 0;
        __syncthreads();
#pragma unroll
        for (int e = 0; e < OW_K; e++) {
            const int q = e * TPB + t;
            if (s_k[q] != EMPTY_KEY) s_list[atomicAdd(&s_n, 1u)] = (uint16_t)q;
        }
        __syncthreads();
        const u32 nl = s_n;
        u64 kk[OW_K], vv[OW_K], k0[OW_K], hs[OW_K];
#pragma unroll
        for (int e = 0; e < OW_K; e++) {
            const u32 li = (u32)e * TPB + t;
            kk[e] = EMPTY_KEY;
            if (li >= nl) continue;
            const u32 q = s_list[li];
            kk[e] = s_k[q];
            const u64 w = s_w[q];
            const u32 pos = (u32)(w >> 32) - 1;
            vv[e] = pos < pb.cap ? pb.bval[(u64)b * pb.cap + pos] : pb.oval[(u32)w];
            hs[e] = table_home(kk[e], shift);
            k0[e] = table[hs[e]].key;
        }
#pragma unroll
        for (int e = 0; e < OW_K; e++) {
            if (kk[e] == EMPTY_KEY) continue;
            const long long sl = find_or_claim(table, kk[e], hs[e], tmask, k0[e], epoch, &created);
            if (sl < 0) {
                atomicOr(&ctl->err, ERR_TABLE_FULL);
                continue;
            }
            table[sl].val = vv[e];
        }
        __syncthreads();
    }
    if (s_full) atomicOr(&ctl->err, ERR_TABLE_FULL);  // LDS table overflow (hash skew): reported, not hidden
    if (o == 0 && t == 0) {  // the side slot
        const u64 st = *slot_stamp(&ctl->sp, epoch & 1);
        if ((u32)(st >> 32) == epoch) {
            if (ctl->sp.created == 0) {
                ctl->sp.created = epoch;
                created++;
            }
            ctl->sp.val = rec.at((u64)(u32)st - 1).val;
        }
    }
    if (created) atomicAdd(&s_created, created);
    __syncthreads();
    if (t == 0 && s_created) atomicAdd(&created_acc[o % HM_CREATED_SLOTS], (u64)s_created);
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

template <int K1, int G, bool BK = false>
static void launch_round(nrg_ctx* c, const IndexJob& ij, const ApplyJob& aj, const ReadJob& rj) {
    const u32 blocks = ij.nblocks + aj.nblocks + rj.nblocks;
    NRG_LAUNCH(c, "hm_round", (hm_round_kernel<K1, G, BK>), blocks, TPB, 0, c->stream, ij, aj, rj, c->d_table,
               c->slot_shift, (u64)(c->slots - 1), c->d_ctl);
}

// Puts per index thread in bucket rounds: 4 below 600k Puts, 8 above (400k + 900k Gets: 64.3
// vs 68.4 us per round; 500k + 500k: 67.9 vs 71.9; 800k + 900k: 99.7 vs 95.7). NRG_BK_K1 overrides.
static u32 bk_k1(const nrg_ctx* c, u64 n) { return c->bk_k1 ? c->bk_k1 : (n >= 600000 ? 8u : 4u); }

static hipError_t launch(nrg_ctx* c, IndexJob& ij, ApplyJob& aj, ReadJob& rj) {
    // Puts per index thread: a hot key costs one same-address stamp atomic per index block
    // that holds it (same-address atomics serialise), so large (write-heavy) rounds use fewer,
    // bigger blocks (Zipf 0.99 at 50 % writes: 99 us with 1, 79 with 4, 65 with 8; uniform
    // unchanged); small rounds use 2 (B1: 36.4 us with 1 or 2, 39.0 with 4; Zipf 0.99 at 10 %
    // writes: 54.2 with 1, 47.7 with 2, 39.2 with 4). NRG_K1_ITEMS overrides.
    const bool bk = ij.bk_ent != nullptr;  // bucket election: 8 Puts per index thread
    const u32 k1 = bk ? bk_k1(c, ij.n) : c->k1_items ? c->k1_items : (ij.n >= (1u << 18) ? 8 : 2);
    const u32 K1 = k1 >= 8 ? 8 : k1 >= 4 ? 4 : (k1 == 2 ? 2 : 1);
    const u32 G = c->gets_per_thread >= 4 ? 4 : (c->gets_per_thread == 2 ? 2 : 1);
    ij.exp = c->exp;
    ij.created_acc = c->d_created;
    if (c->exp & 4) aj.n = 0;
    if (c->exp & 8) ij.n = 0;
    ij.nblocks = (u32)((ij.n + TPB * K1 - 1) / (TPB * K1));
    aj.nblocks = (u32)((aj.n + TPB - 1) / TPB);
    rj.nblocks = (u32)((rj.R + TPB * G - 1) / (TPB * G));
    if (ij.nblocks + aj.nblocks + rj.nblocks == 0) return hipSuccess;
    if (bk) {
        if (K1 == 4) launch_round<4, 1, true>(c, ij, aj, rj);
        else if (K1 == 2) launch_round<2, 1, true>(c, ij, aj, rj);
        else launch_round<8, 1, true>(c, ij, aj, rj);
        return hipGetLastError();
    }
#define NRG_RK(A, B) \
    if (K1 == A && G == B) launch_round<A, B>(c, ij, aj, rj)
    NRG_RK(1, 1); else NRG_RK(1, 2); else NRG_RK(1, 4); else NRG_RK(2, 1); else NRG_RK(2, 2); else NRG_RK(2, 4);
    else NRG_RK(4, 1); else NRG_RK(4, 2); else NRG_RK(4, 4); else NRG_RK(8, 1);
#undef NRG_RK
    return hipGetLastError();
}

static void deferred_jobs(nrg_ctx* c, ApplyJob& aj, ReadJob& rj) {
    aj = ApplyJob{};
    rj = ReadJob{};
    const HmDeferred& p = c->pend;
    if (!p.valid) return;
    aj.rec = ring_src(c, p.src, p.lo);
    aj.n = p.n;
    aj.put_slot = c->d_put_slot[p.epoch & 1];
    aj.epoch = p.epoch;
    rj.rec = aj.rec;
    rj.keys = p.keys;
    rj.R = p.R;
    rj.vals = p.vals;
    rj.found = p.found;
    rj.epoch = p.epoch;
}

hipError_t hm_flush(nrg_ctx* c) {
    if (!c->pend.valid) return hipSuccess;
    IndexJob ij{};
    ApplyJob aj;
    ReadJob rj;
    deferred_jobs(c, aj, rj);
    c->pend.valid = false;
    return launch(c, ij, aj, rj);
}

// Reads against the current state (no writes): attached to the deferred round if it has none.
static hipError_t hm_reads(nrg_ctx* c, const u64* keys, u64 R, u64* vals, uint8_t* found) {
    if (R == 0) return hipSuccess;
    if (c->pend.valid && c->pend.R == 0) {
        c->pend.keys = keys;
        c->pend.R = R;
        c->pend.vals = vals;
        c->pend.found = found;
        return hm_flush(c);
    }
    hipError_t e = hm_flush(c);
    if (e != hipSuccess) return e;
    IndexJob ij{};
    ApplyJob aj{};
    ReadJob rj{};
    rj.keys = keys;
    rj.R = R;
    rj.vals = vals;
    rj.found = found;
    rj.epoch = c->epoch;  // every earlier round is applied: values come from the slots
    return launch(c, ij, aj, rj);
}

hipError_t hm_owner_alloc(nrg_ctx* c, u64 mb) {
    OwnerBufs& ob = c->own;
    ob.cap = 2 * ((mb + NBKT - 1) / NBKT) + 4096;
    const u64 tiles = (mb + PT_TILE - 1) / PT_TILE;
    hipError_t e;
#define OB_ALLOC(P, BYTES)                     \
    if ((e = hipMalloc(&(P), (BYTES))) != hipSuccess) return e;
    OB_ALLOC(ob.ctl, 4 * sizeof(u32));
    OB_ALLOC(ob.desc[0], tiles * NBKT * sizeof(u32));
    OB_ALLOC(ob.desc[1], tiles * NBKT * sizeof(u32));
    OB_ALLOC(ob.bkey, NBKT * ob.cap * sizeof(u64));
    OB_ALLOC(ob.bval, NBKT * ob.cap * sizeof(u64));
    OB_ALLOC(ob.okey, mb * sizeof(u64));
    OB_ALLOC(ob.oval, mb * sizeof(u64));
    OB_ALLOC(ob.opos, mb * sizeof(u32));
    OB_ALLOC(ob.obkt, mb * sizeof(u32));
#undef OB_ALLOC
    if ((e = hipMemsetAsync(ob.ctl, 0, 4 * sizeof(u32), c->stream)) != hipSuccess) return e;
    for (int i = 0; i < 2; i++)
        if ((e = hipMemsetAsync(ob.desc[i], 0, tiles * NBKT * sizeof(u32), c->stream)) != hipSuccess) return e;
    return hipSuccess;
}

void hm_owner_free(nrg_ctx* c) {
    OwnerBufs& ob = c->own;
    void* ptrs[] = {ob.ctl, ob.desc[0], ob.desc[1], ob.bkey, ob.bval, ob.okey, ob.oval, ob.opos, ob.obkt};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    ob = OwnerBufs{};
}

// One owner-path round (see hm_part_kernel): partition, then elect + store per bucket.
static hipError_t owner_round(nrg_ctx* c, const nrg_put* src, nrg_put* ring_out, u64 lo, u64 n, u32 epoch) {
    OwnerBufs& ob = c->own;
    const u32 set = c->owner_rounds++ & 1;
    PartBufs pb;
    pb.ticket = ob.ctl + 2 * set;
    pb.ovf_cnt = ob.ctl + 2 * set + 1;
    pb.desc = ob.desc[set];
    pb.bkey = ob.bkey;
    pb.bval = ob.bval;
    pb.okey = ob.okey;
    pb.oval = ob.oval;
    pb.opos = ob.opos;
    pb.obkt = ob.obkt;
    pb.cap = ob.cap;
    const u64 tiles = (n + PT_TILE - 1) / PT_TILE;
    const RecSrc rs = ring_src(c, src, lo);
    NRG_LAUNCH(c, "hm_part", hm_part_kernel, (unsigned)tiles, TPB, 0, c->stream, rs, ring_out, n, epoch, pb, c->d_ctl);
    u32 split = 1;  // sub-buckets per bucket: about <= 768 region entries per owner block
    while ((u64)split * NBKT * 768 < n && split < 64) split <<= 1;
    NRG_LAUNCH(c, "hm_own", hm_own_kernel, NBKT * split, TPB, 0, c->stream, rs, epoch, (u32)tiles, pb, split,
               c->d_table, c->slot_shift, (u64)(c->slots - 1), c->d_ctl, c->d_created, ob.desc[set ^ 1],
               ob.tiles[set ^ 1] * NBKT, ob.ctl + 2 * (set ^ 1));
    ob.tiles[set] = tiles;
    ob.tiles[set ^ 1] = 0;  // cleared by this launch
    return hipGetLastError();
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
    const bool want_prev = d_prev && resp_lo < lo + n && resp_hi > lo;
    if (c->owner_min && n >= c->owner_min && !want_prev) {
        // the previous round's apply + reads see the table before this round's stores
        hipError_t e = hm_flush(c);
        if (e != hipSuccess) return e;
        const u32 epoch = ++c->epoch;
        e = owner_round(c, src, write_ring ? (nrg_put*)c->d_ring : nullptr, lo, n, epoch);
        if (e != hipSuccess) return e;
        const nrg_put* keep = (src && !write_ring) ? src : nullptr;
        HmDeferred& p = c->pend;  // reads only: the values are already in the slots
        p.valid = true;
        p.epoch = epoch;
        p.src = keep;
        p.lo = lo;
        p.n = 0;
        p.keys = d_get_keys;
        p.R = R;
        p.vals = d_get_vals;
        p.found = d_get_found;
        if (!c->pipeline || keep) return hm_flush(c);
        return hipGetLastError();
    }
    const u32 epoch = ++c->epoch;
    IndexJob ij{};
    ij.rec = ring_src(c, src, lo);
    ij.ring_out = write_ring ? (nrg_put*)c->d_ring : nullptr;
    ij.n = n;
    ij.put_slot = c->d_put_slot[epoch & 1];
    ij.epoch = epoch;
    const bool bk = c->elect_min && n >= c->elect_min && !want_prev;
    if (bk) {  // buckets of about 1024 entries (a power of two in [64, HM_BK_MAX])
        u32 nb_log = 6;
        while ((1ull << nb_log) * 1024 < n && (1u << nb_log) < HM_BK_MAX) nb_log++;
        if (nb_log > 64 - c->slot_shift) nb_log = 64 - c->slot_shift;
        ij.bk_ent = (u64x2*)c->d_bk_ent;
        ij.bk_cnt = c->d_bk_cnt;
        ij.bk_nb = 1u << nb_log;
        ij.bk_shift = (64 - c->slot_shift) - nb_log;
    }
    ApplyJob aj;
    ReadJob rj;
    deferred_jobs(c, aj, rj);  // the previous round's second half rides along
    c->pend.valid = false;
    hipError_t e = launch(c, ij, aj, rj);
    if (e != hipSuccess) return e;
    // records of this round for its deferred half: the ring copy if there is one
    const nrg_put* keep = (src && !write_ring) ? src : nullptr;
    if (bk) {
        const u32 nblocks = ij.nblocks;  // index tiles of TPB * bk_k1 Puts
        NRG_LAUNCH(c, "hm_elect", hm_elect_kernel, ij.bk_nb, TPB, (nblocks + 1) * 4 + nblocks * 2, c->stream, (const u64x2*)c->d_bk_ent,
                   c->d_bk_cnt, nblocks, TPB * bk_k1(c, n), ij.bk_shift, ring_src(c, keep, lo), c->d_table, c->d_ctl, epoch);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (d_prev && resp_lo < lo + n && resp_hi > lo) {
        u32 *sk = nullptr, *sv = nullptr;
        timer_begin(c, "hm_prev", c->stream);
        // slot ids < 2^31; the side-slot (0xFFFFFFFF) and full (0xFFFFFFFE) markers sort last
        e = sort_pairs(c->sort, c->d_put_slot[epoch & 1], nullptr, n, 32, c->stream, &sk, &sv);
        if (e != hipSuccess) return e;
        hm_prev_kernel<<<(unsigned)((n + TPB - 1) / TPB), TPB, 0, c->stream>>>(
            sk, sv, n, ring_src(c, keep, lo), c->d_table, c->d_ctl, epoch, resp_lo, resp_hi, d_prev, d_prev_found);
        timer_end(c, "hm_prev", c->stream);
    }
    HmDeferred& p = c->pend;
    p.valid = true;
    p.epoch = epoch;
    p.src = keep;
    p.lo = lo;
    p.n = bk ? 0 : n;  // bucket rounds were applied by hm_elect_kernel: reads only
    p.keys = d_get_keys;
    p.R = R;
    p.vals = d_get_vals;
    p.found = d_get_found;
    if (!c->pipeline || keep) return hm_flush(c);
    return hipGetLastError();
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
    hm_count_kernel<<<1, TPB, 0, c->stream>>>(c->d_created, HM_CREATED_SLOTS, c->d_ctl);
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
