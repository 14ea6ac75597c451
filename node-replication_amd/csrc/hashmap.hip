// hashmap.hip — NrHashMap replica replay on gfx950.
//
// Replaces the hot loop of Log::exec -> NrHashMap::dispatch_mut (nr/src/log.rs:494-518,
// benches/hashmap.rs:114-119, nr/examples/hashmap.rs:46-50) and the read path
// Replica::read_only -> dispatch (nr/src/replica.rs:483-497, benches/hashmap.rs:107-111).
//
// Table: 2^k open-addressing slots of 32 B {key, value, stamp[2]} (common.hpp), linear probing
// from mix64(key) >> (64 - k); the one key equal to the empty marker lives in DevCtl::sp. Every
// replay round covers the log records [lo, lo+n) and takes a fresh epoch e. Two schedules:
//
// Stamp rounds (no previous-value responses, key stream not skewed): ONE launch per round,
//   {index(e) | apply(e-1) | reads(e-1)} on disjoint block ranges of hm_round_kernel:
//   index(e)   per Put: find the key's slot or claim an empty one (64-bit CAS; a fresh slot is
//              marked in the other parity, stamp (e, 0), so the reads of round e-1 running in
//              the same launch see it as absent); elect the round's last writer of every key
//              with atomicMax(st[e&1], e << 32 | i+1), pre-combined per block in LDS.
//   apply(e-1) per Put: the elected writer (st == (e-1, i+1)) stores its value.
//   reads(e-1) a key is present iff its stamp of parity e-1 is nonzero with epoch <= e-1; if the
//              epoch is e-1 the value is the elected record's (apply may be storing it).
//   index(e) touches only st[e&1], claims of empty slots and values apply never reads; apply and
//   reads look only at st[(e-1)&1]. The latency-bound index pass overlaps the reads.
// Partition rounds (previous-value responses, skewed key streams -- see skew_sample -- and rounds
//   of >= PART_MIN Puts): TWO launches per round and no device atomic per Put.
//   hm_round_kernel {partition(e) | reads(e-1)}: partition(e) only reads the records; each tile
//   writes its Puts grouped by the bucket of their key's HOME slot, in log order inside a
//   bucket, and a [tile][bucket] count word (the table is not touched, so the previous round's
//   reads run beside it against a quiescent table, without stamps);
//   hm_papply_kernel(e): one workgroup per bucket takes the bucket's entries (every tile's run,
//   tile order = log order) in chunks, finds each key's last writer in an LDS hash, and that
//   thread finds or claims the key's slot and stores its value: one table line read and written
//   per distinct key. All Puts of a key share its home bucket, so one workgroup decides each key.
//   512-thread workgroups over <= 512 buckets for rounds of >= 64k Puts (256 over <= 1024
//   below), buckets dealt to XCDs in contiguous ranges, the next chunk's entries loaded while a
//   chunk resolves. It runs at the memory-side request floor (profiles/r04_papply_phases.txt).
//   With previous values every Put keeps its entry and one wave walks each chunk in log order:
//   a Put's previous value is its predecessor's, else the key's value before the chunk, else None.
#include <cstring>

#include "internal.hpp"

namespace nrg {

typedef u64 u64x2 __attribute__((ext_vector_type(2)));

// Streaming (nt) stores for the streamed outputs (log copy, read responses) of partition-round and
// reads-only launches: plain stores leave them dirty in the XCD's L2 for the kernel-end write-back
// after the last workgroup; streamed, they drain during the kernel. N = 8 per-GPU round 78.7 vs
// 80.5 us, configs[2] 256.9 vs 263.4; stamp rounds keep plain stores (B1 34.5-34.7 plain vs
// 34.7-35.0 streamed; profiles/r04_nt_stores.txt). NRG_KNOB_EXP bit 6 = plain everywhere (A/B).
// Round 6: the compiler merges st_out's two branches into one plain store and drops the hint, so
// only the 16-B log copy (st_rec) is streamed; the responses are plain stores. Streamed for real
// (the plain branch as a relaxed wavefront-scope atomic store, which is not merged) they measured
// the same on one box: B1 34.15-34.19 us per round by the window (stamp-round reads streamed) vs
// 34.16-34.17, N = 8 per-GPU round 77.2-77.3 both, configs[2] 250.2 vs 250.7
// (profiles/r06/nt_single_stores.txt).
template <typename T>
__device__ __forceinline__ void st_out(T* p, T v, bool plain) {
    if (plain) *p = v;
    else __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ void st_rec(nrg_put* p, const nrg_put& r, bool plain) {
    if (plain) *p = r;
    else __builtin_nontemporal_store(u64x2{r.key, r.val}, (u64x2*)p);
}

// Round 6 (profiles/r06/b1_apply_nt.txt): the stamp-round apply's random value stores are streamed
// (NRG_HM_APPLY_NT): they drain during the launch instead of in its end-of-kernel L2 write-back.
// Same box, three pairs: 34.16-34.20 -> 33.93-34.02 us per B1 step (window 34.03-34.13 ->
// 33.80-33.97); the driver's 20 steps 27,507-27,866 -> 27,823-27,875 Mops/s. Streaming the index
// role's put_slot / win / over words (NRG_HM_TAG_NT) was slower (34.49-34.53 vs 34.25). Build
// with =0 / =1 for the A/B.
#ifndef NRG_HM_APPLY_NT
#define NRG_HM_APPLY_NT 1
#endif
#ifndef NRG_HM_TAG_NT
#define NRG_HM_TAG_NT 0
#endif
// The partition apply's value stores are streamed in rounds of at most PA_NT_MAX Puts: same box,
// two pairs, N = 8 per-GPU round (800k Puts + 900k Gets) 77.24-77.35 -> 75.35-75.57 us, 50 % writes
// 53.7-53.8 -> 53.1-53.2; configs[2]'s 4M Puts slower streamed (251.1-251.3 -> 257.3-258.3), so
// they stay plain above it (profiles/r06/papply_nt.txt). NRG_HM_PA_NT=0 builds it plain throughout.
#ifndef NRG_HM_PA_NT
#define NRG_HM_PA_NT 1
#endif
constexpr u64 PA_NT_MAX = NRG_HM_PA_NT ? 2000000 : 0;
template <bool NT, typename T>
__device__ __forceinline__ void st_pol(T* p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

constexpr int TPB = 256;
constexpr u32 SIDE_ID = 0x7FFFFFFFu;    // slot id standing for the side slot (slot ids are < 2^30)
constexpr u32 FULL_SLOT = 0xFFFFFFFFu;  // no slot could be claimed (table full)

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
    u32 nblocks;
    u32 nb_log;    // slot buckets = 1 << nb_log
    u32 bk_shift;  // bucket of a slot id = id >> bk_shift
    u64x2* ent;    // [nblocks][tile] {id << 32 | i+1, value}
    u32* eidx;     // partition rounds: [nblocks][tile] round offset i of each entry (previous values)
    u32* cnt;      // [bucket][nblocks] start << 16 | count
    u32 exp;       // diagnostic knobs (NRG_EXP; results are wrong when set): 1 no dedup, 2 no
                   // probe (every key new), 4 no ranking/entries
    u64* dup_acc;  // [HM_DUP_SLOTS] Puts overwritten inside their block (key skew statistic)
    bool plain;    // plain stores for the log copy (st_out)
};
struct ReadJob {
    const u64* keys;
    u64 R;
    u64* vals;
    uint8_t* found;
    u32 nblocks;
    u32 epoch;    // the reads see the state after round `epoch`
    bool use_rec; // that round's apply may run in the same launch: take its winners' records
    bool quiet;   // nothing in this launch writes the table (no stamp index, no apply): a key is
                  // present iff its probe chain holds it, and the stamps are not read
    RecSrc rec;
    // key-skew sample riding in this launch (skew_sample): the launch's last block moves the
    // duplicate counters to mapped host memory as {seq, dups}; seq 0 = none
    u64* s_acc;
    volatile u64* s_host;
    u64 s_seq;
    bool plain;  // plain stores for the responses (st_out)
};


// Block-wide exclusive prefix sum of one u32 per thread (NT threads); *total gets the sum.
template <int NT = TPB>
__device__ __forceinline__ u32 block_scan_excl(u32 v, u32* total) {
    __shared__ u32 s_w[NT / 64];
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
    for (int i = 0; i < NT / 64; i++) {
        pre += i < w ? s_w[i] : 0u;
        tot += s_w[i];
    }
    __syncthreads();
    if (total) *total = tot;
    return pre + inc - v;
}

// ---- role: partition(e) (partition rounds) -------------------------------------------------------
// The tile's Puts go to the bucket of their key's HOME slot (home >> bk_shift; the side key to
// bucket 0), grouped by bucket in log order inside a bucket: {key, value} entries (+ the round
// offset i when previous values are wanted) and a count word cnt[bucket][tile] = start << 16 | count.
// Tile = TPB * K1 Puts; wave w owns [w*64*K1, (w+1)*64*K1) of it, so (q, lane) order inside a wave
// is log order and waves follow each other. DEDUP drops a Put that a later Put of the same key in
// the tile overwrites (rounds without previous values). The table is not touched: the previous
// round's reads run beside this pass in the same launch, and hm_papply_kernel does the rest.
template <int K1>
struct PartLds {
    static constexpr int TILE = TPB * K1;
    static constexpr int HSZ = TILE / 2;  // lossy dedup entries (u64 key + u32 position)
    static constexpr int PROBES = 16;
    static unsigned bytes(bool dedup, u32 nb) {
        const unsigned rank = nb * 4 + 4 * nb * 2;
        return dedup && HSZ * 12 > (int)rank ? (unsigned)(HSZ * 12) : rank;
    }
};

template <int K1, bool DEDUP>
__device__ __forceinline__ void part_role(const IndexJob& j, u32 blk, u32 shift, char* lds) {
    constexpr int WT = 64 * K1;
    constexpr int TILE = PartLds<K1>::TILE;
    constexpr int HSZ = PartLds<K1>::HSZ;
    constexpr u32 NOH = 0xFFFFFFFFu;  // the key found no dedup entry: always emitted
    __shared__ u32 s_side;  // dedup of the side-slot key: largest tile position + 1
    __shared__ u32 s_dup;   // Puts whose key another Put of the tile already entered
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const u64 base = (u64)blk * TILE;
    const u32 nb = 1u << j.nb_log;
    u64* s_hk = (u64*)lds;               // [HSZ] dedup keys
    u32* s_hp = (u32*)(lds + HSZ * 8);   // [HSZ] largest tile position + 1 per key
    if (DEDUP) {
        for (int q = threadIdx.x; q < HSZ; q += TPB) {
            s_hk[q] = EMPTY_KEY;
            s_hp[q] = 0;
        }
        if (threadIdx.x == 0) s_side = s_dup = 0;
    }
    nrg_put rec[K1];
    u32 bkt[K1];
    bool valid[K1];
#pragma unroll
    for (int q = 0; q < K1; q++) {
        const u64 i = base + (u64)(w * WT + q * 64 + lane);
        valid[q] = i < j.n;
        rec[q] = valid[q] ? j.rec.at(i) : nrg_put{0, 0};
    }
#pragma unroll
    for (int q = 0; q < K1; q++) {
        const u64 i = base + (u64)(w * WT + q * 64 + lane);
        if (valid[q] && j.ring_out) st_rec(&j.ring_out[(j.rec.lo + i) & j.rec.mask], rec[q], j.plain);
        bkt[q] = rec[q].key == EMPTY_KEY ? 0u : (u32)(table_home(rec[q].key, shift) >> j.bk_shift);
    }
    bool emit[K1];
    if (DEDUP) {
        __syncthreads();  // hash initialised
        u32 hq[K1];
        u32 dup = 0;
#pragma unroll
        for (int q = 0; q < K1; q++) {
            if (!valid[q]) continue;
            const u32 pos1 = (u32)(w * WT + q * 64 + lane) + 1;
            if (rec[q].key == EMPTY_KEY) {
                atomicMax(&s_side, pos1);
                continue;
            }
            // Lossy: a key that finds no entry within PROBES steps is not deduplicated. That is
            // consistent for all Puts of a key (entries are never freed, so every Put of a key that
            // got one walks into it); hot keys, the ones that matter, get one early.
            u32 h = (u32)(((mix64(rec[q].key) >> 32) * (u64)HSZ) >> 32);
            hq[q] = NOH;
            for (int pr = 0; pr < PartLds<K1>::PROBES; pr++) {
                const u64 old = atomicCAS((unsigned long long*)&s_hk[h], (unsigned long long)EMPTY_KEY,
                                          (unsigned long long)rec[q].key);
                if (old == EMPTY_KEY || old == rec[q].key) {
                    dup += old == rec[q].key ? 1u : 0u;
                    hq[q] = h;
                    break;
                }
                h = h + 1 == (u32)HSZ ? 0u : h + 1;
            }
            if (hq[q] != NOH) atomicMax(&s_hp[h], pos1);
        }
        if (dup) atomicAdd(&s_dup, dup);
        __syncthreads();
        if (threadIdx.x == 0 && s_dup && j.dup_acc) atomicAdd(&j.dup_acc[blk % HM_DUP_SLOTS], (u64)s_dup);
#pragma unroll
        for (int q = 0; q < K1; q++) {
            const u32 pos1 = (u32)(w * WT + q * 64 + lane) + 1;
            emit[q] = valid[q] && (rec[q].key == EMPTY_KEY ? s_side == pos1 : hq[q] == NOH || s_hp[hq[q]] == pos1);
        }
        __syncthreads();  // the hash region is reused below
    } else {
#pragma unroll
        for (int q = 0; q < K1; q++) emit[q] = valid[q];
    }
    // ---- stable grouping by bucket: wave-private counts, then a prefix over waves ----
    u32* s_start = (u32*)lds;                       // [nb] bucket start in the tile
    uint16_t* s_wc = (uint16_t*)(lds + nb * 4);     // [4][nb] per-wave counts -> wave offsets
    for (u32 b = threadIdx.x; b < 4 * nb; b += TPB) s_wc[b] = 0;
    __syncthreads();
    u32 rnk[K1];
#pragma unroll
    for (int q = 0; q < K1; q++) {
        // one returning LDS add per Put on the wave's packed u16 count (lanes of one instruction
        // get their old values in lane order: synthetic.hip's rankings, nrg_test_lds_add_order)
        if (emit[q]) {
            const u32 ix = w * nb + bkt[q], sh = (ix & 1u) * 16u;
            rnk[q] = (atomicAdd((u32*)s_wc + (ix >> 1), 1u << sh) >> sh) & 0xFFFFu;
        }
    }
    __syncthreads();
    constexpr int PER = HM_BK_MAX / TPB;  // buckets per thread (contiguous ownership)
    u32 tot[PER], loc = 0;
#pragma unroll
    for (int r = 0; r < PER; r++) {
        const u32 b = threadIdx.x * PER + r;
        tot[r] = 0;
        if (b < nb) {
            u32 run = 0;
#pragma unroll
            for (int v = 0; v < 4; v++) {
                const u32 c = s_wc[v * nb + b];
                s_wc[v * nb + b] = (uint16_t)run;
                run += c;
            }
            tot[r] = run;
            loc += run;
        }
    }
    u32 off = block_scan_excl(loc, nullptr);
#pragma unroll
    for (int r = 0; r < PER; r++) {
        const u32 b = threadIdx.x * PER + r;
        if (b < nb) {
            j.cnt[(u64)blk * nb + b] = (off << 16) | tot[r];
            s_start[b] = off;
        }
        off += tot[r];
    }
    __syncthreads();
    u64x2* ent = j.ent + (u64)blk * TILE;
#pragma unroll
    for (int q = 0; q < K1; q++) {
        if (!emit[q]) continue;
        const u32 p = s_start[bkt[q]] + s_wc[w * nb + bkt[q]] + rnk[q];
        u64x2 e;
        e.x = rec[q].key;
        e.y = rec[q].val;
        ent[p] = e;  // (streamed: 75.4-75.8 -> 93.5-93.7 us per N = 8 round, profiles/r06/papply_nt.txt)
        if (j.eidx) j.eidx[(u64)blk * TILE + p] = (u32)(base + (u64)(w * WT + q * 64 + lane));
    }
}

// claim (or find) k's slot from its home slot; *fresh = this call inserted it; -1: table full
__device__ __forceinline__ long long claim_slot(Slot* table, u64 k, u64 s, u64 tmask, bool* fresh) {
    *fresh = false;
    for (u64 pr = 0; pr <= tmask; pr++) {
        const u64 key = ld_relaxed(&table[s].key);
        if (key == k) return (long long)s;
        if (key == EMPTY_KEY) {
            const u64 old = atomicCAS((unsigned long long*)&table[s].key, (unsigned long long)EMPTY_KEY,
                                      (unsigned long long)k);
            if (old == EMPTY_KEY) {
                *fresh = true;
                return (long long)s;
            }
            if (old == k) return (long long)s;
        }
        s = (s + 1) & tmask;
    }
    return -1;
}

// ---- stamp rounds: index(e) with claims and stamps, apply(e-1) ------------------------------------
struct StampJob {
    u64* dup_acc;  // [HM_DUP_SLOTS] Puts combined with another Put of their block (key skew)
    RecSrc rec;
    nrg_put* ring_out;
    u64 n;
    u32 nblocks;
    u32 epoch;
    u32* put_slot;  // [n] slot of each Put (SIDE_SLOT, FULL_SLOT)
    u32* win;       // [n] = epoch: the Put took its slot's stamp (it was the largest so far)
    u32* over;      // [n] = epoch: a later Put of the key took the stamp from it
    u64* created_acc;
    // diagnostic ablations of a round launch (NRG_KNOB_EXP >> 20; RESULTS WRONG, timing only):
    // 1 no stamp atomics, 2 no apply role, 4 no index role, 8 no read role
    u32 exp;
    bool plain;  // plain stores for the log copy (st_out)
};
struct ApplyJob {
    RecSrc rec;
    u64 n;
    const u32* put_slot;
    const u32* win;
    const u32* over;
    u32 epoch;
    u32 nblocks;
};
constexpr u32 SIDE_SLOT = 0xFFFFFFFEu;  // put_slot of the key EMPTY_KEY

template <int K1>
struct StampLds {
    static constexpr int TILE = TPB * K1;
    static constexpr int HT = 2 * TILE;  // LDS combine table (slot -> largest i+1)
    static constexpr unsigned BYTES = HT * 8;
};

// find k from its home slot s (first key loaded: key0), or claim an empty slot; a slot this
// call claims is marked in the other parity (stamp (e, 0)) so the concurrent reads of round
// e-1 see it as absent; -1: table full
__device__ __forceinline__ long long find_or_claim_marked(Slot* table, u64 k, u64 s, u64 tmask, u64 key0, u32 e,
                                                          u32* created) {
    u64 key = key0;
    for (u64 pr = 0; pr <= tmask; pr++) {
        if (key == k) return (long long)s;
        if (key == EMPTY_KEY) {
            const u64 old = atomicCAS((unsigned long long*)&table[s].key, (unsigned long long)EMPTY_KEY,
                                      (unsigned long long)k);
            if (old == EMPTY_KEY) {
                table[s].st[(e - 1) & 1] = stamp_make(e, 0);
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

template <int K1>
__device__ __forceinline__ void stamp_index_role(const StampJob& j, u32 blk, Slot* table, u32 shift, u64 tmask,
                                                 DevCtl* ctl, char* lds) {
    constexpr int TILE = StampLds<K1>::TILE;
    constexpr int HT = StampLds<K1>::HT;
    __shared__ u32 s_side, s_created, s_dup;
    u32* s_slot = (u32*)lds;        // [HT] slot ids, ~0u free
    u32* s_max = (u32*)lds + HT;    // [HT] largest i+1 per slot in this block
    for (int q = threadIdx.x; q < HT; q += TPB) {
        s_slot[q] = 0xFFFFFFFFu;
        s_max[q] = 0;
    }
    if (threadIdx.x == 0) s_side = s_created = s_dup = 0;
    const u32 e = j.epoch, par = e & 1;
    const u64 base = (u64)blk * TILE;
    nrg_put rec[K1];
    u64 home[K1], key0[K1];
    // every record load, then every first probe, in flight before waiting on any of them
#pragma unroll
    for (int q = 0; q < K1; q++) {
        const u64 i = base + (u64)q * TPB + threadIdx.x;
        rec[q] = i < j.n ? j.rec.at(i) : nrg_put{EMPTY_KEY, 0};
    }
#pragma unroll
    for (int q = 0; q < K1; q++) {
        const u64 i = base + (u64)q * TPB + threadIdx.x;
        if (i < j.n && j.ring_out) st_rec(&j.ring_out[(j.rec.lo + i) & j.rec.mask], rec[q], j.plain);
        home[q] = table_home(rec[q].key, shift);
        key0[q] = i < j.n && rec[q].key != EMPTY_KEY ? table[home[q]].key : EMPTY_KEY;
    }
    __syncthreads();  // LDS table initialised
    u32 created = 0, dup = 0;
#pragma unroll
    for (int q = 0; q < K1; q++) {
        const u64 i = base + (u64)q * TPB + threadIdx.x;
        if (i >= j.n) continue;
        const u64 k = rec[q].key;
        if (k == EMPTY_KEY) {  // the side-slot key
            if (ld_relaxed32(&ctl->sp_claim) == 0 && atomicCAS(&ctl->sp_claim, 0u, 1u) == 0u) {
                ctl->sp.st[(e - 1) & 1] = stamp_make(e, 0);
                created++;
            }
            atomicMax(&s_side, (u32)(i + 1));
            st_pol<NRG_HM_TAG_NT>(&j.put_slot[i], SIDE_SLOT);
            continue;
        }
        const long long s = find_or_claim_marked(table, k, home[q], tmask, key0[q], e, &created);
        if (s < 0) {
            atomicOr(&ctl->err, ERR_TABLE_FULL);
            st_pol<NRG_HM_TAG_NT>(&j.put_slot[i], FULL_SLOT);
            continue;
        }
        st_pol<NRG_HM_TAG_NT>(&j.put_slot[i], (u32)s);
        u32 h = (u32)(mix64((u64)s) & (HT - 1));
        for (;;) {
            const u32 old = atomicCAS(&s_slot[h], 0xFFFFFFFFu, (u32)s);
            if (old == 0xFFFFFFFFu || old == (u32)s) {
                dup += old == (u32)s ? 1u : 0u;
                break;
            }
            h = (h + 1) & (HT - 1);
        }
        atomicMax(&s_max[h], (u32)(i + 1));
    }
    if (created) atomicAdd(&s_created, created);
    if (dup) atomicAdd(&s_dup, dup);
    __syncthreads();
    // one stamp atomic per distinct slot of the block (a hot key costs one per block). Its old
    // value settles who stores: a Put that raised the stamp is the winner so far (win = e); if the
    // stamp was already this round's, the Put it took it from is overtaken (over = e). So apply
    // finds the last writer from two coalesced words per Put, not from a random read of the
    // slot's stamp (n8: 31 us of apply for 800k Puts).
    for (int q = threadIdx.x; q < HT; q += TPB) {
        const u32 sl = s_slot[q];
        if (sl != 0xFFFFFFFFu && !(j.exp & 1)) {
            const u64 mine = stamp_make(e, s_max[q]);
            const u64 old = atomicMax((unsigned long long*)&table[sl].st[par], (unsigned long long)mine);
            if (old < mine) {
                st_pol<NRG_HM_TAG_NT>(&j.win[s_max[q] - 1], e);
                if (stamp_epoch(old) == e && (u32)old) st_pol<NRG_HM_TAG_NT>(&j.over[(u32)old - 1], e);
            }
        }
    }
    if (threadIdx.x == 0) {
        if (s_side) atomicMax((unsigned long long*)&ctl->sp.st[par], (unsigned long long)stamp_make(e, s_side));
        if (s_created) atomicAdd(&j.created_acc[blk % HM_CREATED_SLOTS], (u64)s_created);
        if (s_dup && j.dup_acc) atomicAdd(&j.dup_acc[blk % HM_DUP_SLOTS], (u64)s_dup);
    }
}

// apply(e): per Put, the elected writer stores its value
__device__ __forceinline__ void apply_role(const ApplyJob& j, u32 blk, Slot* table, DevCtl* ctl) {
    const u64 i = (u64)blk * TPB + threadIdx.x;
    if (i >= j.n) return;
    const u32 par = j.epoch & 1;
    const u32 s = j.put_slot[i];
    const u64 want = stamp_make(j.epoch, i + 1);
    if (s == SIDE_SLOT) {
        if (ctl->sp.st[par] == want) ctl->sp.val = j.rec.at(i).val;
    } else if (s != FULL_SLOT) {
        // (a 16-B {key, val} store costs the same: a partial-line write is priced per line,
        // profiles/r03_apply_store_width.txt)
        if (j.win[i] == j.epoch && j.over[i] != j.epoch) st_pol<NRG_HM_APPLY_NT>(&table[s].val, j.rec.at(i).val);
    }
}

// ---- role: reads -------------------------------------------------------------------------------
// Present iff the stamp of the round's parity is nonzero with epoch <= ep (0: claim in flight;
// a later epoch: created by the concurrent round); epoch == ep: written by round ep, whose
// elected record holds the value while its apply may run in this launch.
__device__ __forceinline__ bool resolve(u64 val, u64 st, const ReadJob& j, u64* v) {
    const u32 se = stamp_epoch(st);
    if (st == 0 || se > j.epoch) return false;
    *v = (se == j.epoch && j.use_rec) ? j.rec.at((u32)st - 1).val : val;
    return true;
}

// RPT Gets per thread, q = blk * TPB * RPT + r * TPB + tid: every key load and every home-line
// load of the thread in flight together. Measured on one box (profiles/r03_read_rpt.txt), B1 per
// round: RPT 1 34.4 us, 2 36.2, 4 39.8; the N=8 per-GPU round 99.3 / 100.8 / 105.4 us.
constexpr int RPT = 1;

__device__ __forceinline__ void read_role(const ReadJob& j, u32 blk, const Slot* table, u32 shift, u64 tmask,
                                          const DevCtl* ctl) {
    const u32 par = j.epoch & 1;
    const u64 q0 = (u64)blk * TPB * RPT + threadIdx.x;
    u64 k[RPT], s[RPT];
    bool on[RPT];
#pragma unroll
    for (int r = 0; r < RPT; r++) {
        const u64 q = q0 + (u64)r * TPB;
        on[r] = q < j.R;
        k[r] = on[r] ? j.keys[q] : EMPTY_KEY;
    }
    // first probe of every key: {key, val} and the stamp, two loads of one line, all issued together
    u64x2 w[RPT];
    u64 st[RPT];
#pragma unroll
    for (int r = 0; r < RPT; r++) {
        s[r] = table_home(k[r], shift);
        const bool probe = on[r] && k[r] != EMPTY_KEY;
        w[r].x = EMPTY_KEY;
        w[r].y = 0;
        st[r] = 0;
        if (probe) {
            // (round 6: with the streaming hint on these two loads, 34.04-34.13 -> 44.25-44.36 us per
            // B1 round; profiles/r06/b1_apply_nt.txt)
            w[r] = *(const u64x2*)&table[s[r]];
            if (!j.quiet) st[r] = table[s[r]].st[par];
        }
    }
#pragma unroll
    for (int r = 0; r < RPT; r++) {
        if (!on[r]) continue;
        u64 v = 0;
        bool f = false;
        if (k[r] == EMPTY_KEY) {
            if (ctl->sp_claim) {
                if (j.quiet) {
                    f = true;
                    v = ctl->sp.val;
                } else {
                    f = resolve(ctl->sp.val, ctl->sp.st[par], j, &v);
                }
            }
        } else if (j.quiet) {
            u64 kk = w[r].x, vv = w[r].y, sl = s[r];
            for (u64 pr = 0; pr <= tmask; pr++) {
                if (kk == k[r]) {
                    f = true;
                    v = vv;
                    break;
                }
                if (kk == EMPTY_KEY) break;
                sl = (sl + 1) & tmask;
                const u64x2 x = *(const u64x2*)&table[sl];
                kk = x.x;
                vv = x.y;
            }
        } else {
            u64 kk = w[r].x, vv = w[r].y, stt = st[r], sl = s[r];
            asm volatile("" : "+v"(kk), "+v"(vv), "+v"(stt));
            for (u64 pr = 0; pr <= tmask; pr++) {
                if (kk == k[r]) {
                    f = resolve(vv, stt, j, &v);
                    break;
                }
                if (kk == EMPTY_KEY) break;
                sl = (sl + 1) & tmask;
                const u64x2 x = *(const u64x2*)&table[sl];
                stt = table[sl].st[par];
                kk = x.x;
                vv = x.y;
                asm volatile("" : "+v"(kk), "+v"(vv), "+v"(stt));
            }
        }
        if (!f) v = 0;
        const u64 q = q0 + (u64)r * TPB;
        st_out(&j.vals[q], v, j.plain);
        st_out(&j.found[q], (uint8_t)(f ? 1 : 0), j.plain);
    }
}

// index-role kinds of a round launch
constexpr int IX_STAMP = 2;       // stamp round
constexpr int IX_PART = 3;        // partition round, dedup (hm_papply_kernel<false> follows)
constexpr int IX_PART_ALL = 4;    // partition round, every Put kept (previous values)
constexpr int IX_PART_NODUP = 5;  // partition round, every Put kept, no previous values (uniform keys)

// One launch = {index(e)} + {apply(e-1)} + {reads(e-1)} over disjoint block ranges (any may be
// empty). Index blocks come first so the latency-bound pass starts first.
// <= 80 SGPRs: 256-thread blocks are admitted 8 per CU only up to 80 SGPRs (82-96: 7 per CU,
// MI355X_MICROARCH.md "Residency"), and the read role needs every resident wave.
// DIAG: the instantiation that honours the diagnostic ablation bits (NRG_KNOB_EXP); the release
// instantiations fold them away and are the only ones launched unless such a bit is set.
template <int K1, int IX, bool DIAG>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_num_sgpr(80))) void hm_round_kernel(IndexJob ij, StampJob sj,
                                                                                             ApplyJob aj, ReadJob rj,
                                                       Slot* table, u32 shift, u64 tmask, DevCtl* ctl) {
    extern __shared__ __attribute__((aligned(16))) char s_lds[];
    if constexpr (!DIAG) {
        ij.exp = 0;
        sj.exp = 0;
    }
    u32 b = blockIdx.x;
    if (rj.s_seq && b == gridDim.x - 1) {  // the tail block
        // the skew sample (counters read and cleared atomically)
        if (rj.s_seq && threadIdx.x < HM_DUP_SLOTS) {
            u64 v = atomicExch((unsigned long long*)&rj.s_acc[threadIdx.x], 0ull);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
            if (threadIdx.x == 0) {
                rj.s_host[1] = v;
                __threadfence_system();
                rj.s_host[0] = rj.s_seq;
            }
        }
        return;
    }
    const u32 nix = IX == IX_STAMP ? sj.nblocks : ij.nblocks;
    if (b < nix) {
        if (sj.exp & 4) return;
        if constexpr (IX == IX_STAMP) stamp_index_role<K1>(sj, b, table, shift, tmask, ctl, s_lds);
        else part_role<K1, IX == IX_PART>(ij, b, shift, s_lds);
        return;
    }
    b -= nix;
    if (b < aj.nblocks) {
        if (!(sj.exp & 2)) apply_role(aj, b, table, ctl);
        return;
    }
    b -= aj.nblocks;
    if (!(sj.exp & 8)) read_role(rj, b, table, shift, tmask, ctl);
}

// ---- hm_papply_kernel: partition rounds' table pass, one workgroup per bucket ---------------------
// The bucket's entries (every tile's run, tile order = log order) are taken in chunks of PA_C:
// an LDS hash finds each key's last entry in the chunk, whose thread finds the key's slot from
// its home (or claims an empty one: a new key) and stores the value -- one table line read and
// written per distinct key, no device atomics per Put. All Puts of a key share a bucket (the
// bucket is the home slot's), so one workgroup decides each key; a later chunk of the bucket
// overwrites an earlier one's store in log order. Claims of other buckets' workgroups only fill
// empty slots and cannot cut a present key's probe chain.
// PREV (HashMap::insert's previous values, nr/examples/hashmap.rs:46-50): every Put has an entry;
// the first entry of a key in the chunk finds (or claims) the slot and its value before the
// chunk; wave 0 then walks the chunk in log order, 64 entries a step: a Put's previous value is
// its predecessor's value, else the key's value before the chunk, else None.
struct PApplyJob {
    const u64x2* ent;  // [tiles][tile] {key, value}
    const u32* eidx;   // [tiles][tile] round offset (PREV)
    const u32* cnt;    // [tiles][bucket] start << 16 | count
    u32 ntiles, tile, nb;
    Slot* table;
    u32 shift;
    u64 tmask;
    DevCtl* ctl;
    u64* created_acc;
    u64 lo, resp_lo, resp_hi;
    u64* prev;
    uint8_t* prevf;
    u32 stall;  // NRG_KNOB_STALL (tests)
    u64* dbg;   // (NRG_KNOB_EXP bit 2, diagnostic) per bucket, 8 words: [0] start [1] counts scanned
                // [2] first chunk hashed [3] its slots resolved [4] its stores done [5] end [6] chunks
};

// T threads per workgroup (rounds without previous values: 256, 512 or 1024 over at most 1024,
// 512 or 256 buckets). Wider workgroups over wider buckets: a bucket's run in a tile holds more
// entries (a 128-B line at 1024 instead of ~32 B at 256) and there are fewer [tile][bucket] count
// words to gather, each a line.
template <bool PREV, int T>
struct PaGeo {
    static_assert(!PREV || T == 256, "previous values use 256-thread workgroups");
    static constexpr int TPB = T;
    static constexpr int C = PREV ? 512 : 4 * T;  // entries per chunk
    static constexpr int HT = 2 * C;              // LDS hash entries (load <= 1/2)
    static constexpr int PER = C / TPB;
    static constexpr u32 NB_LOG = T == 1024 ? 8 : T == 512 ? 9 : 10;  // at most this many buckets
};

__device__ __forceinline__ u32 pa_hash(u64 k, u32 ht) { return (u32)(mix64(k) >> 40) & (ht - 1); }

// Find or claim the slots of up to N keys of one thread together: every probe load, then every
// CAS on an empty slot, of all N keys is in flight before any is resolved (one or two memory
// round trips for most keys instead of one or two per key). on[r]: key r takes part (not the
// side key). Out: slot[r] (-1: table full), fresh[r] (this call claimed it: epoch-1 stamps
// written), val[r] = the slot's value before this call (found keys; WANT_VAL).
template <int N, bool WANT_VAL>
__device__ __forceinline__ void pa_resolve(Slot* table, u32 shift, u64 tmask, const u64* k, const bool* on,
                                           long long* slot, bool* fresh, u64* val) {
    u64 s[N], kk[N], vv[N];
    u32 st[N];  // 0 done, 1 key loaded, 2 CAS needed
#pragma unroll
    for (int r = 0; r < N; r++) {
        st[r] = on[r] ? 1u : 0u;
        s[r] = on[r] ? table_home(k[r], shift) : 0;
        slot[r] = -1;
        fresh[r] = false;
        kk[r] = EMPTY_KEY;
        vv[r] = 0;
        if (on[r]) {
            if (WANT_VAL) {
                const u64x2 x = *(const u64x2*)&table[s[r]];
                kk[r] = x.x;
                vv[r] = x.y;
            } else {
                kk[r] = ld_relaxed(&table[s[r]].key);
            }
        }
    }
    for (u64 pr = 0; pr <= tmask; pr++) {
        bool any = false;
#pragma unroll
        for (int r = 0; r < N; r++) {
            if (st[r] != 1) continue;
            if (kk[r] == k[r]) {
                slot[r] = (long long)s[r];
                if (WANT_VAL) val[r] = vv[r];
                st[r] = 0;
            } else if (kk[r] == EMPTY_KEY) {
                st[r] = 2;
            } else {
                s[r] = (s[r] + 1) & tmask;
                st[r] = 3;
            }
            any = any || st[r] != 0;
        }
        if (!any) return;
        u64 old[N];
#pragma unroll
        for (int r = 0; r < N; r++)
            if (st[r] == 2)
                old[r] = atomicCAS((unsigned long long*)&table[s[r]].key, (unsigned long long)EMPTY_KEY,
                                   (unsigned long long)k[r]);
#pragma unroll
        for (int r = 0; r < N; r++) {
            if (st[r] != 2) continue;
            if (old[r] == EMPTY_KEY) {  // claimed: a new key, present for every later read
                u64x2 z;
                z.x = z.y = STAMP_PRESENT;
                *(u64x2*)&table[s[r]].st[0] = z;
                slot[r] = (long long)s[r];
                fresh[r] = true;
                st[r] = 0;
            } else if (old[r] == k[r]) {
                slot[r] = (long long)s[r];
                if (WANT_VAL) val[r] = ld_relaxed(&table[s[r]].val);
                st[r] = 0;
            } else {
                s[r] = (s[r] + 1) & tmask;
                st[r] = 3;
            }
        }
#pragma unroll
        for (int r = 0; r < N; r++) {
            if (st[r] != 3) continue;
            if (WANT_VAL) {
                const u64x2 x = *(const u64x2*)&table[s[r]];
                kk[r] = x.x;
                vv[r] = x.y;
            } else {
                kk[r] = ld_relaxed(&table[s[r]].key);
            }
            st[r] = 1;
        }
    }
}

// NT: the table values are stored streamed (round 6; rounds of <= PA_NT_MAX Puts, see the launch)
template <bool PREV, int T, bool NT = false>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(PREV ? 3 : 4))) void hm_papply_kernel(PApplyJob j) {
    using G = PaGeo<PREV, T>;
    constexpr int PA_TPB = G::TPB, C = G::C, HT = G::HT, PER = G::PER;
    constexpr u32 NOFIRST = 0xFFFFFFFFu;
    extern __shared__ u32 s_dyn[];  // s_pre[ntiles + 1] entry prefix, s_off[ntiles] (u16)
    __shared__ u64 s_hk[HT];
    __shared__ u32 s_hp[HT + 1];   // last chunk position + 1 of the key; [HT]: the side key
    __shared__ uint16_t s_tile[2][C];        // entry tile maps of this chunk and the next
    __shared__ u32 s_h1[PREV ? HT + 1 : 1];  // PREV: first chunk position + 1
    __shared__ u32 s_hs[PREV ? HT + 1 : 1];  // PREV: the key's slot (SIDE_ID, FULL_SLOT)
    __shared__ u64 s_lv[PREV ? HT + 1 : 1];  // PREV: the key's value so far in the walk
    __shared__ u32 s_hf[PREV ? HT + 1 : 1];  // PREV: s_lv holds a value
    __shared__ u64 s_mk[PREV ? HT + 1 : 1];  // PREV: lanes of the current walk step per key
    __shared__ u64 s_ev[PREV ? C : 1];       // PREV: the chunk's values, hash entries, round offsets
    __shared__ uint16_t s_eh[PREV ? C : 1];
    __shared__ u32 s_ei[PREV ? C : 1];
    __shared__ u32 s_created;
    // Workgroups are dealt to the 8 XCDs round-robin; bucket b goes to workgroup 8 (b % per) + b / per
    // (per = nb / 8), so each XCD takes a contiguous range of buckets. Neighbouring buckets' entry
    // runs and count words share lines, and those lines are then fetched into one XCD's L2
    // instead of several.
    const u32 per = j.nb >> 3;
    const u32 nt = j.ntiles, b = j.nb >= 64 ? (blockIdx.x & 7u) * per + (blockIdx.x >> 3) : blockIdx.x;
#define PA_MARK(K, V) \
    if (j.dbg && threadIdx.x == 0) j.dbg[(u64)b * 8 + (K)] = (V)
    PA_MARK(0, wall_clock64());
    u32* s_pre = s_dyn;
    uint16_t* s_off = (uint16_t*)(s_dyn + nt + 1);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // this bucket's (offset, count) in every tile; thread owns tiles [tid*K, tid*K + K)
    const u32 K = (nt + PA_TPB - 1) / PA_TPB;
    u32 loc = 0;
    for (u32 q = 0; q < K; q++) {
        const u32 t = threadIdx.x * K + q;
        if (t < nt) {
            const u32 v = j.cnt[(u64)t * j.nb + b];
            s_off[t] = (uint16_t)(v >> 16);
            s_pre[t] = v & 0xFFFFu;
            loc += v & 0xFFFFu;
        }
    }
    for (int h = threadIdx.x; h <= HT; h += PA_TPB) {
        if (h < HT) s_hk[h] = EMPTY_KEY;
        s_hp[h] = 0;
        if (PREV) {
            s_h1[h] = NOFIRST;
            s_mk[h] = 0;
        }
    }
    u32 total;
    u32 run = block_scan_excl<PA_TPB>(loc, &total);  // (its barriers also order the initialisation above)
    for (u32 q = 0; q < K; q++) {
        const u32 t = threadIdx.x * K + q;
        if (t < nt) {
            const u32 c = s_pre[t];
            s_pre[t] = run;
            run += c;
        }
    }
    if (threadIdx.x == 0) {
        s_pre[nt] = total;
        s_created = 0;
    }
    __syncthreads();
    PA_MARK(1, wall_clock64());
    PA_MARK(6, (total + C - 1) / C);
    u32 created = 0;
    // entry tile map of the chunk at `base`
    auto map_chunk = [&](u32 base, uint16_t* map) {
        const u32 cn = total - base < (u32)C ? total - base : (u32)C;
        for (u32 q = 0; q < K; q++) {
            const u32 t = threadIdx.x * K + q;
            if (t >= nt) break;
            const u32 lo_ = s_pre[t] > base ? s_pre[t] : base;
            const u32 hi_ = s_pre[t + 1] < base + cn ? s_pre[t + 1] : base + cn;
            for (u32 i = lo_; i < hi_; i++) map[i - base] = (uint16_t)t;
        }
    };
    // this thread's entries of the chunk at `base` (issued; used a chunk later)
    u64x2 xn[PER];
    u32 in_[PER];
    auto load_chunk = [&](u32 base, const uint16_t* map) {
        const u32 cn = total - base < (u32)C ? total - base : (u32)C;
#pragma unroll
        for (int r = 0; r < PER; r++) {
            const u32 p = r * PA_TPB + threadIdx.x;
            xn[r].x = EMPTY_KEY;
            xn[r].y = 0;
            in_[r] = 0;
            if (p < cn) {
                const u32 t = map[p];
                const u64 e = (u64)t * j.tile + s_off[t] + (base + p - s_pre[t]);
                xn[r] = j.ent[e];
                if (PREV) in_[r] = j.eidx[e];
            }
        }
    };
    if (total) {
        map_chunk(0, s_tile[0]);
        __syncthreads();
        test_stall(j.stall & 1, w);  // (tests) slow waves read the map while the next is built
        load_chunk(0, s_tile[0]);
    }
    // Software pipelined: the next chunk's entries are in flight while this chunk resolves.
    for (u32 base = 0, pb = 0; base < total; base += C, pb ^= 1) {
        const u32 cn = total - base < (u32)C ? total - base : (u32)C;
        u64x2 x[PER];
        u32 ix[PER], hh[PER];
#pragma unroll
        for (int r = 0; r < PER; r++) {
            x[r] = xn[r];
            ix[r] = in_[r];
        }
        const u32 nbase = base + C;
        if (nbase < total) map_chunk(nbase, s_tile[pb ^ 1]);  // (published by the barrier below)
        // one hash entry per key: its last (and first) position in the chunk
#pragma unroll
        for (int r = 0; r < PER; r++) {
            const u32 p = r * PA_TPB + threadIdx.x;
            hh[r] = HT;
            if (p >= cn) continue;
            const u64 k = x[r].x;
            u32 h = HT;
            if (k != EMPTY_KEY) {
                h = pa_hash(k, HT);
                for (;;) {  // at most C keys in 2C entries: an entry is always found
                    const u64 old = atomicCAS((unsigned long long*)&s_hk[h], (unsigned long long)EMPTY_KEY,
                                              (unsigned long long)k);
                    if (old == EMPTY_KEY || old == k) break;
                    h = (h + 1) & (HT - 1);
                }
            }
            hh[r] = h;
            atomicMax(&s_hp[h], p + 1);
            if (PREV) {
                atomicMin(&s_h1[h], p + 1);
                s_ev[p] = x[r].y;
                s_eh[p] = (uint16_t)h;
                s_ei[p] = ix[r];
            }
        }
        __syncthreads();
        if (base == 0) PA_MARK(2, wall_clock64());
        if (nbase < total) {
            test_stall(j.stall & 1, w);  // (tests) slow waves read the next map after the others moved on
            load_chunk(nbase, s_tile[pb ^ 1]);
        }
        if (!PREV) {
            // the key's last entry finds or claims its slot and stores its value
            bool dec[PER], on[PER], fr[PER];
            u64 kx[PER], vx[PER];
            long long sl[PER];
#pragma unroll
            for (int r = 0; r < PER; r++) {
                const u32 p = r * PA_TPB + threadIdx.x;
                dec[r] = p < cn && s_hp[hh[r]] == p + 1;
                on[r] = dec[r] && x[r].x != EMPTY_KEY;
                kx[r] = x[r].x;
            }
            pa_resolve<PER, false>(j.table, j.shift, j.tmask, kx, on, sl, fr, vx);
            if (base == 0) PA_MARK(3, wall_clock64());
#pragma unroll
            for (int r = 0; r < PER; r++) {
                if (!dec[r]) continue;
                if (x[r].x == EMPTY_KEY) {
                    if (!j.ctl->sp_claim) {
                        j.ctl->sp_claim = 1;
                        j.ctl->sp.st[0] = j.ctl->sp.st[1] = STAMP_PRESENT;
                        created++;
                    }
                    j.ctl->sp.val = x[r].y;
                } else if (sl[r] < 0) {
                    atomicOr(&j.ctl->err, ERR_TABLE_FULL);
                } else {
                    st_pol<NT>(&j.table[sl[r]].val, x[r].y);
                    created += fr[r];
                }
            }
            __syncthreads();  // every decider has read s_hp
#pragma unroll
            for (int r = 0; r < PER; r++) {  // the deciders free their keys' entries for the next chunk
                if (!dec[r]) continue;
                if (hh[r] < (u32)HT) s_hk[hh[r]] = EMPTY_KEY;
                s_hp[hh[r]] = 0;
            }
        } else {
            // the key's first entry: its slot and its value before the chunk
            bool fst[PER], on[PER], fr[PER];
            u64 kx[PER], vx[PER];
            long long sl[PER];
#pragma unroll
            for (int r = 0; r < PER; r++) {
                const u32 p = r * PA_TPB + threadIdx.x;
                fst[r] = p < cn && s_h1[hh[r]] == p + 1;
                on[r] = fst[r] && x[r].x != EMPTY_KEY;
                kx[r] = x[r].x;
                vx[r] = 0;
            }
            pa_resolve<PER, true>(j.table, j.shift, j.tmask, kx, on, sl, fr, vx);
#pragma unroll
            for (int r = 0; r < PER; r++) {
                if (!fst[r]) continue;
                const u32 h = hh[r];
                if (x[r].x == EMPTY_KEY) {
                    s_hs[h] = SIDE_ID;
                    if (j.ctl->sp_claim) {
                        s_lv[h] = j.ctl->sp.val;
                        s_hf[h] = 1;
                    } else {
                        j.ctl->sp_claim = 1;
                        j.ctl->sp.st[0] = j.ctl->sp.st[1] = STAMP_PRESENT;
                        created++;
                        s_hf[h] = 0;
                    }
                } else if (sl[r] < 0) {
                    atomicOr(&j.ctl->err, ERR_TABLE_FULL);
                    s_hs[h] = FULL_SLOT;
                    s_hf[h] = 0;
                } else {
                    s_hs[h] = (u32)sl[r];
                    created += fr[r];
                    s_hf[h] = fr[r] ? 0u : 1u;
                    s_lv[h] = vx[r];
                }
            }
            __syncthreads();
            // wave 0 walks the chunk in log order, 64 entries a step
            if (w == 0) {
                for (u32 s0 = 0; s0 < cn; s0 += 64) {
                    const u32 p = s0 + lane;
                    const bool v = p < cn;
                    const u32 h = v ? s_eh[p] : 0u;
                    const u64 val = v ? s_ev[p] : 0ull;
                    if (v) atomicOr((unsigned long long*)&s_mk[h], 1ull << lane);
                    const u64 m = v ? s_mk[h] : 0ull;
                    const u64 lower = m & ((1ull << lane) - 1);
                    const int pl = lower ? 63 - __clzll((long long)lower) : lane;
                    const u64 pv_lane = __shfl(val, pl, 64);
                    if (v) {
                        u64 pv;
                        uint8_t pf;
                        if (lower) {
                            pv = pv_lane;
                            pf = 1;
                        } else {
                            pf = s_hf[h] ? 1 : 0;
                            pv = pf ? s_lv[h] : 0;
                        }
                        const u64 g = j.lo + s_ei[p];
                        if (g >= j.resp_lo && g < j.resp_hi) {
                            j.prev[g - j.resp_lo] = pv;
                            j.prevf[g - j.resp_lo] = pf;
                        }
                        if ((m >> lane) == 1ull) {  // the key's last entry in this step
                            s_lv[h] = val;
                            s_hf[h] = 1;
                            s_mk[h] = 0;
                        }
                    }
                }
            }
            __syncthreads();
            // the key's last entry stores its final value
#pragma unroll
            for (int r = 0; r < PER; r++) {
                const u32 p = r * PA_TPB + threadIdx.x;
                if (p >= cn || s_hp[hh[r]] != p + 1) continue;
                const u32 h = hh[r];
                const u32 sl = s_hs[h];
                if (sl == SIDE_ID) j.ctl->sp.val = s_lv[h];
                else if (sl != FULL_SLOT) j.table[sl].val = s_lv[h];  // (streamed, with the answers: slower, profiles/r06/papply_nt.txt)
                if (h < HT) s_hk[h] = EMPTY_KEY;
                s_hp[h] = 0;
                s_h1[h] = NOFIRST;
            }
        }
        __syncthreads();  // hash entries free; the next iteration builds the map after next in s_tile[pb]
        if (base == 0) PA_MARK(4, wall_clock64());
    }
    if (created) atomicAdd(&s_created, created);
    __syncthreads();
    if (threadIdx.x == 0 && s_created) atomicAdd(&j.created_acc[b % HM_CREATED_SLOTS], (u64)s_created);
    PA_MARK(5, wall_clock64());
#undef PA_MARK
}

// ---- small rounds: one workgroup, one launch (the flat combiner's batches) ----------------------
// A round of at most SM_W Puts and SM_R Gets, whole in one 1024-thread workgroup: the Puts are
// hashed by key in LDS (how many, the last one); one thread per distinct key finds or claims
// its slot, answers the previous values of the key's Puts in log order (the slot's value before
// the round for the first; nr/examples/hashmap.rs:46-50) and stores the last value. No deferred
// half and no device atomics per Put: round 2's index + elector + reads launches for the
// combiner's batches (about 20 us of GPU time for a few hundred ops) became one.
// The Gets do not wait for the Puts: a Get of a key the round Puts is answered from the LDS hash
// (the key's last value), and for any other key the round changes nothing the Get reads -- a
// present key's probe chain holds no empty slot, so claims (which fill empty slots) cannot
// change where its chain ends, and only Put keys' values are stored. So every Get's table probe
// is issued with the Put records, and resolves while the Puts claim and store.
// Runs with no other round in flight (the caller flushes first). Keys present in the table are
// present (quiescent: no claim in flight); fresh claims get epoch-1 stamps, as the partition
// apply's.
constexpr int SM_TPB = 1024;
constexpr u32 SM_W = 2048, SM_R = 8192, SM_HT = 4096;  // SM_HT: LDS hash entries (+1: the side key)
struct SmallJob {
    RecSrc rec;
    nrg_put* ring_out;  // log copy to write (nullptr: the records are in the ring)
    u32 n;
    u64 lo, resp_lo, resp_hi;
    u64* prev;
    uint8_t* prevf;
    const u64* keys;  // Gets
    u32 R;
    u64* vals;
    uint8_t* found;
    u32* e_out;  // the replica's error latch after the round (the combiner's batch), or nullptr
    u64* created_acc;
};

__device__ __forceinline__ u32 sm_hash(u64 k) { return (u32)(mix64(k) >> 40) & (SM_HT - 1); }

struct SmallLds {
    u64 val[SM_W];
    uint16_t ent[SM_W];    // hash entry of each Put
    u64 hk[SM_HT];
    u32 cnt[SM_HT + 1];    // Puts of the key; [SM_HT]: the side key
    u32 last[SM_HT + 1];   // its last Put + 1
    u32 created;
};

// a word for the host, stored write-through (system scope: the line leaves the L2), so the host
// sees it now and not at the next L2 writeback (the resident server has no kernel end to flush it)
__device__ __forceinline__ void host_put(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// RQ Gets per thread (RQ * SM_TPB <= SM_R per round); FLUSH: the responses and the error word are
// made visible to the host at once (the resident server's rounds)
template <int RQ, bool FLUSH>
__device__ __forceinline__ void small_body(const SmallJob& j, Slot* table, u32 shift, u64 tmask, DevCtl* ctl,
                                           SmallLds& L) {
    u64* s_val = L.val;
    uint16_t* s_ent = L.ent;
    u64* s_hk = L.hk;
    u32* s_cnt = L.cnt;
    u32* s_last = L.last;
    u32& s_created = L.created;
    const int tid = threadIdx.x;
    constexpr int WQ = (int)(SM_W / SM_TPB);
    // every Put record, every Get key and every Get's first probe in flight together
    nrg_put r[WQ];
#pragma unroll
    for (int q = 0; q < WQ; q++) {
        const u32 i = q * SM_TPB + tid;
        r[q] = i < j.n ? j.rec.at(i) : nrg_put{EMPTY_KEY, 0};
    }
    u64 k[RQ], s[RQ];
    u64x2 w[RQ];
#pragma unroll
    for (int q = 0; q < RQ; q++) {
        const u32 i = q * SM_TPB + tid;
        k[q] = i < j.R ? j.keys[i] : EMPTY_KEY;
    }
#pragma unroll
    for (int q = 0; q < RQ; q++) {
        const u32 i = q * SM_TPB + tid;
        s[q] = table_home(k[q], shift);
        w[q].x = EMPTY_KEY;
        w[q].y = 0;
        if (i < j.R && k[q] != EMPTY_KEY) w[q] = *(const u64x2*)&table[s[q]];
    }
    for (int h = tid; h <= (int)SM_HT; h += SM_TPB) {
        if (h < (int)SM_HT) s_hk[h] = EMPTY_KEY;
        s_cnt[h] = 0;
        s_last[h] = 0;
    }
    if (tid == 0) s_created = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < WQ; q++) {
        const u32 i = q * SM_TPB + tid;
        if (i >= j.n) continue;
        if (j.ring_out) j.ring_out[(j.rec.lo + i) & j.rec.mask] = r[q];
        s_val[i] = r[q].val;
        const u64 kk = r[q].key;
        u32 h = SM_HT;
        if (kk != EMPTY_KEY) {
            h = sm_hash(kk);
            for (;;) {  // at most SM_W keys in SM_HT entries: an entry is always found
                const u64 old = atomicCAS((unsigned long long*)&s_hk[h], (unsigned long long)EMPTY_KEY,
                                          (unsigned long long)kk);
                if (old == EMPTY_KEY || old == kk) break;
                h = (h + 1) & (SM_HT - 1);
            }
        }
        s_ent[i] = (uint16_t)h;
        atomicAdd(&s_cnt[h], 1u);
        atomicMax(&s_last[h], i + 1);
    }
    __syncthreads();
    // one thread per distinct key: its slot, its Puts' previous values, its last value
    u32 created = 0;
    for (int h = tid; h <= (int)SM_HT; h += SM_TPB) {
        const u32 c = s_cnt[h];
        if (!c) continue;
        u64 cur = 0;
        bool has = false;
        Slot* slot = nullptr;
        if (h == (int)SM_HT) {  // the key EMPTY_KEY lives in the side slot
            has = ctl->sp_claim != 0;
            if (has) {
                cur = ctl->sp.val;
            } else {
                ctl->sp_claim = 1;
                ctl->sp.st[0] = ctl->sp.st[1] = STAMP_PRESENT;
                created++;
            }
        } else {
            bool fresh = false;
            const u64 kk = s_hk[h];
            const long long sl = claim_slot(table, kk, table_home(kk, shift), tmask, &fresh);
            if (sl < 0) {
                atomicOr(&ctl->err, ERR_TABLE_FULL);
                s_cnt[h] = 0;  // the Gets of this key find it absent, as the other paths leave it
                continue;
            }
            slot = &table[sl];
            if (fresh) {
                slot->st[0] = slot->st[1] = STAMP_PRESENT;
                created++;
            } else {
                cur = slot->val;
                has = true;
            }
        }
        const u32 last = s_last[h] - 1;
        if (c == 1) {  // the common case: one Put of the key in the round
            const u64 g = j.lo + last;
            if (j.prev && g >= j.resp_lo && g < j.resp_hi) {
                j.prev[g - j.resp_lo] = has ? cur : 0;
                j.prevf[g - j.resp_lo] = has ? 1 : 0;
            }
            cur = s_val[last];
        } else {  // the key's Puts in log order (a scan of the round; rare for uniform keys)
            for (u32 i = 0, seen = 0; seen < c; i++) {
                if (s_ent[i] != (uint16_t)h) continue;
                seen++;
                const u64 g = j.lo + i;
                if (j.prev && g >= j.resp_lo && g < j.resp_hi) {
                    j.prev[g - j.resp_lo] = has ? cur : 0;
                    j.prevf[g - j.resp_lo] = has ? 1 : 0;
                }
                cur = s_val[i];
                has = true;
            }
        }
        if (slot) slot->val = cur;
        else ctl->sp.val = cur;
    }
    if (created) atomicAdd(&s_created, created);
    // Gets: keys of the round's Puts from the LDS hash (read only after the barrier: a full
    // table zeroes the key's count above), every other key from its probe chain
    const u64 sp_val = ctl->sp.val;
    const bool sp_has = ctl->sp_claim != 0;
    __syncthreads();
    if (tid == 0 && s_created) atomicAdd(&j.created_acc[0], (u64)s_created);
#pragma unroll
    for (int q = 0; q < RQ; q++) {
        const u32 i = q * SM_TPB + tid;
        if (i >= j.R) continue;
        u64 v = 0;
        bool f = false;
        u32 h = SM_HT;
        if (k[q] != EMPTY_KEY) {
            h = sm_hash(k[q]);
            while (s_hk[h] != k[q] && s_hk[h] != EMPTY_KEY) h = (h + 1) & (SM_HT - 1);
            if (s_hk[h] != k[q]) h = SM_HT + 1;  // not a key of the round's Puts
        }
        if (h <= SM_HT && s_cnt[h]) {
            f = true;
            v = s_val[s_last[h] - 1];
        } else if (k[q] == EMPTY_KEY) {
            f = sp_has;
            v = f ? sp_val : 0;
        } else {
            u64 kk = w[q].x, vv = w[q].y, sl = s[q];
            for (u64 pr = 0; pr <= tmask; pr++) {
                if (kk == k[q]) {
                    f = true;
                    v = vv;
                    break;
                }
                if (kk == EMPTY_KEY) break;
                sl = (sl + 1) & tmask;
                const u64x2 x = *(const u64x2*)&table[sl];
                kk = x.x;
                vv = x.y;
            }
        }
        j.vals[i] = v;
        j.found[i] = f ? 1 : 0;
    }
    if (j.e_out) {  // the round's last write: the host (nrg_combiner) polls it as the round's completion
        // every wave's response stores issued before the barrier (the barrier alone does not wait
        // for them), then one lane's system release and the word (MI355X_MICROARCH.md, producer form)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            const u32 e = atomicExch(&ctl->err, 0u);
            if constexpr (FLUSH) {
                // the responses (plain stores, every wave waited for them above) written back
                // from the L2 by one system release, then the word itself write-through: the
                // resident server has no kernel end to write its L2 back (write-through stores
                // of every response, bytes included, measured slower: 18.8 vs 15.2 us a round)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                __hip_atomic_store(j.e_out, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                __threadfence_system();
                *(volatile u32*)j.e_out = e;
            }
        }
    }
}

__global__ __launch_bounds__(SM_TPB) void hm_small_round_kernel(SmallJob j, Slot* table, u32 shift, u64 tmask,
                                                                DevCtl* ctl) {
    __shared__ SmallLds L;
    small_body<(int)(SM_R / SM_TPB), false>(j, table, shift, tmask, ctl, L);
}

// ---- the combiner's round server: small rounds without a launch per round -----------------------
// One resident workgroup serves the flat combiner's hashmap batches (nrg_combiner) from mapped
// host memory. It reads every batch slot's fixed job fields (its buffers) once, then per round k
// polls slot k's doorbell, `(k + 1) << 32 | Puts << 16 | Gets`, runs the round as
// hm_small_round_kernel would (its log position tracked here: each round starts where the last
// ended) and ends it with the batch's error word, as there, and `served`. The host's launch and the
// dispatch from an idle queue leave the round's critical path. It exits when the host asks
// (`stop`, every rung round served) or after idle_ticks of the 100-MHz wall clock without a round,
// and then writes its session number to `exited`: every wave reaches that exit, so a host that
// stops posting (or dies) never leaves it running. A host that finds `exited` at its session with
// rounds still unserved relaunches from `served` (the old server never reads a doorbell again).
static_assert(sizeof(SmallJob) <= sizeof(SmallJobBlob), "a server slot holds one SmallJob");
static_assert(SERVE_R <= SM_R && SERVE_R % SM_TPB == 0, "server rounds are small rounds");
__device__ __forceinline__ u64 sgpr64(u64 v) {
    // (readfirstlane returns int: through u32, or a set bit 31 sign-extends over the high word)
    return ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(v >> 32)) << 32) |
           (u64)(u32)__builtin_amdgcn_readfirstlane((u32)v);
}
__global__ __launch_bounds__(SM_TPB) void hm_serve_kernel(ServeCtl* sc, const SmallJobBlob* hdr, u32 nslots, u64 first,
                                                          u64 first_lo, u64 session, u64 idle_ticks, Slot* table,
                                                          u32 shift, u64 tmask, DevCtl* ctl) {
    __shared__ SmallLds L;
    __shared__ SmallJob s_job[SERVE_SLOTS];  // the slots' fixed job fields, read once
    __shared__ int s_cmd;
    __shared__ u32 s_n, s_r;
    __shared__ u64 s_k, s_lo;  // (in LDS: nothing of the loop stays live in registers across a round)
    constexpr u32 JW = (u32)(sizeof(SmallJob) / 8);
    static_assert(sizeof(SmallJob) % 8 == 0, "job copied in words");
    for (u32 t = threadIdx.x; t < nslots * JW; t += SM_TPB)
        ((u64*)s_job)[t] = __hip_atomic_load((const u64*)hdr[t / JW].b + t % JW, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
    if (threadIdx.x == 0) {
        s_k = first;
        s_lo = first_lo;
    }
    __syncthreads();
    // wave 0 polls the round's doorbell, as a whole wave in uniform control flow (readfirstlane'd
    // values, scalar branches): a loop run by lane 0 alone under an exec mask never saw the host's
    // next post (microbench/serve_mech.hip)
    const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (;;) {
        if (wave == 0) {
            const u64 k = sgpr64(s_k);
            const u64* door = &sc->door[k % nslots];
            const u64 t0 = wall_clock64();
            u64 d = 0;
            int cmd = 0;
            for (u64 polls = 0;; polls++) {
                d = sgpr64(__hip_atomic_load(door, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
                if ((polls & 4095) == 0 && threadIdx.x == 0) {  // (diagnostic trace, Combiner.probe)
                    host_put(&sc->trace[1], k);
                    host_put(&sc->trace[2], d >> 32);
                    host_put(&sc->trace[3], polls);
                }
                if ((d >> 32) == k + 1) {
                    cmd = 1;
                    break;
                }
                if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&sc->stop, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM))) {
                    // the host rings every doorbell before it asks to stop: look once more
                    d = sgpr64(__hip_atomic_load(door, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
                    cmd = (d >> 32) == k + 1 ? 1 : 0;
                    break;
                }
                if (wall_clock64() - t0 > idle_ticks) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (threadIdx.x == 0) {
                s_cmd = cmd;
                s_n = (u32)(d >> 16) & 0xFFFFu;
                s_r = (u32)d & 0xFFFFu;
            }
        }
        __syncthreads();  // (also: every wave is done with the previous round's LDS)
        if (!s_cmd) break;
        // the round's job: the slot's fixed fields, the round's counts, its log position
        const SmallJob& h = s_job[s_k % nslots];
        const u64 lo = sgpr64(s_lo);
        const u32 n = (u32)__builtin_amdgcn_readfirstlane(s_n), R = (u32)__builtin_amdgcn_readfirstlane(s_r);
        SmallJob j;
        j.rec.src = (const nrg_put*)sgpr64((u64)h.rec.src);
        j.rec.ring = (const nrg_put*)sgpr64((u64)h.rec.ring);
        j.rec.mask = sgpr64(h.rec.mask);
        j.rec.lo = lo;
        j.ring_out = (nrg_put*)sgpr64((u64)h.ring_out);
        j.n = n;
        j.lo = lo;
        j.resp_lo = lo;
        j.resp_hi = lo + n;
        j.prev = n ? (u64*)sgpr64((u64)h.prev) : nullptr;
        j.prevf = n ? (uint8_t*)sgpr64((u64)h.prevf) : nullptr;
        j.keys = R ? (const u64*)sgpr64((u64)h.keys) : nullptr;
        j.R = R;
        j.vals = (u64*)sgpr64((u64)h.vals);
        j.found = (uint8_t*)sgpr64((u64)h.found);
        j.e_out = (u32*)sgpr64((u64)h.e_out);
        j.created_acc = (u64*)sgpr64((u64)h.created_acc);
        small_body<(int)(SERVE_R / SM_TPB), true>(j, table, shift, tmask, ctl, L);  // ends with the error word
        if (threadIdx.x == 0) {
            s_k = s_k + 1;
            s_lo = s_lo + n;
            host_put(&sc->served, s_k);
        }
    }
    if (threadIdx.x == 0) {
        __threadfence_system();
        host_put(&sc->exited, session);
    }
}

static RecSrc ring_src(nrg_ctx* c, const nrg_put* src, u64 lo);

// A round through hm_small_round_kernel (hm_replay_chunk decides; n <= SM_W, R <= SM_R).
static hipError_t small_round(nrg_ctx* c, const nrg_put* src, u64 lo, u64 n, bool write_ring, const u64* keys, u64 R,
                              u64* vals, uint8_t* found, u64 resp_lo, u64 resp_hi, u64* prev, uint8_t* prevf) {
    hipError_t e = hm_flush(c);
    if (e != hipSuccess) return e;
    SmallJob j;
    j.rec = ring_src(c, src, lo);
    j.ring_out = write_ring ? (nrg_put*)c->d_ring : nullptr;
    j.n = (u32)n;
    j.lo = lo;
    j.resp_lo = resp_lo;
    j.resp_hi = resp_hi;
    j.prev = prev;
    j.prevf = prev ? prevf : nullptr;
    j.keys = keys;
    j.R = keys ? (u32)R : 0u;
    j.vals = vals;
    j.found = found;
    j.e_out = c->err_out;
    c->err_out = nullptr;
    j.created_acc = c->d_created;
    NRG_LAUNCH(c, "hm_small", hm_small_round_kernel, 1, SM_TPB, 0, c->stream, j, c->d_table, c->slot_shift,
               (u64)(c->slots - 1), c->d_ctl);
    return hipGetLastError();
}

// The job of a small round of records [lo, lo + W) (hm_small_round_kernel's, as small_round would
// launch it with the log copy written) into `blob`, for hm_serve_kernel; runtime.cpp hm_small_job
// does the replica's log bookkeeping around it.
bool hm_small_fill(nrg_ctx* c, const nrg_put* recs, u64 lo, u64 W, const u64* keys, u64 R, u64* vals, uint8_t* found,
                   u64* prev, uint8_t* prevf, u32* e_out, SmallJobBlob* blob) {
    if (W > SM_W || R > SERVE_R || c->pend.valid) return false;
    if (!blob) return true;  // (the server's slots hold the fixed fields; only the checks)
    SmallJob j;
    j.rec = ring_src(c, recs, lo);
    j.ring_out = (nrg_put*)c->d_ring;
    j.n = (u32)W;
    j.lo = lo;
    j.resp_lo = lo;
    j.resp_hi = lo + W;
    j.prev = (prev && prevf && W) ? prev : nullptr;
    j.prevf = j.prev ? prevf : nullptr;
    j.keys = R ? keys : nullptr;
    j.R = R ? (u32)R : 0u;
    j.vals = vals;
    j.found = found;
    j.e_out = e_out;
    j.created_acc = c->d_created;
    std::memcpy(blob->b, &j, sizeof j);
    return true;
}

hipError_t hm_serve_launch(nrg_ctx* c, ServeCtl* sc, const SmallJobBlob* hdr, u32 nslots, u64 first, u64 first_lo,
                           u64 session, u64 idle_ticks) {
    if (nslots > SERVE_SLOTS) return hipErrorInvalidValue;
    NRG_LAUNCH(c, "hm_serve", hm_serve_kernel, 1, SM_TPB, 0, c->stream, sc, hdr, nslots, first, first_lo, session,
               idle_ticks, c->d_table, c->slot_shift, (u64)(c->slots - 1), c->d_ctl);
    return hipGetLastError();
}

__global__ __launch_bounds__(TPB) void hm_init_table_kernel(Slot* table, u64 slots) {
    for (u64 s = blockIdx.x * (u64)TPB + threadIdx.x; s < slots; s += (u64)gridDim.x * TPB) {
        u64x2 z;
        z.x = EMPTY_KEY;
        z.y = 0;
        *(u64x2*)&table[s] = z;
        z.x = z.y = 0;
        *(u64x2*)&table[s].st[0] = z;
    }
}

// Epoch renormalisation (before the 32-bit epoch wraps): every present key becomes "present
// since before the replay rounds" (epoch 1); claims in flight do not exist at this point.
__global__ __launch_bounds__(TPB) void hm_renorm_kernel(Slot* table, u64 slots, DevCtl* ctl) {
    for (u64 s = blockIdx.x * (u64)TPB + threadIdx.x; s < slots; s += (u64)gridDim.x * TPB) {
        if (table[s].key == EMPTY_KEY) continue;
        u64x2 z;
        z.x = z.y = STAMP_PRESENT;
        *(u64x2*)&table[s].st[0] = z;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && ctl->sp_claim) ctl->sp.st[0] = ctl->sp.st[1] = STAMP_PRESENT;
}

// NrHashMap::default (benches/hashmap.rs:91-100): keys 0..n-1 -> k + off, inserted directly.
__global__ __launch_bounds__(TPB) void hm_prefill_range_kernel(Slot* table, u64 n, u64 off, u32 shift, u64 tmask,
                                                               DevCtl* ctl, u32 part, u32 parts) {
    __shared__ u32 s_ins;
    if (threadIdx.x == 0) s_ins = 0;
    __syncthreads();
    u32 inserted = 0;
    for (u64 k = blockIdx.x * (u64)TPB + threadIdx.x; k < n; k += (u64)gridDim.x * TPB) {
        if (parts > 1 && key_owner(k, parts) != part) continue;  // a key partition's share only
        if (k == EMPTY_KEY) {  // only reachable for n = 2^64, kept for the full key domain
            inserted += ctl->sp_claim == 0;
            ctl->sp.val = k + off;
            ctl->sp.st[0] = ctl->sp.st[1] = STAMP_PRESENT;
            ctl->sp_claim = 1;
            continue;
        }
        bool fresh;
        const long long s = claim_slot(table, k, table_home(k, shift), tmask, &fresh);
        if (s < 0) {
            atomicOr(&ctl->err, ERR_TABLE_FULL);
            continue;
        }
        table[s].val = k + off;
        table[s].st[0] = table[s].st[1] = STAMP_PRESENT;
        inserted += fresh;
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
    if (gid == 0 && ctl->sp_claim) {
        const u64 i = atomicAdd(&ctl->counter, 1ull);
        ok[i] = EMPTY_KEY;
        ov[i] = ctl->sp.val;
    }
    for (u64 s = gid; s < slots; s += (u64)gridDim.x * TPB) {
        const u64x2 e = *(const u64x2*)&table[s];
        if (e.x != EMPTY_KEY) {
            const u64 i = atomicAdd(&ctl->counter, 1ull);
            ok[i] = e.x;
            ov[i] = e.y;
        }
    }
}

__global__ __launch_bounds__(TPB) void hm_digest_kernel(const Slot* __restrict__ table, u64 slots,
                                                        const DevCtl* ctl, u64* out3) {
    __shared__ u64 s_c[TPB / 64], s_s[TPB / 64], s_x[TPB / 64];
    const u64 gid = blockIdx.x * (u64)TPB + threadIdx.x;
    u64 c = 0, sm = 0, x = 0;
    if (gid == 0 && ctl->sp_claim) {
        const u64 h = mix64(EMPTY_KEY ^ mix64(ctl->sp.val));
        c++;
        sm += h;
        x ^= h;
    }
    for (u64 s = gid; s < slots; s += (u64)gridDim.x * TPB) {
        const u64x2 e = *(const u64x2*)&table[s];
        if (e.x != EMPTY_KEY) {
            const u64 h = mix64(e.x ^ mix64(e.y));
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

// ---- host side ----------------------------------------------------------------------------
static RecSrc ring_src(nrg_ctx* c, const nrg_put* src, u64 lo) {
    RecSrc r;
    r.src = src;
    r.ring = (const nrg_put*)c->d_ring;
    r.mask = c->log_size - 1;
    r.lo = lo;
    return r;
}

// Stamp rounds: Puts per index thread by round size (one Get per read thread). K1 1 / 2 / 4 in us
// per round (profiles/r03_stamp_k1.txt): 50k Puts + 950k Gets 31.4 / 32.0, B1 (100k + 900k)
// 33.7 / 34.2 / 38.7, 200k + 800k 39.0 / 39.5, 200k + 900k 41.5 / 41.9, 400k + 900k 63.2 / 59.0,
// 500k + 500k 62.5 / 58.3 / 63.8, 800k + 900k (the N = 8 per-GPU round) - / 106.6 / 98.9; at
// 4 there the read blocks behind the index blocks start earlier, but without that many Gets 4
// loses (1M Puts, 2M Puts). NRG_KNOB_K1 overrides.
static u32 stamp_k1_for(const nrg_ctx* c, u64 n, u64 R) {
    if (c->k1_items) return c->k1_items >= 4 ? 4u : c->k1_items >= 2 ? 2u : 1u;
    if (n <= (1u << 18)) return 1u;
    return n >= 655360 && R >= n ? 4u : 2u;
}

// The jobs of one hm_round_kernel launch.
struct Launch {
    IndexJob ij{};
    StampJob sj{};
    ApplyJob aj{};
    ReadJob rj{};
    int ix = IX_PART_NODUP;
    u32 K1 = 1;
    u32 nb = 0;
};

// The deferred half of the last round rides in this launch: its apply (stamp rounds) and reads.
static void attach_deferred(nrg_ctx* c, Launch& L) {
    const HmDeferred& p = c->pend;
    L.rj.epoch = c->epoch;  // reads without a deferred round: every round applied
    if (p.valid) {
        const RecSrc rs = ring_src(c, p.src, p.lo);
        L.rj.keys = p.keys;
        L.rj.R = p.R;
        L.rj.vals = p.vals;
        L.rj.found = p.found;
        L.rj.epoch = p.epoch;
        L.rj.use_rec = p.apply;
        L.rj.rec = rs;
        if (p.apply) {
            L.aj.rec = rs;
            L.aj.n = p.n;
            L.aj.put_slot = c->d_put_slot[p.epoch & 1];
            L.aj.win = L.aj.put_slot + c->stamp_alloc;
            L.aj.over = L.aj.put_slot + 2 * c->stamp_alloc;
            L.aj.epoch = p.epoch;
            L.aj.nblocks = (u32)((p.n + TPB - 1) / TPB);
        }
    }
    c->pend = HmDeferred{};
}

template <int K1, int IX>
static void launch_round(nrg_ctx* c, const Launch& L, u32 blocks, unsigned lds) {
    if ((L.ij.exp | L.sj.exp) != 0)
        NRG_LAUNCH(c, "hm_round", (hm_round_kernel<K1, IX, true>), blocks, TPB, lds, c->stream, L.ij, L.sj, L.aj, L.rj,
                   c->d_table, c->slot_shift, (u64)(c->slots - 1), c->d_ctl);
    else
        NRG_LAUNCH(c, "hm_round", (hm_round_kernel<K1, IX, false>), blocks, TPB, lds, c->stream, L.ij, L.sj, L.aj,
                   L.rj, c->d_table, c->slot_shift, (u64)(c->slots - 1), c->d_ctl);
}

static hipError_t launch(nrg_ctx* c, Launch& L) {
    L.rj.nblocks = (u32)((L.rj.R + TPB * RPT - 1) / (TPB * RPT));
    L.sj.exp = c->exp >> 20;
    const u32 nix = L.ix == IX_STAMP ? L.sj.nblocks : L.ij.nblocks;
    L.ij.plain = L.sj.plain = L.rj.plain = ((c->exp >> 6) & 1) || (L.ix == IX_STAMP && nix);
    // reads beside a bucket or partition pass (which only read the table, or not even that), or
    // alone, with no stamp round's apply riding along: the table is quiescent
    L.rj.quiet = (L.ix != IX_STAMP || nix == 0) && L.aj.nblocks == 0;
    u32 blocks = nix + L.aj.nblocks + L.rj.nblocks;
    if (blocks == 0) return hipSuccess;
    // a pending skew sample rides in the launch's last block. (The combiner's error copy,
    // c->err_out, is taken only by hm_small_round_kernel, whose last write it is: a multi-block
    // launch's tail block may run before its other blocks' responses land, nrg_combiner retire().)
    if (c->sample_seq) {
        L.rj.s_acc = c->d_dup + ((c->dup_seq - 1) & 1) * HM_DUP_SLOTS;  // the window just ended
        L.rj.s_host = c->h_dup_dev;
        L.rj.s_seq = c->sample_seq;
        c->sample_seq = 0;
        blocks++;
    }
    unsigned lds = 0;
    if (nix && L.ix == IX_STAMP) {
        lds = L.K1 == 4 ? StampLds<4>::BYTES : L.K1 == 2 ? StampLds<2>::BYTES : StampLds<1>::BYTES;
    } else if (nix) {
        const bool dedup = L.ix == IX_PART;
        lds = L.K1 == 8   ? PartLds<8>::bytes(dedup, L.nb)
              : L.K1 == 4 ? PartLds<4>::bytes(dedup, L.nb)
              : L.K1 == 2 ? PartLds<2>::bytes(dedup, L.nb)
                          : PartLds<1>::bytes(dedup, L.nb);
    }
    if (!nix) launch_round<1, IX_PART_NODUP>(c, L, blocks, 0);
#define NRG_RK(KK, XX) else if (L.K1 == KK && L.ix == XX) launch_round<KK, XX>(c, L, blocks, lds)
    NRG_RK(1, IX_STAMP); NRG_RK(2, IX_STAMP); NRG_RK(4, IX_STAMP);
    NRG_RK(1, IX_PART); NRG_RK(1, IX_PART_ALL); NRG_RK(1, IX_PART_NODUP);
    NRG_RK(2, IX_PART); NRG_RK(2, IX_PART_ALL); NRG_RK(2, IX_PART_NODUP);
    NRG_RK(4, IX_PART); NRG_RK(4, IX_PART_ALL); NRG_RK(4, IX_PART_NODUP);
    NRG_RK(8, IX_PART); NRG_RK(8, IX_PART_ALL); NRG_RK(8, IX_PART_NODUP);
#undef NRG_RK
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t hm_flush(nrg_ctx* c) {
    if (!c->pend.valid) return hipSuccess;
    Launch L;
    attach_deferred(c, L);
    return launch(c, L);
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
    Launch L;
    attach_deferred(c, L);
    L.rj.keys = keys;
    L.rj.R = R;
    L.rj.vals = vals;
    L.rj.found = found;
    return launch(c, L);
}

hipError_t hm_alloc(nrg_ctx* c, u64 mb) {
    const u64 tiles = (mb + TPB - 1) / TPB;  // index tiles of >= TPB Puts
    const u64 ents = tiles * TPB;
    hipError_t e;
    if ((e = hipMalloc(&c->d_bk_ent, ents * 16)) != hipSuccess) return e;
    if ((e = hipMalloc(&c->d_bk_idx, ents * 4)) != hipSuccess) return e;
    if ((e = hipMalloc(&c->d_bk_cnt, (u64)HM_BK_MAX * tiles * sizeof(u32))) != hipSuccess) return e;
    if (c->stamp_max > mb) c->stamp_max = mb;
    // per parity: put_slot, win and over (stamp_max each; epoch tags, zeroed here and whenever
    // the epochs restart, hm_renorm)
    for (int i = 0; i < 2 && c->stamp_max; i++) {
        if ((e = hipMalloc(&c->d_put_slot[i], 3 * c->stamp_max * sizeof(u32))) != hipSuccess) return e;
        if ((e = hipMemsetAsync(c->d_put_slot[i], 0, 3 * c->stamp_max * sizeof(u32), c->stream)) != hipSuccess) return e;
    }
    // two sets of duplicate counters, by sample-window parity: the launch that takes a window's
    // sample reads and clears its set while its own index blocks add to the other
    if ((e = hipMalloc(&c->d_dup, 2 * HM_DUP_SLOTS * sizeof(u64))) != hipSuccess) return e;
    if ((e = hipMemsetAsync(c->d_dup, 0, 2 * HM_DUP_SLOTS * sizeof(u64), c->stream)) != hipSuccess) return e;
    void* h = nullptr;
    if ((e = hipHostMalloc(&h, 2 * sizeof(u64), hipHostMallocMapped)) != hipSuccess) return e;
    c->h_dup = (volatile u64*)h;
    c->h_dup[0] = c->h_dup[1] = 0;
    void* dp = nullptr;
    if ((e = hipHostGetDevicePointer(&dp, h, 0)) != hipSuccess) return e;
    c->h_dup_dev = (u64*)dp;
    return hipSuccess;
}

void hm_free(nrg_ctx* c) {
    for (int i = 0; i < 2; i++) {
        if (c->d_put_slot[i]) (void)hipFree(c->d_put_slot[i]);
        c->d_put_slot[i] = nullptr;
    }
    if (c->d_dup) (void)hipFree(c->d_dup);
    if (c->h_dup) (void)hipHostFree((void*)c->h_dup);
    c->d_dup = nullptr;
    c->h_dup = nullptr;
}

// Every dup_every rounds: read the previous sample (if it has landed) and decide whether the
// stream is skewed, then sample the rounds since. Skewed: more than 1/64 of the Puts were
// combined inside their index block or tile (Zipf 0.99 is far above, uniform keys far below).
// Stamp rounds then cost one same-address atomic per block for each hot key, and partition
// rounds (no atomics per Put) are faster at every size (Zipf 0.99 at 10 % / 50 % writes: 31.9 /
// 55.3 us, profiles/r04_part_sweep.txt); uniform streams below PART_MIN take stamp rounds.
static hipError_t skew_sample(nrg_ctx* c) {
    if (c->dup_seq && c->h_dup[0] == c->dup_seq && c->dup_puts_sampled)
        c->skewed = c->h_dup[1] * 64 > c->dup_puts_sampled;
    c->sample_seq = ++c->dup_seq;  // taken by the next hm_round launch (its last block)
    c->dup_puts_sampled = c->dup_puts;
    c->dup_puts = 0;
    c->dup_rounds = 0;
    return hipSuccess;
}

hipError_t hm_init(nrg_ctx* c) {
    hm_init_table_kernel<<<grid_for(c->slots, 16384), TPB, 0, c->stream>>>(c->d_table, c->slots);
    return hipGetLastError();
}

// The next round's epoch; before the 32-bit epoch wraps, every stamp is renormalised to epoch 1.
static hipError_t next_epoch(nrg_ctx* c, u32* e) {
    if (c->epoch >= c->epoch_limit) {
        hipError_t r = hm_flush(c);
        if (r != hipSuccess) return r;
        hm_renorm_kernel<<<grid_for(c->slots, 16384), TPB, 0, c->stream>>>(c->d_table, c->slots, c->d_ctl);
        if ((r = hipGetLastError()) != hipSuccess) return r;
        for (int i = 0; i < 2 && c->d_put_slot[i]; i++)  // win / over epoch tags of the old epochs
            if ((r = hipMemsetAsync(c->d_put_slot[i], 0, 3 * c->stamp_alloc * sizeof(u32), c->stream)) != hipSuccess)
                return r;
        c->epoch = 1;
    }
    *e = ++c->epoch;
    return hipSuccess;
}

// Replay the records [lo, lo+n) (from `src_recs` if given, else from the ring; writing the
// ring copy if write_ring) and answer R reads against the state after them.
hipError_t hm_replay_chunk(nrg_ctx* c, const void* src_recs, u64 lo, u64 n, bool write_ring, const u64* d_get_keys,
                           u64 R, u64* d_get_vals, uint8_t* d_get_found, u64 resp_lo, u64 resp_hi, u64* d_prev,
                           uint8_t* d_prev_found) {
    // (an empty round still completes the last round's deferred half: "the next call" does)
    if (n == 0) return R ? hm_reads(c, d_get_keys, R, d_get_vals, d_get_found) : hm_flush(c);
    if (n > HM_MAX_BATCH) return hipErrorInvalidValue;
    const nrg_put* src = (const nrg_put*)src_recs;
    const bool want_prev = d_prev && resp_lo < lo + n && resp_hi > lo;
    if (c->small_max && n <= c->small_max && n <= SM_W && R <= SM_R) {  // one launch, nothing deferred
        hipError_t e = small_round(c, src, lo, n, write_ring, d_get_keys, R, d_get_vals, d_get_found, resp_lo, resp_hi,
                                   want_prev ? d_prev : nullptr, d_prev_found);
        c->rounds++;
        return e;
    }
    // records the deferred half reads: the caller's buffer only when no ring copy is written
    const nrg_put* keep = (src && !write_ring) ? src : nullptr;
    hipError_t e;
    u32 epoch;
    if ((e = next_epoch(c, &epoch)) != hipSuccess) return e;
    Launch L;
    bool measured = false;  // the round's index role counts the Puts its per-tile dedup drops (key skew)
    // Round kinds (NRG_KNOB_PART 1, the default): stamp rounds (one launch, one stamp atomic per
    // distinct key per block) for unskewed rounds without previous values of fewer than
    // PART_MIN Puts; partition rounds (two launches, no device atomic per Put) for the rest.
    // Measured per round (profiles/r04_part_sweep.txt): B1 100k Puts + 900k Gets 34.8 stamp vs
    // 38.1 partition us, 200k + 900k 41.9 / 44.2, 400k + 900k 59.7 / 57.7, 800k + 900k 99.0 / 84.8,
    // 4M + 500k 413 / 271; previous values and skewed streams: partition rounds everywhere.
    constexpr u64 PART_MIN = 3ull << 17;
    const bool stamp0 = !want_prev && c->stamp_max && n <= c->stamp_max && !c->skewed;
    const bool part = !stamp0 || c->part_mode >= 2 || (c->part_mode == 1 && n >= PART_MIN);
    const bool stamp = stamp0 && !part;
    if (part) {
        // ---- partition round: {partition(e) | apply(e-1) | reads(e-1)}, then hm_papply_kernel(e) ----
        // Tiles of 256..2048 Puts, buckets of >= 64 Puts up to 1024 (one apply workgroup each): the
        // [tile][bucket] count words stay <= n / 2
        const u32 K1 = n <= (1u << 14) ? 1u : n <= (1u << 16) ? 2u : n <= (1u << 18) ? 4u : 8u;
        const u32 tile = TPB * K1;
        const u32 log2_slots = 64 - c->slot_shift;
        u32 nb_log = 0;
        while ((64ull << nb_log) < n && (1u << nb_log) < HM_BK_MAX) nb_log++;
        // apply workgroup width (NRG_KNOB_PA_TPB; 0: 512 threads over <= 512 buckets for rounds of
        // >= PA_WIDE_MIN Puts without previous values, else 256 over <= 1024). Round 6, 512 vs 1024
        // (profiles/r06/papply_width.txt): N = 8 per-GPU round 77.2 vs 78.9 us, N = 4 53.9-54.2 vs 54.9,
        // configs[2] 251.1-251.6 vs 255.0, 100 % writes 71.4 vs 72.9, 50 % 54.0 vs 55.1, Zipf 10 % 30.4
        // vs 30.8, Zipf 50 % 47.5 vs 47.9 (scrambled: equal)
        constexpr u64 PA_WIDE_MIN = 1ull << 16;
        const u32 pa_t = want_prev ? 256u : c->pa_tpb ? c->pa_tpb : n >= PA_WIDE_MIN ? 512u : 256u;
        const u32 pa_nb_log = pa_t == 1024 ? PaGeo<false, 1024>::NB_LOG : pa_t == 512 ? PaGeo<false, 512>::NB_LOG
                                                                                      : PaGeo<false, 256>::NB_LOG;
        if (nb_log > pa_nb_log) nb_log = pa_nb_log;
        if (nb_log > log2_slots) nb_log = log2_slots;
        // previous values keep every Put; otherwise a Put overwritten later in its tile is dropped
        // when the key stream is skewed (uniform streams have next to no such Puts: no LDS hash)
        // (the last round of every skew-sample window deduplicates too: it measures the skew)
        L.ix = want_prev ? IX_PART_ALL : (c->skewed || c->dup_rounds + 1 >= c->dup_every) ? IX_PART : IX_PART_NODUP;
        measured = L.ix == IX_PART;
        L.K1 = K1;
        L.nb = 1u << nb_log;
        IndexJob& ij = L.ij;
        ij.rec = ring_src(c, src, lo);
        ij.ring_out = write_ring ? (nrg_put*)c->d_ring : nullptr;
        ij.n = n;
        ij.nblocks = (u32)((n + tile - 1) / tile);
        ij.nb_log = nb_log;
        ij.bk_shift = log2_slots - nb_log;
        ij.ent = (u64x2*)c->d_bk_ent;
        ij.eidx = want_prev ? c->d_bk_idx : nullptr;
        ij.cnt = c->d_bk_cnt;
        ij.exp = 0;
        ij.dup_acc = c->d_dup + (c->dup_seq & 1) * HM_DUP_SLOTS;
        attach_deferred(c, L);  // the previous round's apply and reads ride along (partition only reads)
        if ((e = launch(c, L)) != hipSuccess) return e;
        PApplyJob aj{};
        aj.ent = ij.ent;
        aj.eidx = ij.eidx;
        aj.cnt = ij.cnt;
        aj.ntiles = ij.nblocks;
        aj.tile = tile;
        aj.nb = 1u << nb_log;
        aj.table = c->d_table;
        aj.shift = c->slot_shift;
        aj.tmask = c->slots - 1;
        aj.ctl = c->d_ctl;
        aj.created_acc = c->d_created;
        aj.lo = lo;
        aj.resp_lo = resp_lo;
        aj.resp_hi = resp_hi;
        aj.prev = d_prev;
        aj.prevf = d_prev_found;
        aj.stall = c->stall;
        aj.dbg = (c->exp & 2) ? c->d_dbg : nullptr;
        const unsigned dyn = ((ij.nblocks + 1) * 4 + ij.nblocks * 2 + 3) & ~3u;
        if (want_prev) NRG_LAUNCH(c, "hm_papply", (hm_papply_kernel<true, 256>), 1u << nb_log, 256, dyn, c->stream, aj);
        else if (pa_t == 1024) NRG_LAUNCH(c, "hm_papply", (hm_papply_kernel<false, 1024>), 1u << nb_log, 1024, dyn, c->stream, aj);
        else if (pa_t == 512 && n <= PA_NT_MAX)
            NRG_LAUNCH(c, "hm_papply", (hm_papply_kernel<false, 512, true>), 1u << nb_log, 512, dyn, c->stream, aj);
        else if (pa_t == 512) NRG_LAUNCH(c, "hm_papply", (hm_papply_kernel<false, 512>), 1u << nb_log, 512, dyn, c->stream, aj);
        else NRG_LAUNCH(c, "hm_papply", (hm_papply_kernel<false, 256>), 1u << nb_log, 256, dyn, c->stream, aj);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    } else if (stamp) {
        // ---- stamp round: one launch {index(e) | apply(e-1) | reads(e-1)} ----
        const u32 K1 = stamp_k1_for(c, n, R);
        const u32 tile = TPB * K1;
        L.ix = IX_STAMP;
        L.K1 = K1;
        measured = true;
        L.sj.rec = ring_src(c, src, lo);
        L.sj.ring_out = write_ring ? (nrg_put*)c->d_ring : nullptr;
        L.sj.n = n;
        L.sj.nblocks = (u32)((n + tile - 1) / tile);
        L.sj.epoch = epoch;
        L.sj.put_slot = c->d_put_slot[epoch & 1];
        L.sj.win = L.sj.put_slot + c->stamp_alloc;
        L.sj.over = L.sj.put_slot + 2 * c->stamp_alloc;
        L.sj.created_acc = c->d_created;
        L.sj.dup_acc = c->d_dup + (c->dup_seq & 1) * HM_DUP_SLOTS;
        attach_deferred(c, L);
        if ((e = launch(c, L)) != hipSuccess) return e;
    }
    c->rounds++;
    if (measured) c->dup_puts += n;  // the skew ratio is over the rounds that measured it
    if (++c->dup_rounds >= c->dup_every && (e = skew_sample(c)) != hipSuccess) return e;
    HmDeferred& p = c->pend;
    p.valid = true;
    p.epoch = epoch;
    p.apply = stamp;
    p.src = keep;
    p.lo = lo;
    p.n = n;
    p.keys = d_get_keys;
    p.R = R;
    p.vals = d_get_vals;
    p.found = d_get_found;
    if (!c->pipeline || (stamp && keep)) return hm_flush(c);
    return hipSuccess;
}

hipError_t hm_get_only(nrg_ctx* c, const u64* d_keys, u64 n, u64* d_vals, uint8_t* d_found) {
    return hm_reads(c, d_keys, n, d_vals, d_found);
}

hipError_t hm_prefill_range(nrg_ctx* c, u64 n, u64 off, u32 part, u32 parts) {
    hipError_t e = hm_flush(c);
    if (e != hipSuccess) return e;
    hm_prefill_range_kernel<<<grid_for(n, 8192), TPB, 0, c->stream>>>(c->d_table, n, off, c->slot_shift,
                                                                      c->slots - 1, c->d_ctl, part, parts);
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
