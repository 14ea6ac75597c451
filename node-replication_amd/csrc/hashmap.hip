// hashmap.hip — NrHashMap replica replay on gfx950.
//
// Replaces the hot loop of Log::exec -> NrHashMap::dispatch_mut (nr/src/log.rs:494-518,
// benches/hashmap.rs:114-119, nr/examples/hashmap.rs:46-50) and the read path
// Replica::read_only -> dispatch (nr/src/replica.rs:483-497, benches/hashmap.rs:107-111).
//
// Table: 2^k open-addressing slots of 32 B {key, val, stamp, created}; four slots per 128-B
// line, the HBM access granule for random reads on MI355X (microbench/random_gather.hip,
// profiles/r01_random_gather_fetch_size.txt). A replay "round" covers the log records
// [lo, lo+n) with a fresh epoch e (one per round, never reused):
//
//   K1 hm_index     one thread per Put (4 per thread): probe the key's slot (read-only), or
//                   claim an empty one with a 64-bit CAS (new key, created = e); the last
//                   writer in log order is elected by atomicMax(slot.stamp, e<<32 | i+1),
//                   pre-combined per block in LDS so a hot key costs one global atomic per
//                   block (Zipf streams). Writes the log copy when the round is appended here.
//   prev path       only when previous-value responses are requested: stable radix sort of
//                   (slot, i) -> a Put's previous value is its in-group predecessor's value,
//                   or the slot's pre-round value (absent if created == e). Runs before K2.
//   K2 hm_apply_get one launch, two roles: Put threads whose stamp is (e, i+1) store the
//                   final value; Get threads probe the table once and read the value from
//                   the round's log record when the slot's stamp carries epoch e.
// The result equals the sequential replay: last-writer-wins per key in log order, reads
// after the round's writes (SURVEY.md §8a round semantics).
#include "internal.hpp"

namespace nrg {

constexpr int TPB = 256;
// K1 geometry: ITEMS puts per thread, an LDS combining table of 2*TPB*ITEMS entries per block

// record i of the round: from the caller's segment when given (fused append), else the ring
__device__ __forceinline__ nrg_put rec_at(const nrg_put* __restrict__ src, const nrg_put* ring, u64 ring_mask,
                                          u64 lo, u64 i) {
    return src ? src[i] : ring[(lo + i) & ring_mask];
}

__device__ __forceinline__ u64 stamp_of(u32 epoch, u64 i) { return ((u64)epoch << 32) | (i + 1); }

// Load a whole slot with two 16-B loads issued together. The empty asm pins both values at
// this point: otherwise hipcc sinks the {val, stamp} load below the key compare of the probe
// loop, turning every Get into two dependent accesses to its line.
__device__ __forceinline__ Slot load_slot(const Slot* p) {
    typedef u64 u64x2 __attribute__((ext_vector_type(2)));
    const u64x2 a = *(const u64x2*)p;
    const u64x2 b = *((const u64x2*)p + 1);
    u64 k = a.x, v = a.y, st = b.x;
    asm volatile("" : "+v"(k), "+v"(v), "+v"(st));
    Slot s;
    s.key = k;
    s.val = v;
    s.stamp = st;
    s.created = (u32)b.y;
    s.pad = 0;
    return s;
}

// Read-only probe from slot s whose contents `sl` the caller already loaded: slot or -1.
__device__ __forceinline__ long long probe_from(const Slot* __restrict__ table, u64 k, u64 s, u64 tmask, Slot sl,
                                                Slot* out) {
    for (u64 pr = 0; pr <= tmask; pr++) {
        if (sl.key == k) {
            *out = sl;
            return (long long)s;
        }
        if (sl.key == EMPTY_KEY) return -1;
        s = (s + 1) & tmask;
        sl = load_slot(&table[s]);
    }
    return -2;
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

template <int K1_ITEMS>
__global__ __launch_bounds__(TPB) void hm_index_kernel(const nrg_put* __restrict__ src, nrg_put* ring, u64 ring_mask,
                                                       u64 lo, u64 n, int write_ring, Slot* table, u32 shift,
                                                       u64 tmask, u32* __restrict__ put_slot, DevCtl* ctl, u32 epoch) {
    constexpr int K1_TILE = TPB * K1_ITEMS;
    constexpr int K1_LDS = 2 * K1_TILE;
    __shared__ u32 s_slot[K1_LDS];
    __shared__ u32 s_max[K1_LDS];
    for (int q = threadIdx.x; q < K1_LDS; q += TPB) {
        s_slot[q] = 0xFFFFFFFFu;
        s_max[q] = 0;
    }
    __syncthreads();
    const u64 base = (u64)blockIdx.x * K1_TILE;
    u32 created = 0;
    u64 sl_idx[K1_ITEMS];
    u64 key0[K1_ITEMS];
    nrg_put rec[K1_ITEMS];
    // issue every record load and every first probe before waiting on any of them
#pragma unroll
    for (int j = 0; j < K1_ITEMS; j++) {
        const u64 i = base + (u64)j * TPB + threadIdx.x;
        rec[j] = i < n ? rec_at(src, ring, ring_mask, lo, i) : nrg_put{EMPTY_KEY, 0};
    }
#pragma unroll
    for (int j = 0; j < K1_ITEMS; j++) {
        const u64 i = base + (u64)j * TPB + threadIdx.x;
        if (i < n && write_ring) ring[(lo + i) & ring_mask] = rec[j];
        sl_idx[j] = table_home(rec[j].key, shift);
        key0[j] = rec[j].key != EMPTY_KEY ? table[sl_idx[j]].key : EMPTY_KEY;
    }
#pragma unroll
    for (int j = 0; j < K1_ITEMS; j++) {
        const u64 i = base + (u64)j * TPB + threadIdx.x;
        if (i >= n) continue;
        const u64 k = rec[j].key;
        if (k == EMPTY_KEY) {  // the side-slot key
            atomicMax(&ctl->sp_stamp, stamp_of(epoch, i));
            put_slot[i] = 0xFFFFFFFFu;
            continue;
        }
        const long long s = find_or_claim(table, k, sl_idx[j], tmask, key0[j], epoch, &created);
        if (s < 0) {
            atomicOr(&ctl->err, ERR_TABLE_FULL);
            put_slot[i] = 0xFFFFFFFEu;
            continue;
        }
        put_slot[i] = (u32)s;
        // combine in LDS: max (i+1) per slot within the block
        u32 h = (u32)(mix64((u64)s) & (K1_LDS - 1));
        for (;;) {
            const u32 old = atomicCAS(&s_slot[h], 0xFFFFFFFFu, (u32)s);
            if (old == 0xFFFFFFFFu || old == (u32)s) break;
            h = (h + 1) & (K1_LDS - 1);
        }
        atomicMax(&s_max[h], (u32)(i + 1));
    }
    if (created) atomicAdd(&ctl->nkeys, (u64)created);
    __syncthreads();
    for (int q = threadIdx.x; q < K1_LDS; q += TPB) {
        const u32 s = s_slot[q];
        if (s != 0xFFFFFFFFu) atomicMax(&table[s].stamp, ((u64)epoch << 32) | s_max[q]);
    }
}

// K2a: the round's last writer of each key (stamp == (e, i+1)) stores the final value.
__global__ __launch_bounds__(TPB) void hm_apply_kernel(const nrg_put* __restrict__ src, const nrg_put* __restrict__ ring,
                                                       u64 ring_mask, u64 lo, u64 n, const u32* __restrict__ put_slot,
                                                       Slot* table, DevCtl* ctl, u32 epoch) {
    u32 inserted = 0;
    for (u64 i = blockIdx.x * (u64)TPB + threadIdx.x; i < n; i += (u64)gridDim.x * TPB) {
        const u32 s = put_slot[i];
        const u64 want = stamp_of(epoch, i);
        if (s == 0xFFFFFFFFu) {  // side-slot key
            if (ctl->sp_stamp == want) {
                if (!ctl->sp_present) inserted++;
                ctl->sp_val = rec_at(src, ring, ring_mask, lo, i).val;
                ctl->sp_present = 1;
            }
            continue;
        }
        if (s == 0xFFFFFFFEu) continue;  // table full (reported)
        if (table[s].stamp == want) table[s].val = rec_at(src, ring, ring_mask, lo, i).val;
    }
    if (inserted) atomicAdd(&ctl->nkeys, (u64)inserted);
}

// K2b: Gets against the state after round `epoch` (dispatch after sync-to-tail). A slot
// counts only if 0 < created <= epoch: with rounds pipelined, the next round's hm_index may
// already be claiming slots for its new keys (created is 0 until its claimer writes it, then
// epoch+1), and those keys do not exist yet for these reads.
template <int G>
__global__ __launch_bounds__(TPB) void hm_get_kernel(const Slot* __restrict__ table, u32 shift, u64 tmask,
                                                     const DevCtl* ctl, u32 epoch, const u64* __restrict__ gkeys, u64 R,
                                                     u64* __restrict__ gvals, uint8_t* __restrict__ gfound) {
    // G Gets per thread: all key loads, then all first-slot loads, are in flight together
    const u64 jb = (u64)blockIdx.x * TPB * G + threadIdx.x;
    u64 k[G];
    Slot first[G];
#pragma unroll
    for (int g = 0; g < G; g++) {
        const u64 j = jb + (u64)g * TPB;
        k[g] = j < R ? gkeys[j] : EMPTY_KEY;
    }
#pragma unroll
    for (int g = 0; g < G; g++) first[g] = load_slot(&table[table_home(k[g], shift)]);
#pragma unroll
    for (int g = 0; g < G; g++) {
        const u64 j = jb + (u64)g * TPB;
        if (j >= R) break;
        u64 v = 0;
        uint8_t f = 0;
        if (k[g] == EMPTY_KEY) {
            if (ctl->sp_present) {
                v = ctl->sp_val;
                f = 1;
            }
        } else {
            Slot sl;
            const long long s = probe_from(table, k[g], table_home(k[g], shift), tmask, first[g], &sl);
            if (s >= 0 && sl.created != 0 && sl.created <= epoch) {
                f = 1;
                v = sl.val;
            }
        }
        gvals[j] = v;
        gfound[j] = f;
    }
}

__global__ __launch_bounds__(TPB) void hm_prev_kernel(const u32* __restrict__ sk, const u32* __restrict__ sv, u64 n,
                                                      const nrg_put* __restrict__ src, const nrg_put* __restrict__ ring,
                                                      u64 ring_mask, u64 lo, const Slot* __restrict__ table,
                                                      const DevCtl* ctl, u32 epoch, u64 resp_lo, u64 resp_hi,
                                                      u64* __restrict__ prev, uint8_t* __restrict__ prevf) {
    const u64 p = blockIdx.x * (u64)TPB + threadIdx.x;
    if (p >= n) return;
    const u32 s = sk[p];
    const u64 gidx = lo + sv[p];
    if (gidx < resp_lo || gidx >= resp_hi) return;
    u64 v = 0;
    uint8_t f = 0;
    const bool has_pred = p > 0 && sk[p - 1] == s;
    if (has_pred) {
        v = rec_at(src, ring, ring_mask, lo, sv[p - 1]).val;
        f = 1;
    } else if (s == 0xFFFFFFFFu) {  // side slot, before K2 of this round: pre-round state
        f = (uint8_t)(ctl->sp_present != 0);
        v = f ? ctl->sp_val : 0;
    } else if (s != 0xFFFFFFFEu && table[s].created != epoch) {  // existed before; K2 not run yet
        v = table[s].val;
        f = 1;
    }
    prev[gidx - resp_lo] = v;
    prevf[gidx - resp_lo] = f;
}

__global__ __launch_bounds__(TPB) void hm_init_table_kernel(Slot* table, u64 slots) {
    for (u64 s = blockIdx.x * (u64)TPB + threadIdx.x; s < slots; s += (u64)gridDim.x * TPB) {
        Slot z;
        z.key = EMPTY_KEY;
        z.val = 0;
        z.stamp = 0;
        z.created = 0;
        z.pad = 0;
        table[s] = z;
    }
}

__global__ __launch_bounds__(TPB) void hm_prefill_range_kernel(Slot* table, u64 n, u64 off, u32 shift, u64 tmask,
                                                               DevCtl* ctl, u32 epoch) {
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
    if (inserted) atomicAdd(&ctl->nkeys, (u64)inserted);
}

__global__ __launch_bounds__(TPB) void hm_dump_kernel(const Slot* __restrict__ table, u64 slots, DevCtl* ctl,
                                                      u64* __restrict__ ok, u64* __restrict__ ov) {
    const u64 gid = blockIdx.x * (u64)TPB + threadIdx.x;
    if (gid == 0 && ctl->sp_present) {
        const u64 i = atomicAdd(&ctl->counter, 1ull);
        ok[i] = EMPTY_KEY;
        ov[i] = ctl->sp_val;
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
    if (gid == 0 && ctl->sp_present) {
        const u64 h = mix64(EMPTY_KEY ^ mix64(ctl->sp_val));
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

__global__ void gen_uniform_kernel(u64* out, u64 n, u64 seed, u64 span) {
    for (u64 i = blockIdx.x * (u64)TPB + threadIdx.x; i < n; i += (u64)gridDim.x * TPB)
        out[i] = mulhi64(sm64_at(seed, i), span);
}
__global__ void gen_raw_kernel(u64* out, u64 n, u64 seed) {
    for (u64 i = blockIdx.x * (u64)TPB + threadIdx.x; i < n; i += (u64)gridDim.x * TPB) out[i] = sm64_at(seed, i);
}
__global__ void gen_puts_kernel(nrg_put* out, const u64* k, const u64* v, u64 n) {
    for (u64 i = blockIdx.x * (u64)TPB + threadIdx.x; i < n; i += (u64)gridDim.x * TPB) {
        nrg_put p;
        p.key = k[i];
        p.val = v[i];
        out[i] = p;
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

hipError_t hm_init(nrg_ctx* c) {
    hm_init_table_kernel<<<grid_for(c->slots, 16384), TPB, 0, c->stream>>>(c->d_table, c->slots);
    return hipGetLastError();
}

hipError_t hm_replay_chunk(nrg_ctx* c, const void* src_recs, u64 lo, u64 n, bool write_ring,
                           const u64* d_get_keys, u64 R, u64* d_get_vals, uint8_t* d_get_found, u64 resp_lo,
                           u64 resp_hi, u64* d_prev, uint8_t* d_prev_found, bool touch_log) {
    hipStream_t st = c->stream;
    const u64 ring_mask = c->log_size - 1;
    const u64 tmask = c->slots - 1;
    nrg_put* ring = (nrg_put*)c->d_ring;
    const nrg_put* src = (const nrg_put*)src_recs;
    (void)touch_log;
    const u32 epoch = n > 0 ? ++c->epoch : c->epoch;
    if (n > 0) {
        timer_begin(c, "hm_index", st);
#define NRG_K1(IT)                                                                                            \
    hm_index_kernel<IT><<<(unsigned)((n + TPB * IT - 1) / (TPB * IT)), TPB, 0, st>>>(                           \
        src, ring, ring_mask, lo, n, write_ring ? 1 : 0, c->d_table, c->slot_shift, tmask, c->d_put_slot, c->d_ctl, \
        epoch)
        if (c->k1_items >= 4)
            NRG_K1(4);
        else if (c->k1_items == 2)
            NRG_K1(2);
        else
            NRG_K1(1);
#undef NRG_K1
        timer_end(c, "hm_index", st);
        if (d_prev && resp_lo < lo + n && resp_hi > lo) {
            u32 *sk = nullptr, *sv = nullptr;
            timer_begin(c, "hm_prev", st);
            // slot ids < 2^log2_slots; the side-slot key (0xFFFFFFFF) sorts last
            hipError_t e = sort_pairs(c->sort, c->d_put_slot, nullptr, n, 32, st, &sk, &sv);
            if (e != hipSuccess) return e;
            hm_prev_kernel<<<(unsigned)((n + TPB - 1) / TPB), TPB, 0, st>>>(
                sk, sv, n, src, ring, ring_mask, lo, c->d_table, c->d_ctl, epoch, resp_lo, resp_hi, d_prev,
                d_prev_found);
            timer_end(c, "hm_prev", st);
        }
    }
    hipError_t e;
    if (n > 0) {
        // values of this round may only be stored once the previous round's reads (possibly
        // still running on the side stream) are done with the old ones
        if ((e = side_join(c)) != hipSuccess) return e;
        timer_begin(c, "hm_apply", st);
        hm_apply_kernel<<<grid_for(n, 1024), TPB, 0, st>>>(src, ring, ring_mask, lo, n, c->d_put_slot, c->d_table,
                                                           c->d_ctl, epoch);
        timer_end(c, "hm_apply", st);
    }
    if (R > 0) {
        // Reads of this round run on the side stream when pipelining, so that they overlap the
        // next round's hm_index (which only claims slots and raises stamps, see hm_get_kernel).
        hipStream_t gs = st;
        if (c->pipeline) {
            if ((e = hipEventRecord(c->ev_applied, st)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(c->side_stream, c->ev_applied, 0)) != hipSuccess) return e;
            gs = c->side_stream;
        }
        const u32 G = c->gets_per_thread >= 4 ? 4 : (c->gets_per_thread == 2 ? 2 : 1);
        const unsigned gb = (unsigned)((R + TPB * G - 1) / (TPB * G));
        timer_begin(c, "hm_get", gs);
        if (G == 4)
            hm_get_kernel<4><<<gb, TPB, 0, gs>>>(c->d_table, c->slot_shift, tmask, c->d_ctl, epoch, d_get_keys, R,
                                                d_get_vals, d_get_found);
        else if (G == 2)
            hm_get_kernel<2><<<gb, TPB, 0, gs>>>(c->d_table, c->slot_shift, tmask, c->d_ctl, epoch, d_get_keys, R,
                                                d_get_vals, d_get_found);
        else
            hm_get_kernel<1><<<gb, TPB, 0, gs>>>(c->d_table, c->slot_shift, tmask, c->d_ctl, epoch, d_get_keys, R,
                                                d_get_vals, d_get_found);
        timer_end(c, "hm_get", gs);
        if (c->pipeline) {
            if ((e = hipEventRecord(c->ev_reads_done, gs)) != hipSuccess) return e;
            c->side_pending = true;
        }
    }
    return hipGetLastError();
}

hipError_t side_join(nrg_ctx* c) {
    if (!c->side_pending) return hipSuccess;
    c->side_pending = false;
    return hipStreamWaitEvent(c->stream, c->ev_reads_done, 0);
}

hipError_t hm_get_only(nrg_ctx* c, const u64* d_keys, u64 n, u64* d_vals, uint8_t* d_found) {
    if (n == 0) return hipSuccess;
    return hm_replay_chunk(c, nullptr, 0, 0, false, d_keys, n, d_vals, d_found, 0, 0, nullptr, nullptr, false);
}

hipError_t hm_prefill_range(nrg_ctx* c, u64 n, u64 off) {
    hipError_t e = side_join(c);
    if (e != hipSuccess) return e;
    hm_prefill_range_kernel<<<grid_for(n, 8192), TPB, 0, c->stream>>>(c->d_table, n, off, c->slot_shift,
                                                                      c->slots - 1, c->d_ctl, c->epoch);
    return hipGetLastError();
}

hipError_t hm_dump(nrg_ctx* c, u64* d_keys, u64* d_vals) {
    hipError_t e = hipMemsetAsync(&c->d_ctl->counter, 0, sizeof(u64), c->stream);
    if (e != hipSuccess) return e;
    hm_dump_kernel<<<grid_for(c->slots, 8192), TPB, 0, c->stream>>>(c->d_table, c->slots, c->d_ctl, d_keys, d_vals);
    return hipGetLastError();
}

hipError_t hm_digest(nrg_ctx* c, u64* d_out3) {
    hipError_t e = hipMemsetAsync(d_out3, 0, 3 * sizeof(u64), c->stream);
    if (e != hipSuccess) return e;
    hm_digest_kernel<<<grid_for(c->slots, 8192), TPB, 0, c->stream>>>(c->d_table, c->slots, c->d_ctl, d_out3);
    return hipGetLastError();
}

hipError_t gen_uniform(nrg_ctx* c, u64* d, u64 n, u64 seed, u64 span) {
    gen_uniform_kernel<<<grid_for(n, 8192), TPB, 0, c->stream>>>(d, n, seed, span);
    return hipGetLastError();
}
hipError_t gen_raw(nrg_ctx* c, u64* d, u64 n, u64 seed) {
    gen_raw_kernel<<<grid_for(n, 8192), TPB, 0, c->stream>>>(d, n, seed);
    return hipGetLastError();
}
hipError_t gen_puts(nrg_ctx* c, nrg_put* d, const u64* k, const u64* v, u64 n) {
    gen_puts_kernel<<<grid_for(n, 8192), TPB, 0, c->stream>>>(d, k, v, n);
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
