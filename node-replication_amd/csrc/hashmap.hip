// hashmap.hip — NrHashMap replica replay on gfx950.
//
// Replaces the hot loop of Log::exec -> NrHashMap::dispatch_mut (nr/src/log.rs:494-518,
// benches/hashmap.rs:114-119, nr/examples/hashmap.rs:46-50) and the read path
// Replica::read_only -> dispatch (nr/src/replica.rs:483-497, benches/hashmap.rs:107-111).
//
// A replay "round" covers the log records [lo, lo+n) (one combined batch, or one chunk of
// a longer exec range) followed by a batch of R reads answered against the post-round state
// (the reads' sync-to-ctail contract: every write appended before the read is visible).
//
//   K1 hm_index     one thread per Put: claim the key's entry in a batch-local table (BLT,
//                   ~2n entries, L2/MALL resident) with a 64-bit CAS; atomicMax(last, i+1)
//                   selects the last writer in log order (= HashMap::insert sequence
//                   semantics for the final value); the entry's owner probes the main table
//                   once (read-only) and records the key's slot and pre-round value.
//                   Also clears the previous round's BLT entries (double-buffered BLT).
//   K2 hm_apply_get one launch, two roles: Put threads whose i+1 == last write the final
//                   value (update in place, or a CAS insert for new keys); Get threads
//                   probe BLT and main table concurrently (two independent loads in flight)
//                   and answer from the round's last writer when the key was written.
//   prev path       (only when previous-value responses are requested): stable radix sort
//                   of (BLT entry, i) pairs → each Put's previous value is its in-group
//                   predecessor's value, or the pre-round value captured by K1.
#include "internal.hpp"

namespace nrg {

constexpr int TPB = 256;

// record i of the round: from the caller's segment when given (fused append), else the ring
__device__ __forceinline__ nrg_put rec_at(const nrg_put* __restrict__ src, const nrg_put* ring, u64 ring_mask,
                                          u64 lo, u64 i) {
    return src ? src[i] : ring[(lo + i) & ring_mask];
}

__device__ __forceinline__ bool table_probe(const Slot* __restrict__ table, u64 k, u32 shift, u64 tmask,
                                            u64* slot, u64* val) {
    u64 s = table_home(k, shift);
    for (u64 pr = 0; pr <= tmask; pr++) {
        const Slot sl = table[s];
        if (sl.key == k) {
            *slot = s;
            *val = sl.val;
            return true;
        }
        if (sl.key == EMPTY_KEY) return false;
        s = (s + 1) & tmask;
    }
    return false;
}

// insert a key known to be absent (or overwrite if present); returns true if newly inserted
__device__ __forceinline__ int table_insert(Slot* table, u64 k, u64 v, u32 shift, u64 tmask) {
    u64 s = table_home(k, shift);
    for (u64 pr = 0; pr <= tmask; pr++) {
        const u64 old = atomicCAS(&table[s].key, EMPTY_KEY, k);
        if (old == EMPTY_KEY) {
            table[s].val = v;
            return 1;
        }
        if (old == k) {
            table[s].val = v;
            return 0;
        }
        s = (s + 1) & tmask;
    }
    return -1;
}

__global__ __launch_bounds__(TPB) void hm_index_kernel(
    const nrg_put* __restrict__ src, nrg_put* ring, u64 ring_mask, u64 lo, u64 n, int write_ring,
    BltEntry* blt, u64* __restrict__ blt_old, u64 bmask, u32* __restrict__ bslot,
    const Slot* __restrict__ table, u32 shift, u64 tmask, BltEntry* blt_prev, const u32* __restrict__ bslot_prev,
    u64 n_prev, DevCtl* ctl, u32 par, u32 special) {
    const u64 gid = blockIdx.x * (u64)TPB + threadIdx.x;
    const u64 stride = (u64)gridDim.x * TPB;
    if (gid == 0) {
        ctl->sp_last[par ^ 1u] = 0;
        ctl->sp_old_present = ctl->sp_present;
        ctl->sp_old_val = ctl->sp_val;
    }
    for (u64 j = gid; j < n_prev; j += stride) {
        const u32 b = bslot_prev[j];
        if (b != special) {
            BltEntry z;
            z.key = EMPTY_KEY;
            z.last = 0;
            z.info = 0;
            blt_prev[b] = z;
        }
    }
    for (u64 i = gid; i < n; i += stride) {
        const nrg_put rec = rec_at(src, ring, ring_mask, lo, i);
        if (write_ring) ring[(lo + i) & ring_mask] = rec;
        const u64 k = rec.key;
        if (k == EMPTY_KEY) {
            atomicMax(&ctl->sp_last[par], (u32)(i + 1));
            bslot[i] = special;
            continue;
        }
        u64 b = blt_home(k) & bmask;
        bool owner = false;
        for (u64 probes = 0;; probes++) {
            const u64 cur = ld_relaxed(&blt[b].key);
            if (cur == k) break;
            if (cur == EMPTY_KEY) {
                const u64 old = atomicCAS(&blt[b].key, EMPTY_KEY, k);
                if (old == EMPTY_KEY) {
                    owner = true;
                    break;
                }
                if (old == k) break;
            }
            b = (b + 1) & bmask;
            if (probes > bmask) {
                atomicOr(&ctl->err, ERR_BLT_FULL);
                break;
            }
        }
        atomicMax(&blt[b].last, (u32)(i + 1));
        bslot[i] = (u32)b;
        if (owner) {
            u64 s = 0, v = 0;
            const bool f = table_probe(table, k, shift, tmask, &s, &v);
            blt[b].info = f ? (u32)s : NEW_SLOT;
            blt_old[b] = f ? v : 0;
        }
    }
}

__global__ __launch_bounds__(TPB) void hm_apply_get_kernel(
    const nrg_put* __restrict__ src, const nrg_put* __restrict__ ring, u64 ring_mask, u64 lo, u64 n, u32 put_blocks,
    const BltEntry* __restrict__ blt, u64 bmask, const u32* __restrict__ bslot, Slot* table, u32 shift,
    u64 tmask, DevCtl* ctl, u32 par, u32 special, const u64* __restrict__ gkeys, u64 R,
    u64* __restrict__ gvals, uint8_t* __restrict__ gfound, int use_blt) {
    if (blockIdx.x < put_blocks) {
        u32 inserted = 0;
        for (u64 i = blockIdx.x * (u64)TPB + threadIdx.x; i < n; i += (u64)put_blocks * TPB) {
            const u32 b = bslot[i];
            if (b == special) {
                if (ctl->sp_last[par] == (u32)(i + 1)) {
                    if (!ctl->sp_present) inserted++;
                    ctl->sp_val = rec_at(src, ring, ring_mask, lo, i).val;
                    ctl->sp_present = 1;
                }
                continue;
            }
            const BltEntry e = blt[b];
            if (e.last != (u32)(i + 1)) continue;
            const nrg_put rec = rec_at(src, ring, ring_mask, lo, i);
            if (e.info != NEW_SLOT) {
                table[e.info].val = rec.val;
            } else {
                const int r = table_insert(table, rec.key, rec.val, shift, tmask);
                if (r < 0) atomicOr(&ctl->err, ERR_TABLE_FULL);
                if (r > 0) inserted++;
            }
        }
        if (inserted) atomicAdd(&ctl->nkeys, (u64)inserted);
        return;
    }
    const u64 j = (u64)(blockIdx.x - put_blocks) * TPB + threadIdx.x;
    if (j >= R) return;
    const u64 k = gkeys[j];
    u64 v = 0;
    uint8_t f = 0;
    if (k == EMPTY_KEY) {
        const u32 last = use_blt ? ctl->sp_last[par] : 0u;
        if (last) {
            v = rec_at(src, ring, ring_mask, lo, last - 1).val;
            f = 1;
        } else if (ctl->sp_present) {
            v = ctl->sp_val;
            f = 1;
        }
    } else {
        u64 s = table_home(k, shift);
        Slot sl = table[s];
        bool done = false;
        if (use_blt) {
            u64 b = blt_home(k) & bmask;
            BltEntry e = blt[b];
            while (e.key != EMPTY_KEY) {
                if (e.key == k) {
                    v = rec_at(src, ring, ring_mask, lo, e.last - 1).val;
                    f = 1;
                    done = true;
                    break;
                }
                b = (b + 1) & bmask;
                e = blt[b];
            }
        }
        if (!done) {
            for (u64 pr = 0; pr <= tmask; pr++) {
                if (sl.key == k) {
                    v = sl.val;
                    f = 1;
                    break;
                }
                if (sl.key == EMPTY_KEY) break;
                s = (s + 1) & tmask;
                sl = table[s];
            }
        }
    }
    gvals[j] = v;
    gfound[j] = f;
}

__global__ __launch_bounds__(TPB) void hm_prev_kernel(const u32* __restrict__ sk, const u32* __restrict__ sv, u64 n,
                                                      const nrg_put* __restrict__ src, const nrg_put* __restrict__ ring, u64 ring_mask, u64 lo,
                                                      const BltEntry* __restrict__ blt,
                                                      const u64* __restrict__ blt_old, const DevCtl* ctl,
                                                      u32 special, u64 resp_lo, u64 resp_hi,
                                                      u64* __restrict__ prev, uint8_t* __restrict__ prevf) {
    const u64 p = blockIdx.x * (u64)TPB + threadIdx.x;
    if (p >= n) return;
    const u32 b = sk[p];
    const u64 gidx = lo + sv[p];
    if (gidx < resp_lo || gidx >= resp_hi) return;
    u64 v = 0;
    uint8_t f = 0;
    if (p > 0 && sk[p - 1] == b) {
        v = rec_at(src, ring, ring_mask, lo, sv[p - 1]).val;
        f = 1;
    } else if (b == special) {
        f = (uint8_t)(ctl->sp_old_present != 0);
        v = f ? ctl->sp_old_val : 0;
    } else if (blt[b].info != NEW_SLOT) {
        v = blt_old[b];
        f = 1;
    }
    prev[gidx - resp_lo] = v;
    prevf[gidx - resp_lo] = f;
}

__global__ __launch_bounds__(TPB) void hm_prefill_range_kernel(Slot* table, u64 n, u64 off, u32 shift, u64 tmask,
                                                               DevCtl* ctl) {
    u32 inserted = 0;
    for (u64 k = blockIdx.x * (u64)TPB + threadIdx.x; k < n; k += (u64)gridDim.x * TPB) {
        const int r = table_insert(table, k, k + off, shift, tmask);
        if (r < 0) atomicOr(&ctl->err, ERR_TABLE_FULL);
        if (r > 0) inserted++;
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
        const Slot sl = table[s];
        if (sl.key != EMPTY_KEY) {
            const u64 i = atomicAdd(&ctl->counter, 1ull);
            ok[i] = sl.key;
            ov[i] = sl.val;
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
        const Slot sl = table[s];
        if (sl.key != EMPTY_KEY) {
            const u64 h = mix64(sl.key ^ mix64(sl.val));
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
        const u64* src = base + s * seg_stride_words + j * a.words;
        u64* dst = ring + ((dst_lo + r) & ring_mask) * a.words;
        for (u32 q = 0; q < a.words; q++) dst[q] = src[q];
    }
}

static inline unsigned grid_for(u64 n, u64 cap = 4096) {
    u64 g = (n + TPB - 1) / TPB;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

hipError_t hm_replay_chunk(nrg_ctx* c, const void* src_recs, u64 lo, u64 n, bool write_ring,
                           const u64* d_get_keys, u64 R, u64* d_get_vals, uint8_t* d_get_found, u64 resp_lo,
                           u64 resp_hi, u64* d_prev, uint8_t* d_prev_found, bool touch_log) {
    hipStream_t st = c->stream;
    const u64 ring_mask = c->log_size - 1;
    const u64 bmask = c->blt_size - 1;
    const u32 special = (u32)c->blt_size;
    const u64 tmask = c->slots - 1;
    nrg_put* ring = (nrg_put*)c->d_ring;
    const u32 par = c->parity;
    (void)touch_log;
    if (n > 0) {
        const u64 work = n > c->prev_n ? n : c->prev_n;
        timer_begin(c, "hm_index");
        hm_index_kernel<<<grid_for(work), TPB, 0, st>>>(
            (const nrg_put*)src_recs, ring, ring_mask, lo, n, write_ring ? 1 : 0, c->d_blt[par], c->d_blt_old[par],
            bmask, c->d_bslot[par], c->d_table, c->slot_shift, tmask, c->d_blt[par ^ 1], c->d_bslot[par ^ 1],
            c->prev_n, c->d_ctl, par, special);
        timer_end(c, "hm_index");
    }
    const u32 put_blocks = n ? grid_for(n, 1024) : 0;
    const u64 get_blocks = (R + TPB - 1) / TPB;
    if (put_blocks + get_blocks > 0) {
        timer_begin(c, "hm_apply_get");
        hm_apply_get_kernel<<<(unsigned)(put_blocks + get_blocks), TPB, 0, st>>>(
            (const nrg_put*)src_recs, ring, ring_mask, lo, n, put_blocks, c->d_blt[par], bmask, c->d_bslot[par], c->d_table, c->slot_shift,
            tmask, c->d_ctl, par, special, d_get_keys, R, d_get_vals, d_get_found, n > 0 ? 1 : 0);
        timer_end(c, "hm_apply_get");
    }
    if (n > 0 && d_prev && resp_lo < lo + n && resp_hi > lo) {
        u32 *sk = nullptr, *sv = nullptr;
        int bits = 1;
        while ((1ull << bits) <= c->blt_size) bits++;  // keys in [0, blt_size]
        timer_begin(c, "hm_prev");
        hipError_t e = sort_pairs(c->sort, c->d_bslot[par], nullptr, n, bits, st, &sk, &sv);
        if (e != hipSuccess) return e;
        hm_prev_kernel<<<(unsigned)((n + TPB - 1) / TPB), TPB, 0, st>>>(
            sk, sv, n, (const nrg_put*)src_recs, ring, ring_mask, lo, c->d_blt[par], c->d_blt_old[par], c->d_ctl, special, resp_lo, resp_hi,
            d_prev, d_prev_found);
        timer_end(c, "hm_prev");
    }
    if (n > 0) {
        c->prev_n = n;
        c->parity ^= 1u;
    }
    return hipGetLastError();
}

hipError_t hm_get_only(nrg_ctx* c, const u64* d_keys, u64 n, u64* d_vals, uint8_t* d_found) {
    if (n == 0) return hipSuccess;
    return hm_replay_chunk(c, nullptr, 0, 0, false, d_keys, n, d_vals, d_found, 0, 0, nullptr, nullptr, false);
}

hipError_t hm_prefill_range(nrg_ctx* c, u64 n, u64 off) {
    hm_prefill_range_kernel<<<grid_for(n, 8192), TPB, 0, c->stream>>>(c->d_table, n, off, c->slot_shift,
                                                                      c->slots - 1, c->d_ctl);
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
