// common.hpp — shared device/host definitions for the nrgpu HIP kernels (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nrg {

typedef uint64_t u64;
typedef unsigned int u32;

// Empty-slot marker of the open-addressing tables. Keys span all of u64 (key 0 is used by
// benches/hashmap.rs:95-96,150), so the one key equal to the marker lives in a side slot
// (DevCtl::sp), giving the full HashMap<u64,u64> key domain (SURVEY.md §7 "Sentinels").
constexpr u64 EMPTY_KEY = ~0ull;

// Device error bits latched in DevCtl::err and reported by nrg_sync.
constexpr u32 ERR_TABLE_FULL = 1u;
constexpr u32 ERR_CAPACITY = 4u;

// Counters of keys created by replay rounds (index blocks add to slot blk % HM_CREATED_SLOTS).
constexpr u64 HM_CREATED_SLOTS = 8192;
// Slot buckets of the bucket election (hashmap.hip hm_elect_kernel): at most this many.
constexpr u32 HM_BK_MAX = 1024;

// splitmix64 finaliser — identical constants to oracle/nr_oracle.c (orc_mix64) so that
// device-generated workloads are reproducible by the CPU oracle.
__host__ __device__ __forceinline__ u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ u64 sm64_at(u64 seed, u64 i) {
    return mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ull);
}
__device__ __forceinline__ u64 mulhi64(u64 a, u64 b) { return __umul64hi(a, b); }

// Home slot of a key: top bits of the mixed key.
__device__ __forceinline__ u64 table_home(u64 key, u32 shift) { return mix64(key) >> shift; }

// 64-byte table slot, two per 128-B line. A random read costs one 128-B line at the memory
// side whatever its width (TCC_EA0_RDREQ_128B = 1 per lookup, profiles/r01_rdreq_size.txt),
// so the replay's bookkeeping rides in the same line as key and value:
//   stamp of parity p  last writer of the key in the most recent round of epoch parity p:
//             epoch << 32 | 1 + offset in that round (raised with atomicMax). Two words so a
//             round's index pass (parity e&1) can run while the previous round's apply and
//             reads (parity (e-1)&1) are still in flight.
//   created   epoch of the round that inserted the key (0 while a claim is in progress).
// Layout: a read needs {key, val} and {created, stamp of its parity}; `created` sits between
// the two stamps so that both pairs are one 16-B load (bytes 16-31 or 24-39).
struct __attribute__((aligned(64))) Slot {
    u64 key;     // EMPTY_KEY when free
    u64 val;
    u64 stamp1;  // odd epochs
    u32 created;
    u32 pad;
    u64 stamp0;  // even epochs
    u64 pad2[3];
};
__host__ __device__ __forceinline__ u64* slot_stamp(Slot* s, u32 par) { return par ? &s->stamp1 : &s->stamp0; }
__host__ __device__ __forceinline__ const u64* slot_stamp(const Slot* s, u32 par) {
    return par ? &s->stamp1 : &s->stamp0;
}

// One replica-wide control block in HBM.
struct __attribute__((aligned(64))) DevCtl {
    u32 err;          // latched ERR_* bits
    u32 pad0;
    u64 nkeys;        // hashmap: keys inserted directly (prefill)
    long long depth;  // stack: current length
    u64 counter;      // scratch counter (dump compaction)
    u64 nkeys_total;  // hashmap: nkeys + keys created by replay rounds (hm_count)
    long long depth0;      // stack: length before the chunk being replayed
    long long depth_next;  // stack: length after it (st_commit_kernel moves it to depth)
    u64 pad1;
    Slot sp;          // side slot for key == EMPTY_KEY (present iff sp.created != 0)
};

__device__ __forceinline__ u64 ld_relaxed(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32 ld_relaxed32(const u32* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave-wide (64-lane) inclusive scan helpers.
__device__ __forceinline__ u32 lane_id() { return threadIdx.x & 63; }

}  // namespace nrg
