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

// Counters of keys created by replay rounds (elector blocks add to slot blk % HM_CREATED_SLOTS).
constexpr u64 HM_CREATED_SLOTS = 8192;
// Slot buckets of a replay round (hashmap.hip hm_elect_kernel): at most this many.
constexpr u32 HM_BK_MAX = 1024;
// Largest hashmap replay chunk: keeps the elector's per-tile LDS tables (one u32 + one u16
// per index tile of >= 1024 Puts) and 16-bit tile offsets within bounds.
constexpr u64 HM_MAX_BATCH = 1ull << 23;

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

// 16-byte table slot {key, value}, eight per 128-B line: 2^26 slots = 1 GiB. Nothing else lives
// in the table: a replay round never writes a slot while the same launch reads it (hashmap.hip:
// the index pass only reads, the elector launch claims keys and stores values), so no epochs,
// stamps or creation marks are needed, and the footprint a random Get ranges over is 4x smaller
// than with the 64-B slots of the first design (1 GiB vs 4 GiB: 23.8 vs 27.5 us per 1M Gets,
// profiles/r01_get_footprint.txt).
struct __attribute__((aligned(16))) Slot {
    u64 key;  // EMPTY_KEY when free
    u64 val;
};

// One replica-wide control block in HBM.
struct __attribute__((aligned(64))) DevCtl {
    u32 err;          // latched ERR_* bits
    u32 sp_present;   // hashmap: the key EMPTY_KEY is present (its value is sp_val)
    u64 nkeys;        // hashmap: keys inserted directly (prefill)
    long long depth;  // stack: current length
    u64 counter;      // scratch counter (dump compaction)
    u64 nkeys_total;  // hashmap: nkeys + keys created by replay rounds (hm_count)
    long long depth0;      // stack: length before the chunk being replayed
    long long depth_next;  // stack: length after it (st_commit_kernel moves it to depth)
    u64 sp_val;       // hashmap: value of the key EMPTY_KEY (side slot)
    u64 sp_st[3];     // hashmap overlay rounds: last writer (i+1) of EMPTY_KEY, per overlay
};

// Overlay slot (hashmap.hip overlay rounds): a key written by the round and the largest i+1
// among its Puts (the round's last writer of the key, raised with atomicMax).
struct __attribute__((aligned(16))) OvSlot {
    u64 key;  // EMPTY_KEY when free
    u64 st;   // i + 1 of the last writer
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
