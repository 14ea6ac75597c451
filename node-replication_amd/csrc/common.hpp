// common.hpp — shared device/host definitions for the nrgpu HIP kernels (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nrg {

typedef uint64_t u64;
typedef unsigned int u32;

// Empty-slot marker of the open-addressing tables. Keys span all of u64 (key 0 is used by
// benches/hashmap.rs:95-96,150), so the one key equal to the marker lives in a side slot
// (DevCtl::sp_*), giving the full HashMap<u64,u64> key domain (SURVEY.md §7 "Sentinels").
constexpr u64 EMPTY_KEY = ~0ull;
constexpr u32 NEW_SLOT = 0xFFFFFFFFu;  // BLT info: key absent from the table before the round

// Device error bits latched in DevCtl::err and reported by nrg_sync.
constexpr u32 ERR_TABLE_FULL = 1u;
constexpr u32 ERR_BLT_FULL = 2u;
constexpr u32 ERR_CAPACITY = 4u;

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

// Main-table home slot: top bits of the mixed key. BLT home slot: low bits (independent).
__device__ __forceinline__ u64 table_home(u64 key, u32 shift) { return mix64(key) >> shift; }
__device__ __forceinline__ u64 blt_home(u64 key) { return mix64(key ^ 0x5bd1e9955bd1e995ull); }

// One replica-wide control block in HBM.
struct DevCtl {
    u32 err;             // latched ERR_* bits
    u32 pad0;
    u64 nkeys;           // hashmap: number of keys (including the side-slot key)
    u64 sp_present;      // side slot for key == EMPTY_KEY
    u64 sp_val;
    u64 sp_stamp;        // epoch << 32 | 1 + round offset of the last Put to EMPTY_KEY
    long long depth;     // stack: current length
    u64 counter;         // scratch counter (dump compaction)
    u64 pad1[8];
};

// 32-byte table slot; a random 16-B read costs a whole 128-B line on MI355X anyway, so the
// last-writer stamp and creation epoch ride in the same line as key and value.
struct __attribute__((aligned(32))) Slot {
    u64 key;      // EMPTY_KEY when free
    u64 val;
    u64 stamp;    // epoch << 32 | 1 + offset of the round's last Put to key (atomicMax)
    u32 created;  // epoch of the round that inserted key
    u32 pad;
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
