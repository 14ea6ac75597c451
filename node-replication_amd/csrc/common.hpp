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
    u64 sp_old_present;  // side slot before the current round (previous-value responses)
    u64 sp_old_val;
    u32 sp_last[2];      // per round parity: 1 + last log offset of a Put to EMPTY_KEY
    long long depth;     // stack: current length
    u64 counter;         // scratch counter (dump compaction)
    u64 pad1[6];
};

// 16-byte table slot {key, value}: one dwordx4 load fetches both (AoS keeps Get at one
// random 64-B sector).
struct __attribute__((aligned(16))) Slot {
    u64 key;
    u64 val;
};

// Batch-local table entry: one per distinct key written in a round.
struct __attribute__((aligned(16))) BltEntry {
    u64 key;   // EMPTY_KEY when free
    u32 last;  // 1 + log offset (within the round) of the last Put to key  (last-writer-wins)
    u32 info;  // main-table slot of key before the round, or NEW_SLOT
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
