// common.hpp — shared device/host definitions for the nrgpu HIP kernels (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nrg {

typedef uint64_t u64;
typedef unsigned int u32;
typedef unsigned short u16;

// Empty-slot marker of the open-addressing tables. Keys span all of u64 (key 0 is used by
// benches/hashmap.rs:95-96,150), so the one key equal to the marker lives in a side slot
// (DevCtl::sp), giving the full HashMap<u64,u64> key domain (SURVEY.md §7 "Sentinels").
constexpr u64 EMPTY_KEY = ~0ull;

// Device error bits latched in DevCtl::err and reported by nrg_sync.
constexpr u32 ERR_TABLE_FULL = 1u;
constexpr u32 ERR_CAPACITY = 4u;
constexpr u32 ERR_GROUP = 8u;  // a replica group's ranks disagreed on a round's segment lengths (group.cpp)

// Counters of keys created by replay rounds (claiming blocks add to slot blk % HM_CREATED_SLOTS).
constexpr u64 HM_CREATED_SLOTS = 8192;
// Counters of Puts combined inside their index block (key skew statistic, hm_dup_sample_kernel).
constexpr u64 HM_DUP_SLOTS = 64;
// Slot buckets of a partition round (hashmap.hip part_role / hm_papply_kernel): at most this many.
constexpr u32 HM_BK_MAX = 1024;
// Largest hashmap replay chunk: keeps the partition apply's per-tile LDS prefix (one u32 + one
// u16 per tile of 2048 Puts) and 16-bit tile offsets within bounds.
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

// Owner of a key among `parts` key partitions (partition.hip): the low 32 bits of the mixed key
// scaled to [0, parts), independent of the home-slot bits below.
constexpr u32 PT_MAX_PARTS = 64;
__host__ __device__ __forceinline__ u32 key_owner(u64 key, u32 parts) {
    return (u32)(((mix64(key) & 0xFFFFFFFFull) * parts) >> 32);
}

// Home slot of a key: top bits of the mixed key.
__device__ __forceinline__ u64 table_home(u64 key, u32 shift) { return mix64(key) >> shift; }

// 32-byte table slot, four per 128-B line (2^26 slots = 2 GiB). A random read costs one 128-B
// line at the memory side whatever its width (profiles/r01_rdreq_size.txt), so the replay's
// per-key bookkeeping rides in the key's line: a Get reads {key, val} and the stamp of its
// round's parity, two 16-B loads of one line.
//   st[p]  stamp of the last round of parity p that wrote or created the key:
//          epoch << 32 | (i+1) for the round's last writer (raised with atomicMax), or
//          epoch << 32 | 0 as the mark a round leaves in the OTHER parity when it creates the key.
//          0 = never stamped: a slot whose claim is still in flight reads as absent.
// Epoch 1 means "present since before any replay round" (prefill, bucket-round claims); replay
// rounds take epochs 2, 3, ... and are renormalised before the 32-bit epoch wraps.
// A Get of round ep reads st[ep & 1]:  0 or epoch > ep -> absent (created by a later round);
// epoch == ep -> the round's last writer (its record); epoch < ep -> present, value in `val`.
struct __attribute__((aligned(32))) Slot {
    u64 key;  // EMPTY_KEY when free
    u64 val;
    u64 st[2];
};
__host__ __device__ __forceinline__ u64 stamp_make(u32 epoch, u64 i1) { return ((u64)epoch << 32) | i1; }
__host__ __device__ __forceinline__ u32 stamp_epoch(u64 st) { return (u32)(st >> 32); }
constexpr u64 STAMP_PRESENT = 1ull << 32;  // epoch 1, no writer: present since before the replay rounds

// One replica-wide control block in HBM.
struct __attribute__((aligned(64))) DevCtl {
    u32 err;          // latched ERR_* bits
    u32 sp_claim;     // hashmap: the key EMPTY_KEY has been inserted (its slot is `sp`)
    u64 nkeys;        // hashmap: keys inserted directly (prefill)
    long long depth;  // stack: current length
    u64 counter;      // scratch counter (dump compaction)
    u64 nkeys_total;  // hashmap: nkeys + keys created by replay rounds (hm_count)
    long long depth0;      // stack: length after the last chunk of buffer parity 0 (stack.hip)
    long long depth_next;  // stack: ... of parity 1; a chunk starts from the other parity's slot
    u64 pad;
    Slot sp;          // hashmap: side slot of the key EMPTY_KEY (val, stamps; key unused)
};

__device__ __forceinline__ u64 ld_relaxed(const u64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32 ld_relaxed32(const u32* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Test-only stall (NRG_KNOB_STALL): odd waves sleep ~30 us at a point where the workgroup's
// waves next reuse LDS another wave may still read, so a missing barrier shows up as a wrong
// result instead of a rare timing accident.
__device__ __forceinline__ void test_stall(u32 on, int wave) {
    if (on && (wave & 1))
        for (int i = 0; i < 32; i++) __builtin_amdgcn_s_sleep(127);
}

// Wave-wide (64-lane) inclusive scan helpers.
__device__ __forceinline__ u32 lane_id() { return threadIdx.x & 63; }

}  // namespace nrg
