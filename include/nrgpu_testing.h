/*
 * nrgpu_testing.h — test hooks into libnrgpu.so's internal kernels (not part of the
 * drop-in ABI). Used by tests/ to unit-test the building blocks of the replay pipelines
 * against numpy: the stable LSD radix sort and the max-scan of the synthetic replay.
 * All pointers are device pointers; work is ordered on the context's stream and
 * completed before return.
 */
#ifndef NRGPU_TESTING_H
#define NRGPU_TESTING_H
#include "nrgpu.h"
#ifdef __cplusplus
extern "C" {
#endif
/* stable sort of n (key, val) pairs by the low key_bits of key; d_vals may be NULL (0..n-1) */
int nrg_test_sort_pairs(nrg_ctx* ctx, const uint32_t* d_keys, const uint32_t* d_vals, uint64_t n,
                        int key_bits, uint32_t* d_out_keys, uint32_t* d_out_vals);
/* M[p] = max{q <= p : q == 0 || keys[q-1] != keys[q] || (vals[q] & 0x80000000)} */
int nrg_test_maxscan(nrg_ctx* ctx, const uint32_t* d_keys, const uint32_t* d_vals, uint64_t n,
                     uint32_t* d_out);
/* copy the record stored at PHYSICAL ring position `phys` (< log size) to host memory `out`
 * (rec bytes per ds kind); syncs first. Lets tests check Log::index (nr/src/log.rs:528-530)
 * against what the replica's HBM ring actually holds. */
int nrg_test_ring_read(nrg_ctx* ctx, uint64_t phys, void* out);
/* diagnostic phase timestamps of the last replay (contexts opened with NRG_EXP & 2) */
int nrg_test_debug_read(nrg_ctx* ctx, uint64_t* out, uint64_t words);
// Hashmap: 1 when the sampled key skew sends rounds to the bucket elector (hashmap.hip
// skew_sample), 0 when they take the one-launch stamp rounds.
int nrg_test_hm_skewed(nrg_ctx* ctx, int* out);
#ifdef __cplusplus
}
#endif
#endif
