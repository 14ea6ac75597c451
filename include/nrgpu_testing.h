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
/* The hardware property the synthetic replay's rankings rest on (synthetic.hip): a
 * returning LDS add gives the lanes of one instruction that hit the same count their old values
 * in lane order. `blocks` (<= 65536) workgroups of 8 waves run `trials` (<= 4096) x 5 adds over `keys` (1..512)
 * counts; out[0] = lanes checked, out[1] = lanes out of lane order (0 expected). */
int nrg_test_lds_add_order(nrg_ctx* ctx, uint32_t keys, uint32_t trials, uint32_t blocks, uint64_t out[2]);
/* copy the record stored at PHYSICAL ring position `phys` (< log size) to host memory `out`
 * (rec bytes per ds kind); syncs first. Lets tests check Log::index (nr/src/log.rs:528-530)
 * against what the replica's HBM ring actually holds. */
int nrg_test_ring_read(nrg_ctx* ctx, uint64_t phys, void* out);
/* diagnostic phase timestamps of the last replay (a stack or synthetic context with NRG_KNOB_EXP
 * bit 2 set); NRG_E_INVAL when `words` exceeds the buffer */
int nrg_test_debug_read(nrg_ctx* ctx, uint64_t* out, uint64_t words);

/* Tuning and diagnostic knobs of an OPEN context. The product never reads the environment:
 * these setters are the only way to change them, so a stray variable in a caller's environment
 * cannot alter a replica. Each call first completes the context's queued work. */
#define NRG_KNOB_STAMP_MAX 1   /* hashmap: largest round replayed by one-launch stamp rounds
                                  (0: every round is a partition round; clamped to max_batch)     */
#define NRG_KNOB_SKEW_EVERY 2  /* hashmap: rounds between key-skew samples (>= 1, default 16)      */
#define NRG_KNOB_EPOCH_LIMIT 3 /* hashmap: renormalise stamps when the round epoch reaches this    */
#define NRG_KNOB_K1 4          /* hashmap: Puts per stamp-round index thread (0: by round size;
                                  1, 2 or 4)                                                      */
#define NRG_KNOB_EXP 6         /* diagnostic bits: phase timestamps (stack/synthetic 2); streamed
                                  outputs' stores: 0x40 stack and hashmap partition rounds plain
                                  instead of streaming, synthetic log copy streaming (0x80 touch
                                  records, 0x100 seen values, 0x200 responses); and stamp-round
                                  ablations that make RESULTS WRONG (0xF00000: no stamp atomics, no
                                  apply, no index, no reads) -- measurement only                   */
#define NRG_KNOB_SY_SORT 7     /* synthetic: 1 = sort-based replay instead of the bucket path      */
#define NRG_KNOB_PIPELINE 8    /* overrides nrg_config.pipeline                                    */
#define NRG_KNOB_SY_FUSED 18   /* synthetic bucket path: 1 (default) = one launch per round (chunk e's
                                  partition, e-1's bucket pass and e-2's sums side by side), 0 = two
                                  launches (partition + previous sums, then the bucket pass)       */
#define NRG_KNOB_COMB_SPIN 10   /* combiner (read by nrg_combiner_open): client threads that may spin
                                   while their round runs (default: max_threads - 1 when every
                                   client fits the CPUs the process may use, else 0 -- parked on
                                   futexes)                                                      */
#define NRG_KNOB_COMB_DEPTH 11  /* combiner: rounds in flight (1..4; default 2, the 2nd for >=512 ops) */
#define NRG_KNOB_PA_TPB 16      /* hashmap partition rounds without previous values: apply workgroup
                                   width 256 / 512 / 1024 over <= 1024 / 512 / 256 buckets (0 = 1024
                                   for rounds of >= 2^16 Puts, else 256: the default) */
#define NRG_KNOB_COMB_GATHER 15 /* combiner: us an idle combiner waits for as many posts as the last
                                   round carried before sealing (0..1000, default 20; 0 = seal at once) */
#define NRG_KNOB_COMB_SERVE 17 /* combiner (hashmap): 1 (default) = small rounds go to the resident round
                                   server (hm_serve_kernel) instead of a launch each; 0 = launched;
                                   v >= 2 (tests) = only rounds of at most v ops are served, so
                                   served and launched rounds alternate                          */
#define NRG_KNOB_SMALL_MAX 12   /* hashmap: rounds of at most this many Puts (<= 2048, and <= 8192
                                   Gets) replay in one one-workgroup launch (0: never; the
                                   combiner sets 2048 while it is open)                          */
#define NRG_KNOB_PART 13        /* hashmap: partition rounds (Puts grouped by home-slot bucket, one
                                   workgroup per bucket finds/claims and stores each key: no
                                   device atomic per Put) -- 1 (default) for previous values,
                                   skewed streams and rounds of >= 393216 Puts, 2 for every round,
                                   0 only where a stamp round cannot (previous values, skew,
                                   rounds above STAMP_MAX)                                        */
#define NRG_KNOB_STALL 14       /* tests: 1 = odd waves sleep ~30 us where a workgroup next reuses LDS
                                   another wave may still read (synthetic bucket pass, hashmap
                                   partition-round apply chunks, stack queries/table);
                                   2 (+1) = synthetic only, also drop the barrier that guards the
                                   bucket pass's tile map (diagnostic: results WRONG)            */
int nrg_test_set_knob(nrg_ctx* ctx, int knob, uint64_t value);
/* The combiner's round-server words and round counters: out = {posted, served, exited,
 * session, server running, rounds completed, rounds launched, open round}. */
int nrg_test_combiner_probe(nrg_combiner* m, uint64_t out[8]);
/* The combiner's round phases, summed over its rounds (ns): out = {rounds, batch open -> sealed,
 * sealed -> enqueued, enqueued -> completion seen}. */
int nrg_test_combiner_times(nrg_combiner* m, uint64_t out[4]);

/* Replica groups created after nrg_test_loopback_collectives(1) (nrg_group_open,
 * nrg_group_unique_id / nrg_group_join) use an in-process stand-in for RCCL instead of RCCL:
 * all-gathers and send/recv pairs become device copies on the members' streams, ordered with
 * events exactly where RCCL orders them. With it, nrg_group_open(devices = {0, 0, ...}) runs a
 * G-member group on one GPU from one thread, and G threads that each nrg_group_join the same
 * loopback id (one replica each, any device) form a G-rank group as G processes would: join
 * blocks until all ranks joined, and each collective blocks its thread until its peers posted
 * theirs. Tests check both shapes against the oracle. 0 switches back to RCCL for later groups. */
int nrg_test_loopback_collectives(int on);
// Hashmap: 1 when the sampled key skew sends rounds to partition rounds (hashmap.hip
// skew_sample), 0 when the round size decides.
int nrg_test_hm_skewed(nrg_ctx* ctx, int* out);
#ifdef __cplusplus
}
#endif
#endif
