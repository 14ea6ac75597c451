/*
 * nr_oracle.h — CPU restatement of node-replication's data-plane semantics.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (node-replication_amd/) links, loads or
 * calls this code. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * it, as the checker / the timed CPU baseline.
 *
 * The reference (junghan0611/node-replication) is Rust and cannot be built here (no Rust
 * toolchain). This file restates, sequentially, what one `nr` replica
 * computes when it replays the log:
 *   - NrHashMap        benches/hashmap.rs:77-122, nr/examples/hashmap.rs:12-51
 *                      (Put -> HashMap::insert returning the previous value; Get -> get)
 *   - Stack            benches/stack.rs:36-84, nr/tests/stack.rs:31-96
 *   - Synthetic        benches/synthetic.rs:60-195 (AbstractDataStructure::new(n,20,5,2,1))
 *   - op generators    benches/hashmap.rs:131-162, benches/stack.rs:87-102 with a SEEDED
 *                      splitmix64 stream in place of the reference's unseeded thread_rng.
 * Parity is pinned by the reference's own deterministic tests (ported in tests/) and by the
 * std::collections::HashMap / Vec contracts, checked against an independent Python
 * dict/list model and committed golden fixtures (tests/golden/).
 */
#ifndef NR_ORACLE_H
#define NR_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- seeded streams (identical definitions on the GPU side) --------------------- */
uint64_t orc_mix64(uint64_t z);
uint64_t orc_sm64_at(uint64_t seed, uint64_t i);
void orc_gen_raw(uint64_t* out, uint64_t n, uint64_t seed);
void orc_gen_uniform(uint64_t* out, uint64_t n, uint64_t seed, uint64_t span);
/* Zipf(theta) over ranks 1..N (Gray et al. SIGMOD'94 generator). scramble=0: key=rank-1;
 * scramble=1: key = mix64(rank) % N. Returns keys in out. */
void orc_gen_zipf(uint64_t* out, uint64_t n, uint64_t seed, uint64_t N, double theta, int scramble);
/* Mixed hashmap op stream as benches/hashmap.rs:131-162: op i is a Put iff i%100 < wr,
 * then a seeded Fisher-Yates shuffle. is_put[i] in {0,1}. */
void orc_gen_hashmap_ops(uint8_t* is_put, uint64_t* keys, uint64_t* vals, uint64_t n,
                         uint64_t seed, uint64_t span, uint32_t write_ratio);
/* Stack ops as benches/stack.rs:87-102: op = raw%2 (0 Pop, 1 Push), value = raw>>32. */
void orc_gen_stack_ops(uint32_t* vals, uint32_t* ops, uint64_t n, uint64_t seed);

/* ---- NrHashMap ----------------------------------------------------------------- */
typedef struct orc_hm orc_hm;
orc_hm* orc_hm_new(uint64_t initial_capacity);
void orc_hm_free(orc_hm* m);
/* HashMap::insert: returns 1 and *prev if the key existed. */
int orc_hm_insert(orc_hm* m, uint64_t key, uint64_t val, uint64_t* prev);
int orc_hm_get(const orc_hm* m, uint64_t key, uint64_t* val);
uint64_t orc_hm_len(const orc_hm* m);
/* keys 0..n-1 -> k + off  (NrHashMap::default, benches/hashmap.rs:91-100) */
void orc_hm_prefill_range(orc_hm* m, uint64_t n, uint64_t off);
/* Log::exec over W Put records in log order (interleaved keys/vals). prev/prev_found may
 * be NULL. */
void orc_hm_replay(orc_hm* m, const uint64_t* puts_kv, uint64_t W, uint64_t* prev,
                   uint8_t* prev_found);
void orc_hm_get_batch(const orc_hm* m, const uint64_t* keys, uint64_t n, uint64_t* vals,
                      uint8_t* found);
/* Mixed sequential stream (one nr thread issuing execute_mut/execute in order). */
void orc_hm_run_mixed(orc_hm* m, const uint8_t* is_put, const uint64_t* keys,
                      const uint64_t* vals, uint64_t n, uint64_t* resp, uint8_t* some);
/* Dump all pairs sorted by key; returns count (buffers must hold len). */
uint64_t orc_hm_dump_sorted(const orc_hm* m, uint64_t* keys, uint64_t* vals);
/* Same digest as nrg_hashmap_digest: {count, sum, xor} of mix64(k ^ mix64(v)). */
void orc_hm_digest(const orc_hm* m, uint64_t out[3]);

/* ---- Stack --------------------------------------------------------------------- */
typedef struct orc_stack orc_stack;
orc_stack* orc_stack_new(const uint32_t* init, uint64_t n);
void orc_stack_free(orc_stack* s);
/* Replay n ops (op 1 = Push(val), 0 = Pop). resp/some may be NULL. push_resp selects
 * Push -> Some(v) (1) or None (0). */
void orc_stack_replay(orc_stack* s, const uint32_t* vals, const uint32_t* ops, uint64_t n,
                      int push_resp, uint32_t* resp, uint8_t* some);
uint64_t orc_stack_len(const orc_stack* s);
uint64_t orc_stack_dump(const orc_stack* s, uint32_t* out);
int orc_stack_peek(const orc_stack* s, uint32_t* val);

/* ---- AbstractDataStructure ----------------------------------------------------- */
typedef struct orc_synth orc_synth;
orc_synth* orc_synth_new(uint64_t n, uint64_t cold_reads, uint64_t cold_writes,
                         uint64_t hot_reads, uint64_t hot_writes);
void orc_synth_free(orc_synth* s);
/* ops: 4 u64 per op {tid, r1, r2, op} with op 0 = WriteOnly, 1 = ReadWrite. */
void orc_synth_replay(orc_synth* s, const uint64_t* ops, uint64_t n, uint64_t* resp);
/* reads: 3 u64 per op {tid, r1, r2} -> ReadOnly. */
void orc_synth_read(const orc_synth* s, const uint64_t* ops, uint64_t n, uint64_t* sums);
uint64_t orc_synth_dump(const orc_synth* s, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif
