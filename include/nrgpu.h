/*
 * nrgpu.h — C ABI of the MI355X-native node-replication (NR) log-replay path.
 *
 * One `nrg_ctx` is one NR *replica* living on one GPU: it owns the replicated data
 * structure in HBM (NrHashMap / Stack / AbstractDataStructure), its copy of the shared
 * operation log (an HBM ring of fixed-width records tagged by logical log index), the
 * per-replica replay epoch (`ltail`), scratch for the replay kernels, and a HIP stream.
 *
 * Each entry point replaces one piece of the reference's Rust API (paths relative to the
 * reference checkout `junghan0611/node-replication`):
 *
 *   nrg_open / nrg_close          Replica::new + Log::new            nr/src/replica.rs:184-232, nr/src/log.rs:179-242
 *   nrg_log_append*               Log::append                        nr/src/log.rs:343-427
 *   nrg_log_exec*                 Log::exec -> Dispatch::dispatch_mut nr/src/log.rs:473-524, nr/src/replica.rs:572-581
 *   nrg_log_state                 head/tail/ctail/ltails            nr/src/log.rs:88-131, :671-679
 *   nrg_log_reset                 Log::reset                         nr/src/log.rs:593-611
 *   nrg_hashmap_get*              Replica::execute -> dispatch       nr/src/replica.rs:404-410,483-497; benches/hashmap.rs:107-111
 *   nrg_hashmap_round_async       Replica::combine (append+exec) + read batch   nr/src/replica.rs:544-595
 *   nrg_hashmap_prefill*          NrHashMap::default                 benches/hashmap.rs:91-100
 *   nrg_hashmap_dump / digest     Replica::verify(closure)           nr/src/replica.rs:443-467
 *   nrg_stack_*                   Stack Dispatch                     benches/stack.rs:36-84, nr/tests/stack.rs:31-96
 *   nrg_synth_*                   AbstractDataStructure Dispatch     benches/synthetic.rs:60-195
 *   nrg_group_*                   the shared Log across NUMA nodes   nr/src/log.rs:494-511 (every replica
 *                                 (RCCL all-gather of write segments) replays every entry), :473-524
 *   nrg_key_owner, nrg_hashmap_partition*, nrg_group_partitioned_round
 *                                 cnr's key-partitioned logs         cnr/src/lib.rs:134-167 (LogMapper::hash),
 *                                 (one log per GPU, RCCL send/recv)  cnr/src/replica.rs:430-445, :673-736
 *
 * Conventions
 *   - Every function returns NRG_OK (0) or a negative NRG_E_* code. Nothing throws or aborts.
 *   - A context is NOT thread-safe; callers serialise calls on one context, exactly as the
 *     combiner lock serialises Log::exec on one replica (nr/src/replica.rs:508-540).
 *     Distinct contexts (one per GPU) may be driven from distinct threads.
 *   - `*_async` functions take DEVICE pointers and are ordered on the context's stream
 *     (see nrg_set_stream); buffers are borrowed until the stream reaches that point.
 *     Device-side failures (table full, probe overrun) are latched and reported by the
 *     next nrg_sync / synchronous call.
 *   - Functions without `_async` take HOST pointers and return after the work completed.
 *   - Records in the log are fixed-width structs (below); the log index of a record is its
 *     position in the global total order of writes, exactly as in the reference.
 *   - Responses are produced only for a caller-chosen window [resp_lo, resp_hi) of log
 *     indices: in NR only the replica that appended an op receives its response
 *     (nr/src/replica.rs:576-578), and a replica's own ops form contiguous windows.
 */
#ifndef NRGPU_H
#define NRGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ---------------------------------------------------------------- */
#define NRG_OK 0
#define NRG_E_INVAL (-1)        /* bad argument / wrong data-structure kind              */
#define NRG_E_HIP (-2)          /* a HIP runtime call failed                             */
#define NRG_E_TABLE_FULL (-3)   /* hash table probe exhausted (reference would grow)     */
#define NRG_E_RING_FULL (-4)    /* log ring cannot hold the append even after GC         */
#define NRG_E_NOMEM (-5)        /* device allocation failed                              */
#define NRG_E_NOT_SYNCED (-6)   /* read requested while ltail < tail (sync first)        */
#define NRG_E_CAPACITY (-7)     /* batch exceeds configured max / stack capacity         */
#define NRG_E_NODEV (-8)        /* no HIP device with that ordinal                       */

/* ---- data-structure kinds --------------------------------------------------------- */
#define NRG_DS_HASHMAP 1u   /* NrHashMap: u64 -> u64, Put/Get                       */
#define NRG_DS_STACK 2u     /* Stack: Vec<u32>, Push/Pop, Peek                      */
#define NRG_DS_SYNTHETIC 3u /* AbstractDataStructure(n, 20, 5, 2, 1)                */

/* ---- log record layouts (one WriteOperation each) --------------------------------- */
/* NrHashMap WriteOperation::Put(key, val)               benches/hashmap.rs:52-56       */
typedef struct {
    uint64_t key;
    uint64_t val;
} nrg_put;

/* Stack WriteOperation: op = NRG_STACK_PUSH (val used) or NRG_STACK_POP  benches/stack.rs:22-28 */
#define NRG_STACK_POP 0u
#define NRG_STACK_PUSH 1u
typedef struct {
    uint32_t val;
    uint32_t op;
} nrg_stack_op;

/* Synthetic WriteOperation: WriteOnly/ReadWrite(tid, rnd1, rnd2)  benches/synthetic.rs:33-39 */
#define NRG_SYNTH_WRITE_ONLY 0u
#define NRG_SYNTH_READ_WRITE 1u
typedef struct {
    uint64_t tid;
    uint64_t r1;
    uint64_t r2;
    uint64_t op;
} nrg_synth_op;

/* Synthetic ReadOperation::ReadOnly(tid, rnd1, rnd2)     benches/synthetic.rs:28-31       */
typedef struct {
    uint64_t tid;
    uint64_t r1;
    uint64_t r2;
} nrg_synth_rd;

/* ---- configuration ------------------------------------------------------------------ */
typedef struct {
    uint32_t ds_kind;         /* NRG_DS_*                                                  */
    uint32_t log2_slots;      /* hashmap: table has 2^log2_slots 32-B slots {key, value, two
                                 round stamps} (default 26: 2 GiB of HBM; < 2^30 slots)       */
    uint64_t log_bytes;       /* Log::new(bytes): ring entries = bytes/64 rounded as in the
                                 reference (min 2*GC_FROM_HEAD, power of two). 0 = 32 MiB   */
    uint64_t max_batch;       /* largest number of log records replayed per kernel pass;
                                 larger exec ranges are replayed in order, in chunks
                                 (< 2^30; stack: <= 2^24)                                   */
    uint64_t max_reads;       /* largest read batch per call                               */
    uint64_t stack_capacity;  /* stack: maximum number of elements                          */
    uint64_t synth_n;         /* synthetic: number of words (default 200000)               */
    uint32_t synth_cold_reads, synth_cold_writes, synth_hot_reads, synth_hot_writes; /* 20,5,2,1 */
    uint32_t stack_push_resp; /* 0: Push -> None (benches/stack.rs:77-80, nr/examples/stack.rs:70-73)
                                 1: Push -> Some(v) (nr/tests/stack.rs:89-92)               */
    uint32_t replica_id;      /* this replica's id (Log::register, ids start at 1)         */
    uint32_t pipeline;        /* opt-in (default 0). 0: every output of an *_async call is
                                 ordered on the context's stream. 1: the tail of a replay round
                                 rides in the next round's launch -- hashmap: the apply + reads;
                                 stack: the Pops answered from earlier tiles and the commit;
                                 synthetic: the per-op sums and the hot-word fold. Those outputs
                                 (and the buffers they read) are complete only after nrg_join(),
                                 the next round call on this context (an empty one included), or
                                 nrg_sync(); give back-to-back rounds distinct response buffers.
                                 Synchronous calls are unaffected (their outputs are complete on
                                 return). */
} nrg_config;

/* Fill `cfg` with the defaults of the reference benches for `ds_kind`. */
void nrg_config_default(nrg_config* cfg, uint32_t ds_kind);

typedef struct nrg_ctx nrg_ctx;

/* Replica::new(&log): allocate the replica (data structure + ring + scratch) on device
 * `hip_device`; the data structure starts empty (NrHashMap/Stack) or initialised to
 * storage[i] = i (synthetic, benches/synthetic.rs:97-100). */
int nrg_open(int hip_device, const nrg_config* cfg, nrg_ctx** out);
int nrg_close(nrg_ctx* ctx);

/* Use `hip_stream` (a hipStream_t; NULL is the device's null stream, as in HIP) for all
 * further work on this context. A new context works on a non-blocking stream of its own,
 * returned by nrg_own_stream. Work on a caller's stream is ordered with the caller's other
 * work on it; the own stream is NOT ordered with the null stream. */
int nrg_set_stream(nrg_ctx* ctx, void* hip_stream);
void* nrg_get_stream(nrg_ctx* ctx);
void* nrg_own_stream(nrg_ctx* ctx);

/* Replica::sync analogue: wait for all queued work; report latched device errors. */
int nrg_sync(nrg_ctx* ctx);
/* Order outstanding side-stream reads (config.pipeline = 1) on the context's stream without
 * blocking the host; a no-op when nothing is outstanding. */
int nrg_join(nrg_ctx* ctx);

const char* nrg_strerror(int code);
/* Library build identifier ("nrgpu <version> gfx950"). */
const char* nrg_version(void);
/* Number of visible HIP devices (0 on a host without GPUs; never fails). */
int nrg_device_count(void);

/* ---- Log ------------------------------------------------------------------------------ */
typedef struct {
    uint64_t size;   /* ring entries (power of two)                        */
    uint64_t head;   /* oldest live logical index (GC boundary)            */
    uint64_t tail;   /* next logical index to be appended                  */
    uint64_t ctail;  /* completed tail (max replayed tail)                 */
    uint64_t ltail;  /* this replica's replay epoch (ltails[idx-1])        */
    uint32_t replica_id;
    uint32_t ds_kind;
} nrg_log_info;

/* Log::append(ops, idx): append `n` host records (layout per ds kind) with origin replica
 * `origin`; returns the logical index of the first record. When fewer than GC_FROM_HEAD
 * entries would remain, the replica first replays what it has not replayed (as append's
 * GC path calls exec, nr/src/log.rs:364-387) and advances head to its ltail. */
int nrg_log_append(nrg_ctx* ctx, const void* recs, uint64_t n, uint32_t origin, uint64_t* first_idx);
/* Same, with `d_recs` a device pointer (stream ordered). */
int nrg_log_append_async(nrg_ctx* ctx, const void* d_recs, uint64_t n, uint32_t origin,
                         uint64_t* first_idx);
/* Append `nseg` device segments (e.g. the output of an all-gather of per-GPU write
 * segments): segment s starts at d_base + s*seg_stride records, holds lens[s] records and
 * has origin origins[s]. Segments are appended in order s = 0..nseg-1, which is the global
 * log order of the round. `first_idx[s]` receives each segment's first log index. */
int nrg_log_append_segments_async(nrg_ctx* ctx, const void* d_base, uint32_t nseg,
                                  uint64_t seg_stride, const uint64_t* lens,
                                  const uint32_t* origins, uint64_t* first_idx);

/* Log::exec(idx, dispatch_mut): replay [ltail, tail) into the replica in log order.
 * Responses for log indices in [resp_lo, resp_hi) are written densely:
 *   hashmap  : resp[u64] = previous value, some[u8] = 1 iff the key existed
 *              (HashMap::insert's return, nr/examples/hashmap.rs:46-50)
 *   stack    : resp[u32] = popped (or pushed, if stack_push_resp) value, some[u8]
 *   synthetic: resp[u64] = ReadWrite sum (WriteOnly -> 0), some = 1
 * `resp`/`some` may be NULL (no responses wanted, as benches/hashmap.rs:114-119 returns
 * Ok(None)); the hashmap then skips the previous-value pipeline entirely. */
int nrg_log_exec(nrg_ctx* ctx, uint64_t resp_lo, uint64_t resp_hi, void* resp, uint8_t* some);
int nrg_log_exec_async(nrg_ctx* ctx, uint64_t resp_lo, uint64_t resp_hi, void* d_resp,
                       uint8_t* d_some);

int nrg_log_state(const nrg_ctx* ctx, nrg_log_info* out);
/* Log::reset: head = tail = ctail = ltail = 0; the data structure is left untouched. */
int nrg_log_reset(nrg_ctx* ctx);

/* ---- NrHashMap ----------------------------------------------------------------------- */
/* Dispatch::dispatch(Get(k)) for a batch, after sync-to-tail (NRG_E_NOT_SYNCED if the
 * replica has unreplayed log entries): vals[i] = value or 0, found[i] = 1 iff present. */
int nrg_hashmap_get(nrg_ctx* ctx, const uint64_t* keys, uint64_t n, uint64_t* vals, uint8_t* found);
int nrg_hashmap_get_async(nrg_ctx* ctx, const uint64_t* d_keys, uint64_t n, uint64_t* d_vals,
                          uint8_t* d_found);

/* Replica::combine for a single-GPU replica, fused: append the W device records `d_puts`
 * with origin `origin`, replay everything up to the new tail, then answer the R reads
 * `d_get_keys` against the post-replay state. Previous-value responses for the appended
 * puts go to d_prev/d_prev_found if non-NULL. */
int nrg_hashmap_round_async(nrg_ctx* ctx, const nrg_put* d_puts, uint64_t W, uint32_t origin,
                            const uint64_t* d_get_keys, uint64_t R, uint64_t* d_get_vals,
                            uint8_t* d_get_found, uint64_t* d_prev, uint8_t* d_prev_found);

/* Multi-GPU round on one replica: the write segments of every replica (e.g. the output of
 * an RCCL all-gather, segment s at d_base + s*seg_stride records, lens[s] records, origin
 * origins[s]) are appended in order s = 0..nseg-1 (the round's global log order), the log is
 * replayed, and the R local reads are answered against the post-round state. Previous-value
 * responses are produced for segment `resp_seg` (this replica's own writes) if d_prev is
 * non-NULL. When every segment but the last is full (lens[s] == seg_stride) the gathered
 * buffer is replayed in place and the log copy is written by the replay itself. */
int nrg_hashmap_round_segments_async(nrg_ctx* ctx, const nrg_put* d_base, uint32_t nseg,
                                     uint64_t seg_stride, const uint64_t* lens,
                                     const uint32_t* origins, uint32_t resp_seg,
                                     const uint64_t* d_get_keys, uint64_t R, uint64_t* d_get_vals,
                                     uint8_t* d_get_found, uint64_t* d_prev, uint8_t* d_prev_found);

/* NrHashMap::default(): insert (keys[i], vals[i]) directly (no log traffic). */
int nrg_hashmap_prefill(nrg_ctx* ctx, const uint64_t* keys, const uint64_t* vals, uint64_t n);
/* Generated on device: keys k = 0..n-1 -> k + val_offset (benches/hashmap.rs:91-100 uses
 * n = INITIAL_CAPACITY, val_offset = 1). */
int nrg_hashmap_prefill_range(nrg_ctx* ctx, uint64_t n, uint64_t val_offset);
int nrg_hashmap_size(nrg_ctx* ctx, uint64_t* n);
/* Copy out every (key, value) pair (unordered). `*n` receives the number of pairs; if it
 * exceeds `cap`, nothing is copied and NRG_E_CAPACITY is returned. */
int nrg_hashmap_dump(nrg_ctx* ctx, uint64_t* keys, uint64_t* vals, uint64_t cap, uint64_t* n);
/* Order-independent digest of the contents: count, sum and xor of mix64(k ^ mix64(v)). */
int nrg_hashmap_digest(nrg_ctx* ctx, uint64_t out[3]);

/* ---- Flat combining on the host ---------------------------------------------------------- */
/* Replica's flat combiner for many client threads (nr/src/context.rs:88-194,
 * nr/src/replica.rs:345-356, 404-433, 483-497, 508-595), for any of the three data structures:
 * each registered thread posts up to 32 ops (MAX_PENDING_OPS) per call into the open batch and
 * parks; the combiner's own thread seals the batch into ONE GPU round of `ctx` (its writes
 * appended and replayed in batch order, then its reads answered against the post-round state)
 * without waiting for the GPU, so the next batch fills while a round runs (a second round is put
 * in flight only for a batch of 512 ops or more unless NRG_KNOB_COMB_DEPTH fixes the depth).
 * Batches live in mapped pinned host memory that the round's kernels read and write directly.
 * Calls on one token are synchronous and must come from one thread at a time (a second call on
 * a token whose call is still in progress returns NRG_E_INVAL); while a combiner
 * is open, `ctx` is driven only through it, and no thread may be inside a call when it is closed.
 * Needs max_threads * 32 <= max_batch (and <= max_reads for the hashmap). */
typedef struct nrg_combiner nrg_combiner;
int nrg_combiner_open(nrg_ctx* ctx, uint32_t max_threads, nrg_combiner** out);
int nrg_combiner_close(nrg_combiner* comb);
/* Replica::register: a token 0..max_threads-1, or NRG_E_CAPACITY. */
int nrg_combiner_register(nrg_combiner* comb, uint32_t* token);
/* Replica::execute_mut for n <= 32 log records of the replica's kind (nrg_put / nrg_stack_op /
 * nrg_synth_op): resp[i] / some[i] as nrg_log_exec gives them (u64 previous value, u32 popped
 * value, u64 sum). */
int nrg_combiner_execute_mut(nrg_combiner* comb, uint32_t token, const void* recs, uint32_t n, void* resp,
                             uint8_t* some);
/* Replica::execute for n <= 32 reads: hashmap Get (u64 keys -> u64 value, found), stack Peek
 * (`reads` unused -> u32 top, some), synthetic ReadOnly (nrg_synth_rd -> u64 sum, some = 1). */
int nrg_combiner_execute(nrg_combiner* comb, uint32_t token, const void* reads, uint32_t n, void* resp,
                         uint8_t* some);
/* NrHashMap conveniences: Put(keys[i], vals[i]) -> prev[i]/some[i] = HashMap::insert's previous
 * value; Get(keys[i]) -> vals[i]/found[i]. */
int nrg_combiner_put(nrg_combiner* comb, uint32_t token, const uint64_t* keys, const uint64_t* vals, uint32_t n,
                     uint64_t* prev, uint8_t* some);
int nrg_combiner_get(nrg_combiner* comb, uint32_t token, const uint64_t* keys, uint32_t n, uint64_t* vals,
                     uint8_t* found);
/* GPU rounds combined so far and the ops they carried. */
int nrg_combiner_stats(nrg_combiner* comb, uint64_t* rounds, uint64_t* ops);

/* ---- Stack --------------------------------------------------------------------------- */
/* Stack::default(): storage = vals[0..n) (bottom first). */
int nrg_stack_init(nrg_ctx* ctx, const uint32_t* vals, uint64_t n);
/* Replica::combine for one stack batch (nr/src/replica.rs:544-595): Log::append of the n ops
 * in d_ops (device) with `origin`, then Log::exec, fused into one replay pass that writes the
 * log copy itself. Pop responses for these ops (d_pop_vals[i], d_some_bits[i]; nullable) as
 * nrg_log_exec_async gives them. Same result as nrg_log_append_async + nrg_log_exec_async. */
int nrg_stack_round_async(nrg_ctx* ctx, const nrg_stack_op* d_ops, uint64_t n, uint32_t origin,
                          uint32_t* d_pop_vals, uint8_t* d_some_bits);
/* Dispatch::dispatch(Peek) after sync: top of stack. */
int nrg_stack_peek(nrg_ctx* ctx, uint32_t* val, uint8_t* some);
int nrg_stack_len(nrg_ctx* ctx, uint64_t* n);
int nrg_stack_dump(nrg_ctx* ctx, uint32_t* vals, uint64_t cap, uint64_t* n);

/* ---- AbstractDataStructure (synthetic) ------------------------------------------------ */
/* Dispatch::dispatch(ReadOnly(tid, r1, r2)) for a batch, after sync. */
/* Replica::combine for one batch of AbstractDataStructure write ops (device buffer): Log::append
 * fused into the replay's first pass, then Log::exec; sums (responses) for these ops as
 * nrg_log_exec_async gives them (nullable). Same result as append + exec. */
int nrg_synth_round_async(nrg_ctx* ctx, const nrg_synth_op* d_ops, uint64_t n, uint32_t origin,
                          uint64_t* d_resp, uint8_t* d_some);
int nrg_synth_read(nrg_ctx* ctx, const nrg_synth_rd* ops, uint64_t n, uint64_t* sums);
int nrg_synth_read_async(nrg_ctx* ctx, const nrg_synth_rd* d_ops, uint64_t n, uint64_t* d_sums);
int nrg_synth_dump(nrg_ctx* ctx, uint64_t* words, uint64_t cap, uint64_t* n);

/* ---- multi-GPU replica groups (RCCL over xGMI) --------------------------------------------
 * The reference shares ONE log between replicas through cache-coherent memory: every replica's
 * Log::exec reads every entry (nr/src/log.rs:494-511, :473-524). Across GPUs the write segments
 * of a round are all-gathered with RCCL (ncclAllGather, one communicator per GPU, over xGMI)
 * and every replica replays the identical global log W_0 || W_1 || ... || W_{n-1} (rank order);
 * reads stay on their GPU; write responses go to the origin replica only
 * (nr/src/replica.rs:576-578). The all-gather runs on a library-owned stream per GPU and the
 * gathered buffers rotate, so the all-gather of round e+1 overlaps the replay of round e.
 * RCCL is loaded at the first group call (librccl.so.1, the process's own copy if one is
 * already loaded); without it these calls return NRG_E_COMM. */
#define NRG_E_COMM (-9)          /* RCCL unavailable or a collective failed               */
#define NRG_E_TIMEOUT (-10)      /* a peer rank did not take part in a collective before the
                                    group's deadline (nrg_group_set_timeout)                 */
#define NRG_GROUP_DEFAULT_TIMEOUT_MS 300000u
#define NRG_GROUP_ID_BYTES 128   /* ncclUniqueId                                           */

typedef struct nrg_group nrg_group;

/* A group member's part of one round (all pointers are device pointers on its GPU). */
typedef struct {
    const void* recs;          /* this replica's write segment (log records, issue order)       */
    uint64_t n;                /* records in it                                                  */
    void* resp;                /* nullable: responses to its own writes (as nrg_log_exec_async)  */
    uint8_t* some;
    const uint64_t* get_keys;  /* hashmap: reads answered against the post-round state          */
    uint64_t n_gets;
    uint64_t* get_vals;
    uint8_t* get_found;
} nrg_round;

/* ncclGetUniqueId: one process creates the id and ships it to the others (any side channel). */
int nrg_group_unique_id(uint8_t id[NRG_GROUP_ID_BYTES]);
/* One process per GPU: `replica` joins group `id` as rank `rank` of `nranks` (ncclCommInitRank
 * on the replica's device). Replica ids should be rank + 1 (Log::register order). */
int nrg_group_join(nrg_ctx* replica, const uint8_t id[NRG_GROUP_ID_BYTES], int nranks, int rank,
                   nrg_group** out);
/* One process driving n GPUs: opens one replica per device (cfg, replica_id = i + 1) and one
 * communicator per device (ncclCommInitAll). The group owns these replicas. */
int nrg_group_open(const int* devices, int n, const nrg_config* cfg, nrg_group** out);
/* Closes the communicators and the group's buffers (and the replicas nrg_group_open opened). */
int nrg_group_close(nrg_group* g);
/* nranks: group size; nlocal: members driven by this process; rank0: rank of local member 0. */
int nrg_group_info(const nrg_group* g, int* nranks, int* nlocal, int* rank0);
nrg_ctx* nrg_group_replica(nrg_group* g, int member);
/* The all-gather of a member's segment waits for work queued on `hip_stream` when the round is
 * issued (default: the replica's own stream, which also orders it after the previous replay;
 * give the stream the inputs are produced on to let all-gathers run ahead of replays). */
int nrg_group_set_input_stream(nrg_group* g, int member, void* hip_stream);
/* One NR round on every local member: all-gather of the members' write segments (RCCL), then on
 * each replica Log::append of the gathered segments in rank order + Log::exec + its reads.
 * Appends of any length interleave, as in the reference (nr/src/log.rs:343-427): ranks may hold
 * different segment lengths, and every rank must learn all of them before the all-gather.
 *   seg_lens == NULL   the ranks exchange {n, local error} first (one 8-B-per-rank all-gather and
 *                      one host round trip); a rank with a bad segment makes the round return
 *                      NRG_E_INVAL on EVERY rank, before any data moves.
 *   seg_lens != NULL   seg_lens[r] = rank r's segment length; every rank must pass the same array.
 *                      The round stays stream ordered: a header {n, fingerprint of seg_lens}
 *                      travels with each segment and is compared on every rank's comm stream. A
 *                      rank whose n differs from seg_lens[rank] still takes part (with zeros) and
 *                      returns NRG_E_INVAL; any disagreement makes the next nrg_group_sync /
 *                      nrg_sync of every rank return NRG_E_INVAL. (Arrays whose longest segment
 *                      differs would give all-gathers of different sizes: RCCL cannot check that.)
 * A single-process group (nrg_group_open) takes its members' n (seg_lens, if given, must agree).
 * Stream ordered; borrows buffers until the replica stream passes this round (config.pipeline =
 * 1: until nrg_join / the next call). */
int nrg_group_round_async(nrg_group* g, const nrg_round* rounds, const uint64_t* seg_lens);
/* Wait for all queued group work and report latched device errors of every local replica. */
int nrg_group_sync(nrg_group* g);
/* Deadline of every wait on the peer ranks (default NRG_GROUP_DEFAULT_TIMEOUT_MS): the host round
 * trips of the length / count exchanges, buffer regrowth and nrg_group_sync. A rank whose peers do
 * not post their part of a collective in time gets NRG_E_TIMEOUT instead of hanging (its
 * communicators are aborted, so the group can still be closed). Failures that leave the ranks'
 * replicas different -- a timeout, a failed collective, ranks that disagreed on seg_lens -- are
 * sticky: every later round or sync of the group returns the same code; close the group.
 * (Like RCCL, a process blocked inside ncclCommInitRank or ncclGroupEnd itself -- before the
 * stream waits -- is not bounded here; bench.py keeps a whole-process watchdog for that.) */
int nrg_group_set_timeout(nrg_group* g, uint32_t ms);
/* The sticky failure's description ("nrg_group rank R of N, round E: ..."), "" if none. */
const char* nrg_group_last_error(const nrg_group* g);

/* ---- cnr-style key-partitioned NrHashMap ---------------------------------
 * cnr maps each operation to one of several logs with LogMapper::hash() (cnr/src/lib.rs:134-167);
 * the operations of one key share a log, so the logs replay independently
 * (cnr/src/replica.rs:430-445 hash -> log, :673-736 combine(hashidx)). Across GPUs, partition p's
 * log lives on GPU p, which holds only the keys it owns (no full replication): a round's Puts and
 * Gets travel to their owners, each owner replays the Puts it received in rank order -- for every
 * key the same order as the NR global log W_0 || W_1 || ... -- and answers the Gets it received,
 * and answers and previous values travel back in the caller's order. The answers are identical
 * to NR's; the replicas are not (each holds one partition). */
#define NRG_MAX_PARTS 64
/* Owner partition of a key: (low 32 bits of splitmix64(key)) * parts >> 32. */
uint32_t nrg_key_owner(uint64_t key, uint32_t parts);
/* Stable partition of W Puts and R Get keys by owner (device buffers, the replica's stream):
 * puts_out / keys_out hold them grouped by owner, each group in issue order; put_pos[i] / get_pos[i]
 * = where record i went; counts[p] = Puts of owner p, counts[parts + p] = Gets of owner p (u64).
 * W, R < 2^32. */
int nrg_hashmap_partition_async(nrg_ctx* ctx, const nrg_put* d_puts, uint64_t W, const uint64_t* d_keys, uint64_t R,
                                uint32_t parts, nrg_put* d_puts_out, uint32_t* d_put_pos, uint64_t* d_keys_out,
                                uint32_t* d_get_pos, uint64_t* d_counts);
/* dst[i] = src[pos[i]] (u64 and/or u8 arrays; either pair may be NULL): answers back in order. */
int nrg_route_back_async(nrg_ctx* ctx, const uint64_t* d_src, const uint8_t* d_src8, const uint32_t* d_pos, uint64_t n,
                         uint64_t* d_dst, uint8_t* d_dst8);
/* NrHashMap::default restricted to a partition: keys k < n with nrg_key_owner(k, parts) == part. */
int nrg_hashmap_prefill_partition(nrg_ctx* ctx, uint64_t n, uint64_t off, uint32_t part, uint32_t parts);
/* One partitioned round on every local member (group of hashmap replicas, one partition each,
 * rank = partition): rounds[i].recs / n = the member's Puts (nrg_put), get_keys / n_gets its Gets;
 * get_vals / get_found and (nullable) resp / some = the Gets' answers and the Puts' previous values,
 * in the member's order. A round is one fused partition launch (owner regions, no global scan), an
 * all-gather of every rank's per-owner counts, ncclSend / ncclRecv of the Puts and Get keys to
 * their owners (a rank's own part stays on its GPU), the owner's replay, the answers back and one
 * route-back launch. Everything is on the replica's stream. Returns once the round is queued,
 * after one host round trip for the counts (nrg_group_sync waits for the rest). Fails with the
 * same code on every rank when any rank's part is bad, before any payload moves. */
int nrg_group_partitioned_round(nrg_group* g, const nrg_round* rounds);
/* The pipelined form, three calls deep: queues this round's partition and count exchange, moves
 * the previous round's Puts and Gets to their owners and replays it (its counts have landed by
 * then, so the host never waits on the GPU in steady state; its reads ride in the next round's
 * first launch), and sends the round before that back into its caller's order. The caller's
 * buffers of a round stay borrowed for the next two calls, or until nrg_group_partitioned_flush /
 * nrg_group_sync completes every posted round. A round dropped on an agreed error (a rank's bad
 * part) returns that error from the call that moved it (NRG_OK otherwise). A one-rank group
 * partitions on a library-owned side stream, after the work queued on the replica's stream and
 * beside the previous round's replay; the replica's stream waits for it before moving the round. */
int nrg_group_partitioned_round_async(nrg_group* g, const nrg_round* rounds);
/* Complete the round posted by nrg_group_partitioned_round_async, if any (its result). */
int nrg_group_partitioned_flush(nrg_group* g);

/* ---- device memory helpers (for callers without their own allocator) ----------------- */
int nrg_dev_alloc(nrg_ctx* ctx, uint64_t bytes, void** d_ptr);
int nrg_dev_free(nrg_ctx* ctx, void* d_ptr);
int nrg_memcpy_h2d(nrg_ctx* ctx, void* d_dst, const void* h_src, uint64_t bytes);
int nrg_memcpy_d2h(nrg_ctx* ctx, void* h_dst, const void* d_src, uint64_t bytes);

/* ---- synthetic workload generators (device side; identical streams to oracle/) -------- */
/* keys[i] = mulhi64(splitmix64_at(seed, i), span): uniform in [0, span). */
int nrg_gen_uniform_async(nrg_ctx* ctx, uint64_t* d_out, uint64_t n, uint64_t seed, uint64_t span);
/* raw splitmix64_at(seed, i) (values for Puts, push values after >> 32). */
int nrg_gen_raw_async(nrg_ctx* ctx, uint64_t* d_out, uint64_t n, uint64_t seed);
/* interleave: puts[i] = {keys[i], vals[i]} */
int nrg_gen_puts_async(nrg_ctx* ctx, nrg_put* d_out, const uint64_t* d_keys, const uint64_t* d_vals,
                       uint64_t n);
/* Zipf(theta) keys over [0, N) (Gray et al. SIGMOD'94 inverse CDF, ranks 1..N; scramble = 0:
 * key = rank-1 so hot keys are adjacent, 1: key = mix64(rank) % N). Statistically identical to
 * oracle/ orc_gen_zipf (device pow may differ from glibc's in the last ulp). theta != 1. */
int nrg_gen_zipf_async(nrg_ctx* ctx, uint64_t* d_out, uint64_t n, uint64_t seed, uint64_t N, double theta,
                       int scramble);
/* Stack ops as benches/stack.rs:87-102 with a seeded stream: r = splitmix64_at(seed, i),
 * op = r & 1 (1 = Push), val = r >> 32 (oracle/ orc_gen_stack_ops). */
int nrg_gen_stack_ops_async(nrg_ctx* ctx, nrg_stack_op* d_out, uint64_t n, uint64_t seed);

/* ---- timing: HIP events recorded around the dominant replay kernel -------------------- */
/* enable = 0: off; 1: every launch; n > 1: every n-th launch (sampling keeps the timed stream
 * unperturbed). The main replay kernel ("hm_round") is timed with start/stop events stamped
 * from its own dispatch (hipExtLaunchKernelGGL); multi-kernel pipelines ("hm_prev",
 * "st_replay", "sy_replay") with event records around them. nrg_kernel_time reads (timed
 * launches, their total milliseconds) after synchronising. */
int nrg_kernel_timing(nrg_ctx* ctx, int enable);
/* Restrict timing to one kernel name (NULL or "" = all). */
int nrg_kernel_timing_only(nrg_ctx* ctx, const char* which);
int nrg_kernel_time(nrg_ctx* ctx, const char* which, uint64_t* launches, double* total_ms);

#ifdef __cplusplus
}
#endif
#endif /* NRGPU_H */
