/*
 * nr_oracle.c — sequential CPU restatement of node-replication's replay semantics.
 * TEST INFRASTRUCTURE ONLY (see nr_oracle.h): the checker for the HIP path, never shipped.
 */
#include "nr_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---- seeded streams ------------------------------------------------------------ */
/* splitmix64 finaliser; the GPU generator (node-replication_amd/csrc/common.hpp) uses the
 * identical constants so that device-generated workloads can be replayed here. */
uint64_t orc_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

uint64_t orc_sm64_at(uint64_t seed, uint64_t i) {
    return orc_mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ULL);
}

void orc_gen_raw(uint64_t* out, uint64_t n, uint64_t seed) {
    for (uint64_t i = 0; i < n; i++) out[i] = orc_sm64_at(seed, i);
}

static inline uint64_t mulhi64(uint64_t a, uint64_t b) {
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
}

/* uniform in [0, span): benches/hashmap.rs:150 `t_rng.gen_range(0, span)` */
void orc_gen_uniform(uint64_t* out, uint64_t n, uint64_t seed, uint64_t span) {
    for (uint64_t i = 0; i < n; i++) out[i] = mulhi64(orc_sm64_at(seed, i), span);
}

/* Gray, Sundaresan, Englert, Baclawski, Weinberger, "Quickly generating billion-record
 * synthetic databases", SIGMOD 1994 — the standard YCSB-style Zipf(theta) sampler. The
 * reference uses the `zipf` crate (exponent 1.03, benches/hashmap.rs:143-147); BASELINE asks
 * theta = 0.99, so the stream is our own and stated as such. */
void orc_gen_zipf(uint64_t* out, uint64_t n, uint64_t seed, uint64_t N, double theta, int scramble) {
    double zetan = 0.0;
    for (uint64_t i = 1; i <= N; i++) zetan += pow((double)i, -theta);
    double zeta2 = 1.0 + pow(2.0, -theta);
    double alpha = 1.0 / (1.0 - theta);
    double eta = (1.0 - pow(2.0 / (double)N, 1.0 - theta)) / (1.0 - zeta2 / zetan);
    double half_pow = 1.0 + pow(0.5, theta);
    for (uint64_t i = 0; i < n; i++) {
        double u = (double)(orc_sm64_at(seed, i) >> 11) * (1.0 / 9007199254740992.0);
        double uz = u * zetan;
        uint64_t rank;
        if (uz < 1.0)
            rank = 1;
        else if (uz < half_pow)
            rank = 2;
        else
            rank = 1 + (uint64_t)((double)N * pow(eta * u - eta + 1.0, alpha));
        if (rank > N) rank = N;
        out[i] = scramble ? orc_mix64(rank) % N : rank - 1;
    }
}

/* benches/hashmap.rs:131-162 with a seeded stream: key, value, then shuffle */
void orc_gen_hashmap_ops(uint8_t* is_put, uint64_t* keys, uint64_t* vals, uint64_t n,
                         uint64_t seed, uint64_t span, uint32_t write_ratio) {
    for (uint64_t i = 0; i < n; i++) {
        keys[i] = mulhi64(orc_sm64_at(seed, 2 * i), span);
        vals[i] = orc_sm64_at(seed, 2 * i + 1);
        is_put[i] = (i % 100) < write_ratio;
    }
    /* ops.shuffle(&mut t_rng): Fisher-Yates from the back */
    uint64_t sseed = orc_mix64(seed ^ 0x53485546464C45ULL);
    for (uint64_t i = n; i > 1; i--) {
        uint64_t j = mulhi64(orc_sm64_at(sseed, n - i), i);
        uint64_t k = i - 1;
        uint8_t tp = is_put[k]; is_put[k] = is_put[j]; is_put[j] = tp;
        uint64_t tk = keys[k]; keys[k] = keys[j]; keys[j] = tk;
        uint64_t tv = vals[k]; vals[k] = vals[j]; vals[j] = tv;
    }
}

/* benches/stack.rs:87-102: `op % 2` selects Pop (0) / Push (1); value from a second draw */
void orc_gen_stack_ops(uint32_t* vals, uint32_t* ops, uint64_t n, uint64_t seed) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t r = orc_sm64_at(seed, i);
        ops[i] = (uint32_t)(r & 1);
        vals[i] = (uint32_t)(r >> 32);
    }
}

/* ---- NrHashMap: std::collections::HashMap<u64,u64> contract --------------------- */
/* An open-addressing map with its OWN hash (wyhash-style fold, unrelated to the GPU's
 * splitmix slot hash) and growth at load 1/2, so that GPU/oracle agreement is not an
 * artefact of a shared table layout. */
struct orc_hm {
    uint64_t cap; /* power of two */
    uint64_t len;
    uint64_t* keys;
    uint64_t* vals;
    uint8_t* used;
};

static inline uint64_t orc_hm_hash(uint64_t k) {
    unsigned __int128 p = (unsigned __int128)(k ^ 0xa0761d6478bd642fULL) * 0xe7037ed1a0b428dbULL;
    return (uint64_t)p ^ (uint64_t)(p >> 64);
}

orc_hm* orc_hm_new(uint64_t initial_capacity) {
    orc_hm* m = (orc_hm*)calloc(1, sizeof(orc_hm));
    uint64_t cap = 16;
    while (cap < 2 * initial_capacity) cap <<= 1;
    m->cap = cap;
    m->keys = (uint64_t*)malloc(cap * sizeof(uint64_t));
    m->vals = (uint64_t*)malloc(cap * sizeof(uint64_t));
    m->used = (uint8_t*)calloc(cap, 1);
    return m;
}

void orc_hm_free(orc_hm* m) {
    if (!m) return;
    free(m->keys);
    free(m->vals);
    free(m->used);
    free(m);
}

static uint64_t orc_hm_find(const orc_hm* m, uint64_t key, int* present) {
    uint64_t mask = m->cap - 1, i = orc_hm_hash(key) & mask;
    for (;;) {
        if (!m->used[i]) { *present = 0; return i; }
        if (m->keys[i] == key) { *present = 1; return i; }
        i = (i + 1) & mask;
    }
}

static void orc_hm_grow(orc_hm* m) {
    orc_hm tmp = *m;
    m->cap = tmp.cap * 2;
    m->keys = (uint64_t*)malloc(m->cap * sizeof(uint64_t));
    m->vals = (uint64_t*)malloc(m->cap * sizeof(uint64_t));
    m->used = (uint8_t*)calloc(m->cap, 1);
    for (uint64_t i = 0; i < tmp.cap; i++) {
        if (!tmp.used[i]) continue;
        int p;
        uint64_t j = orc_hm_find(m, tmp.keys[i], &p);
        m->used[j] = 1;
        m->keys[j] = tmp.keys[i];
        m->vals[j] = tmp.vals[i];
    }
    free(tmp.keys);
    free(tmp.vals);
    free(tmp.used);
}

int orc_hm_insert(orc_hm* m, uint64_t key, uint64_t val, uint64_t* prev) {
    if (2 * (m->len + 1) > m->cap) orc_hm_grow(m);
    int present;
    uint64_t i = orc_hm_find(m, key, &present);
    if (present) {
        if (prev) *prev = m->vals[i];
        m->vals[i] = val;
        return 1;
    }
    m->used[i] = 1;
    m->keys[i] = key;
    m->vals[i] = val;
    m->len++;
    return 0;
}

int orc_hm_get(const orc_hm* m, uint64_t key, uint64_t* val) {
    int present;
    uint64_t i = orc_hm_find(m, key, &present);
    if (present && val) *val = m->vals[i];
    return present;
}

uint64_t orc_hm_len(const orc_hm* m) { return m->len; }

void orc_hm_prefill_range(orc_hm* m, uint64_t n, uint64_t off) {
    for (uint64_t k = 0; k < n; k++) orc_hm_insert(m, k, k + off, NULL);
}

/* Log::exec closure of Replica::combine (nr/src/replica.rs:572-581) applied to Puts in log
 * order: response = previous value (nr/examples/hashmap.rs:46-50). */
void orc_hm_replay(orc_hm* m, const uint64_t* puts_kv, uint64_t W, uint64_t* prev,
                   uint8_t* prev_found) {
    for (uint64_t i = 0; i < W; i++) {
        uint64_t pv = 0;
        int f = orc_hm_insert(m, puts_kv[2 * i], puts_kv[2 * i + 1], &pv);
        if (prev) prev[i] = f ? pv : 0;
        if (prev_found) prev_found[i] = (uint8_t)f;
    }
}

/* Dispatch::dispatch(Get) after sync (benches/hashmap.rs:107-111): Option<u64> -> (val, found) */
void orc_hm_get_batch(const orc_hm* m, const uint64_t* keys, uint64_t n, uint64_t* vals,
                      uint8_t* found) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t v = 0;
        int f = orc_hm_get(m, keys[i], &v);
        vals[i] = f ? v : 0;
        found[i] = (uint8_t)f;
    }
}

void orc_hm_run_mixed(orc_hm* m, const uint8_t* is_put, const uint64_t* keys,
                      const uint64_t* vals, uint64_t n, uint64_t* resp, uint8_t* some) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t v = 0;
        int f = is_put[i] ? orc_hm_insert(m, keys[i], vals[i], &v) : orc_hm_get(m, keys[i], &v);
        resp[i] = f ? v : 0;
        some[i] = (uint8_t)f;
    }
}

static int cmp_pair(const void* a, const void* b) {
    uint64_t x = ((const uint64_t*)a)[0], y = ((const uint64_t*)b)[0];
    return x < y ? -1 : (x > y ? 1 : 0);
}

uint64_t orc_hm_dump_sorted(const orc_hm* m, uint64_t* keys, uint64_t* vals) {
    uint64_t* pairs = (uint64_t*)malloc((m->len ? m->len : 1) * 2 * sizeof(uint64_t));
    uint64_t n = 0;
    for (uint64_t i = 0; i < m->cap; i++) {
        if (!m->used[i]) continue;
        pairs[2 * n] = m->keys[i];
        pairs[2 * n + 1] = m->vals[i];
        n++;
    }
    qsort(pairs, n, 2 * sizeof(uint64_t), cmp_pair);
    for (uint64_t i = 0; i < n; i++) {
        keys[i] = pairs[2 * i];
        vals[i] = pairs[2 * i + 1];
    }
    free(pairs);
    return n;
}

void orc_hm_digest(const orc_hm* m, uint64_t out[3]) {
    uint64_t cnt = 0, sum = 0, x = 0;
    for (uint64_t i = 0; i < m->cap; i++) {
        if (!m->used[i]) continue;
        uint64_t h = orc_mix64(m->keys[i] ^ orc_mix64(m->vals[i]));
        cnt++;
        sum += h;
        x ^= h;
    }
    out[0] = cnt;
    out[1] = sum;
    out[2] = x;
}

/* ---- Stack: Vec<u32> ----------------------------------------------------------- */
struct orc_stack {
    uint32_t* v;
    uint64_t len, cap;
};

orc_stack* orc_stack_new(const uint32_t* init, uint64_t n) {
    orc_stack* s = (orc_stack*)calloc(1, sizeof(orc_stack));
    s->cap = n > 16 ? n : 16;
    s->v = (uint32_t*)malloc(s->cap * sizeof(uint32_t));
    if (n) memcpy(s->v, init, n * sizeof(uint32_t));
    s->len = n;
    return s;
}

void orc_stack_free(orc_stack* s) {
    if (!s) return;
    free(s->v);
    free(s);
}

/* Stack::dispatch_mut (benches/stack.rs:75-83; nr/tests/stack.rs:87-95) */
void orc_stack_replay(orc_stack* s, const uint32_t* vals, const uint32_t* ops, uint64_t n,
                      int push_resp, uint32_t* resp, uint8_t* some) {
    for (uint64_t i = 0; i < n; i++) {
        uint32_t r = 0;
        uint8_t f = 0;
        if (ops[i]) {
            if (s->len == s->cap) {
                s->cap *= 2;
                s->v = (uint32_t*)realloc(s->v, s->cap * sizeof(uint32_t));
            }
            s->v[s->len++] = vals[i];
            if (push_resp) { r = vals[i]; f = 1; }
        } else if (s->len) {
            r = s->v[--s->len];
            f = 1;
        }
        if (resp) resp[i] = r;
        if (some) some[i] = f;
    }
}

uint64_t orc_stack_len(const orc_stack* s) { return s->len; }

uint64_t orc_stack_dump(const orc_stack* s, uint32_t* out) {
    if (s->len) memcpy(out, s->v, s->len * sizeof(uint32_t));
    return s->len;
}

int orc_stack_peek(const orc_stack* s, uint32_t* val) {
    if (!s->len) return 0;
    *val = s->v[s->len - 1];
    return 1;
}

/* ---- AbstractDataStructure (benches/synthetic.rs:60-195) --------------------------- */
struct orc_synth {
    uint64_t n, cold_reads, cold_writes, hot_reads, hot_writes;
    uint64_t* storage;
};

orc_synth* orc_synth_new(uint64_t n, uint64_t cold_reads, uint64_t cold_writes,
                         uint64_t hot_reads, uint64_t hot_writes) {
    orc_synth* s = (orc_synth*)calloc(1, sizeof(orc_synth));
    s->n = n;
    s->cold_reads = cold_reads;
    s->cold_writes = cold_writes;
    s->hot_reads = hot_reads;
    s->hot_writes = hot_writes;
    s->storage = (uint64_t*)malloc(n * sizeof(uint64_t));
    for (uint64_t i = 0; i < n; i++) s->storage[i] = i; /* :97-100 */
    return s;
}

void orc_synth_free(orc_synth* s) {
    if (!s) return;
    free(s->storage);
    free(s);
}

/* `for i in begin..end` with end = begin + hot_writes wrapping (release build): empty when
 * the addition wraps (benches/synthetic.rs:114-121,136-141,156-161). */
static inline uint64_t hot_count(uint64_t begin, uint64_t hw) {
    uint64_t end = begin + hw;
    return end < begin ? 0 : hw;
}

static uint64_t synth_read_write(orc_synth* s, uint64_t tid, uint64_t r1, uint64_t r2) {
    uint64_t hc = hot_count(r2, s->hot_writes);
    for (uint64_t j = 0; j < hc; j++) {
        uint64_t idx = (r2 + j) % s->hot_reads;
        s->storage[idx] = s->storage[idx] + 1;
    }
    uint64_t sum = 0, begin = r1 * tid;
    for (uint64_t k = 0; k < s->cold_writes; k++) {
        uint64_t idx = begin % (s->n - s->hot_reads) + s->hot_reads;
        begin += r2;
        sum += s->storage[idx];
        s->storage[idx] = s->storage[idx] + 1;
    }
    return sum;
}

static uint64_t synth_write(orc_synth* s, uint64_t tid, uint64_t r1, uint64_t r2) {
    uint64_t hc = hot_count(r2, s->hot_writes);
    for (uint64_t j = 0; j < hc; j++) s->storage[(r2 + j) % s->hot_reads] = tid;
    uint64_t begin = r1 * tid;
    for (uint64_t k = 0; k < s->cold_writes; k++) {
        uint64_t idx = begin % (s->n - s->hot_reads) + s->hot_reads;
        begin += r2;
        s->storage[idx] = tid;
    }
    return 0;
}

void orc_synth_replay(orc_synth* s, const uint64_t* ops, uint64_t n, uint64_t* resp) {
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t* o = ops + 4 * i;
        uint64_t r = o[3] ? synth_read_write(s, o[0], o[1], o[2]) : synth_write(s, o[0], o[1], o[2]);
        if (resp) resp[i] = r;
    }
}

/* AbstractDataStructure::read (:112-132): iterates hot_WRITES over the hot lines, then
 * cold_reads random-stride reads. */
void orc_synth_read(const orc_synth* s, const uint64_t* ops, uint64_t n, uint64_t* sums) {
    for (uint64_t i = 0; i < n; i++) {
        uint64_t tid = ops[3 * i], r1 = ops[3 * i + 1], r2 = ops[3 * i + 2];
        uint64_t sum = 0;
        uint64_t hc = hot_count(r2, s->hot_writes);
        for (uint64_t j = 0; j < hc; j++) sum += s->storage[(r2 + j) % s->hot_reads];
        uint64_t begin = r1 * tid;
        for (uint64_t k = 0; k < s->cold_reads; k++) {
            uint64_t idx = begin % (s->n - s->hot_reads) + s->hot_reads;
            begin += r2;
            sum += s->storage[idx];
        }
        sums[i] = sum;
    }
}

uint64_t orc_synth_dump(const orc_synth* s, uint64_t* out) {
    memcpy(out, s->storage, s->n * sizeof(uint64_t));
    return s->n;
}
