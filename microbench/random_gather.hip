// random_gather.hip — how fast can MI355X serve random small reads from a table far larger
// than the Infinity Cache? Calibrates the roofline of the NrHashMap lookup (SURVEY.md §8d
// "sector-size check"): each Get is one random 16-B slot read from a 1 GiB table.
//
// Variants (all read a 2^26 x 16 B = 1 GiB table at splitmix-random slots):
//   g16xK : each lane issues K independent 16-B loads (K = 1, 2, 4, 8) -> MLP per lane
//   g8xK  : 8-B loads (key only)
//   g64   : 4 lanes cooperatively read one 64-B line (one dwordx4 each)
// Prints per variant: lookups/s, useful GB/s, and GB/s if every access moved a 64-B / 128-B
// sector. Run under rocprofv3 --pmc FETCH_SIZE to see the bytes the L2 actually fetched.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHK(x)                                                                          \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));    \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

typedef unsigned long long u64;

__device__ __forceinline__ u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

struct __attribute__((aligned(16))) Slot {
    u64 k, v;
};

template <int K>
__global__ __launch_bounds__(256) void g16(const Slot* __restrict__ t, u64 mask, u64 n, u64 seed, u64* out) {
    const u64 base = (blockIdx.x * 256ull + threadIdx.x) * K;
    Slot s[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
        const u64 i = base + j;
        s[j] = i < n ? t[mix64(seed + i) & mask] : Slot{0, 0};
    }
    u64 acc = 0;
#pragma unroll
    for (int j = 0; j < K; j++) acc += s[j].k ^ s[j].v;
    if (acc == 0x12345) out[0] = acc;
}

template <int K>
__global__ __launch_bounds__(256) void g8(const u64* __restrict__ t, u64 mask, u64 n, u64 seed, u64* out) {
    const u64 base = (blockIdx.x * 256ull + threadIdx.x) * K;
    u64 s[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
        const u64 i = base + j;
        s[j] = i < n ? t[2 * (mix64(seed + i) & mask)] : 0;
    }
    u64 acc = 0;
#pragma unroll
    for (int j = 0; j < K; j++) acc += s[j];
    if (acc == 0x12345) out[0] = acc;
}

// 4 lanes read one 64-B line (4 consecutive slots), K lines per group
template <int K>
__global__ __launch_bounds__(256) void g64(const Slot* __restrict__ t, u64 mask, u64 n, u64 seed, u64* out) {
    const u64 grp = (blockIdx.x * 256ull + threadIdx.x) >> 2;
    const int sub = threadIdx.x & 3;
    Slot s[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
        const u64 i = grp * K + j;
        s[j] = i < n ? t[((mix64(seed + i) & mask) & ~3ull) + sub] : Slot{0, 0};
    }
    u64 acc = 0;
#pragma unroll
    for (int j = 0; j < K; j++) acc += s[j].k ^ s[j].v;
    if (acc == 0x12345) out[0] = acc;
}

// 32-B slots: key+val (16 B) and stamp (8 B) of one slot, two loads from one 128-B line
struct __attribute__((aligned(32))) Slot32 {
    u64 k, v, st, pad;
};
__global__ __launch_bounds__(256) void g32(const Slot32* __restrict__ t, u64 mask, u64 n, u64 seed, u64* out) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    const Slot32* p = &t[mix64(seed + i) & mask];
    const u64 k = p->k, v = p->v, st = p->st;
    if ((k ^ v ^ st) == 0x12345) out[0] = k;
}

// scattered device-scope atomics / plain stores over a small (L2/MALL-sized) array
__global__ __launch_bounds__(256) void a_cas(u64* a, u64 mask, u64 n, u64 seed, u64* out) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    const u64 h = mix64(seed + i);
    const u64 old = atomicCAS(&a[h & mask], 0ull, h | 1);
    if (old == 0x12345) out[0] = old;
}
__global__ __launch_bounds__(256) void a_max(unsigned* a, u64 mask, u64 n, u64 seed) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    atomicMax(&a[mix64(seed + i) & mask], (unsigned)i);
}
__global__ __launch_bounds__(256) void s_byte(unsigned char* a, u64 mask, u64 n, u64 seed) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    a[mix64(seed + i) & mask] = 1;
}
__global__ __launch_bounds__(256) void s_16(Slot* a, u64 mask, u64 n, u64 seed) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    a[mix64(seed + i) & mask] = Slot{i, i};
}

template <typename F>
float time_it(F f, int reps) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    f();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) f();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms;
    CHK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}


// NrHashMap Get-shaped variants over 64-B slots (the replica's layout): the key comes from a
// streamed key array (dependent load), one or two 16-B loads of the slot's line, value and
// found byte stored. Separates the cost of each piece of hm_round's read role.
struct __attribute__((aligned(16))) Slot64 {
    u64 k, v, s1, c, s0, p0, p1, p2;
};
__global__ void init_keys(u64* keys, u64 n) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i < n) keys[i] = mix64(i + 12345);
}
template <int KEYLOAD, int TWO, int STORE>
__global__ __launch_bounds__(256) void gget(const Slot64* __restrict__ t, const u64* __restrict__ keys, u64 mask,
                                            u64 n, u64* __restrict__ vals, unsigned char* __restrict__ found,
                                            u64* out) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    const u64 key = KEYLOAD ? keys[i] : mix64(i * 0x9E3779B97F4A7C15ull);
    const Slot64* p = &t[mix64(key) & mask];
    const uint4 a = *(const uint4*)&p->k;
    uint4 b = {0, 0, 0, 0};
    if (TWO) b = *(const uint4*)&p->s1;
    const u64 k = ((u64)a.y << 32) | a.x;
    const u64 v = (((u64)a.w << 32) | a.z) + b.x + b.z;
    if (STORE) {
        vals[i] = k == key ? v : 0;
        found[i] = k == key;
    } else if ((k ^ v) == 0x12345) {
        out[0] = k;
    }
}

// lane pairs: lane 2j loads {key, val}, lane 2j+1 the {stamp, created} 16 B of the same slot
// (one 32-B access per Get in one wave instruction), exchanged with a lane shuffle
template <int STORE>
__global__ __launch_bounds__(256) void gpair(const Slot64* __restrict__ t, const u64* __restrict__ keys, u64 mask,
                                             u64 n, u64* __restrict__ vals, unsigned char* __restrict__ found,
                                             u64* out) {
    const u64 i = (blockIdx.x * 256ull + threadIdx.x) >> 1;
    const int half = threadIdx.x & 1;
    const u64 key = i < n ? keys[i] : 0;
    const Slot64* p = &t[mix64(key) & mask];
    const uint4 a = i < n ? *((const uint4*)&p->k + half) : uint4{0, 0, 0, 0};
    uint4 o;
    o.x = __shfl_xor((int)a.x, 1);
    o.y = __shfl_xor((int)a.y, 1);
    o.z = __shfl_xor((int)a.z, 1);
    o.w = __shfl_xor((int)a.w, 1);
    const uint4 kv = half ? o : a, sc = half ? a : o;
    const u64 k = ((u64)kv.y << 32) | kv.x;
    const u64 v = (((u64)kv.w << 32) | kv.z) + sc.x + sc.z;
    if (i >= n) return;
    if (STORE) {
        if (!half) vals[i] = k == key ? v : 0;
        else found[i] = k == key;
    } else if ((k ^ v) == 0x12345) {
        out[0] = k;
    }
}

// scattered stamp atomics into 64-B slots of the replica-sized table: 64-bit vs 32-bit max
template <typename T>
__global__ __launch_bounds__(256) void a_slot(Slot64* t, u64 mask, u64 n, u64 seed, int off) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    T* p = (T*)((char*)&t[mix64(seed + i) & mask] + off);
    atomicMax(p, (T)(i + 1));
}

// scattered plain 8-B stores into 64-B slots of the replica-sized table
__global__ __launch_bounds__(256) void st_slot(Slot64* t, u64 mask, u64 n, u64 seed) {
    const u64 i = blockIdx.x * 256ull + threadIdx.x;
    if (i >= n) return;
    t[mix64(seed + i) & mask].s1 = i + 1;
}

int main(int argc, char** argv) {
    const int log2 = argc > 1 ? atoi(argv[1]) : 26;
    const u64 slots = 1ull << log2, mask = slots - 1;
    const u64 n = argc > 2 ? strtoull(argv[2], 0, 10) : (1ull << 22);
    const int reps = 20;
    Slot* t;
    u64* out;
    CHK(hipMalloc(&t, slots * sizeof(Slot)));
    CHK(hipMemset(t, 1, slots * sizeof(Slot)));
    CHK(hipMalloc(&out, 64));
    if (argc > 3) {  // Get-shaped variants over 2^log2 64-B slots
        CHK(hipFree(t));
        Slot64* t64;
        u64 *keys, *vals;
        unsigned char* fnd;
        // argv[3]: get = hipMalloc; getuc = uncached (MTYPE UC); getfg = fine-grained; getct = contiguous
        if (!strcmp(argv[3], "getuc")) CHK(hipExtMallocWithFlags((void**)&t64, slots * sizeof(Slot64), hipDeviceMallocUncached));
        else if (!strcmp(argv[3], "getct")) CHK(hipExtMallocWithFlags((void**)&t64, slots * sizeof(Slot64), hipDeviceMallocContiguous));
        else if (!strcmp(argv[3], "getfg")) CHK(hipExtMallocWithFlags((void**)&t64, slots * sizeof(Slot64), hipDeviceMallocFinegrained));
        else CHK(hipMalloc(&t64, slots * sizeof(Slot64)));
        printf("table allocation: %s\n", argv[3]);
        CHK(hipMemset(t64, 1, slots * sizeof(Slot64)));
        CHK(hipMalloc(&keys, 16 * n * 8));
        CHK(hipMalloc(&vals, n * 8));
        CHK(hipMalloc(&fnd, n));
        printf("64-B slot table %llu slots (%.2f GiB), %llu Gets per launch\n", slots, slots * 64.0 / (1 << 30), n);
        const unsigned g = (unsigned)((n + 255) / 256);
        init_keys<<<16 * g, 256>>>(keys, 16 * n);
        int rot = 0;  // 16 distinct key batches in rotation: no MALL reuse between launches
#define RUNG(A, B, C)                                                                                      \
    {                                                                                                      \
        float ms = time_it([&] { gget<A, B, C><<<g, 256>>>(t64, keys + (rot++ % 16) * n, mask, n, vals, fnd, out); }, reps); \
        printf("get key%d two%d store%d  %8.2f us  %7.2f Glookups/s\n", A, B, C, ms * 1e3, n / (ms / 1e3) / 1e9); \
    }
        for (int st = 0; st < 2; st++) {
            const unsigned g2 = (unsigned)((2 * n + 255) / 256);
            float ms = time_it([&] {
                const u64* kb = keys + (rot++ % 16) * n;
                if (st) gpair<1><<<g2, 256>>>(t64, kb, mask, n, vals, fnd, out);
                else gpair<0><<<g2, 256>>>(t64, kb, mask, n, vals, fnd, out);
            }, reps);
            printf("get pair  key1 store%d  %8.2f us  %7.2f Glookups/s\n", st, ms * 1e3, n / (ms / 1e3) / 1e9);
        }
        {
            int seed = 0;
            float ms = time_it([&] { a_slot<unsigned long long><<<g, 256>>>(t64, mask, n, 1000 + seed++, 16); }, reps);
            printf("atomicMax u64 into slots  %8.2f us  %7.2f Gops/s\n", ms * 1e3, n / (ms / 1e3) / 1e9);
            ms = time_it([&] { a_slot<unsigned int><<<g, 256>>>(t64, mask, n, 2000 + seed++, 16); }, reps);
            printf("atomicMax u32 into slots  %8.2f us  %7.2f Gops/s\n", ms * 1e3, n / (ms / 1e3) / 1e9);
            ms = time_it([&] { st_slot<<<g, 256>>>(t64, mask, n, 3000 + seed++); }, reps);
            printf("plain u64 store into slots %7.2f us  %7.2f Gops/s\n", ms * 1e3, n / (ms / 1e3) / 1e9);
        }
        RUNG(0, 0, 0) RUNG(0, 1, 0) RUNG(0, 0, 1) RUNG(0, 1, 1) RUNG(1, 0, 0) RUNG(1, 1, 0) RUNG(1, 0, 1) RUNG(1, 1, 1)
        return 0;
    }
    printf("table %llu slots (%.2f GiB), %llu lookups per launch\n", slots, slots * 16.0 / (1 << 30), n);
    auto report = [&](const char* name, float ms, double useful_bytes) {
        double s = ms / 1e3;
        printf("%-8s %8.2f us  %8.2f Glookups/s  useful %7.1f GB/s  @64B %7.1f GB/s  @128B %7.1f GB/s\n", name,
               ms * 1e3, n / s / 1e9, n * useful_bytes / s / 1e9, n * 64.0 / s / 1e9, n * 128.0 / s / 1e9);
    };
#define RUN16(K)                                                                                        \
    {                                                                                                   \
        u64 g = (n + 256 * K - 1) / (256 * K);                                                          \
        float ms = time_it([&] { g16<K><<<(unsigned)g, 256>>>(t, mask, n, 77 + K, out); }, reps);      \
        report("g16x" #K, ms, 16);                                                                      \
    }
#define RUN8(K)                                                                                         \
    {                                                                                                   \
        u64 g = (n + 256 * K - 1) / (256 * K);                                                          \
        float ms = time_it([&] { g8<K><<<(unsigned)g, 256>>>((const u64*)t, mask, n, 99 + K, out); }, reps); \
        report("g8x" #K, ms, 8);                                                                        \
    }
#define RUN64(K)                                                                                        \
    {                                                                                                   \
        u64 g = (n * 4 + 256 * K - 1) / (256 * K);                                                      \
        float ms = time_it([&] { g64<K><<<(unsigned)g, 256>>>(t, mask, n, 55 + K, out); }, reps);      \
        report("g64x" #K, ms, 64);                                                                      \
    }
    RUN16(1) RUN16(2) RUN16(4) RUN16(8)
    RUN8(1) RUN8(4)
    RUN64(1) RUN64(4)
    {  // 32-B slots over the same bytes (half as many slots)
        const unsigned g = (unsigned)((n + 255) / 256);
        float ms = time_it([&] { g32<<<g, 256>>>((const Slot32*)t, mask >> 1, n, 31, out); }, reps);
        report("g32x1", ms, 24);
    }
    // scattered atomics / stores: 100k and 1M ops over a 4 MiB array (the BLT's size at B1)
    for (u64 m : {100000ull, 1000000ull}) {
        const u64 amask = (4ull << 20) / 8 - 1;
        const unsigned g = (unsigned)((m + 255) / 256);
        float ms;
        ms = time_it([&] { CHK(hipMemsetAsync(t, 0, 4 << 20)); a_cas<<<g, 256>>>((u64*)t, amask, m, 5, out); }, reps);
        printf("cas64   n=%7llu  %8.2f us (incl. 4 MiB memset)  %6.2f Gops/s\n", m, ms * 1e3, m / (ms / 1e3) / 1e9);
        ms = time_it([&] { a_max<<<g, 256>>>((unsigned*)t, amask * 2 + 1, m, 6); }, reps);
        printf("max32   n=%7llu  %8.2f us  %6.2f Gops/s\n", m, ms * 1e3, m / (ms / 1e3) / 1e9);
        ms = time_it([&] { s_byte<<<g, 256>>>((unsigned char*)t, (1ull << 20) - 1, m, 7); }, reps);
        printf("byte1MB n=%7llu  %8.2f us  %6.2f Gops/s\n", m, ms * 1e3, m / (ms / 1e3) / 1e9);
        ms = time_it([&] { s_16<<<g, 256>>>(t, (4ull << 20) / 16 - 1, m, 8); }, reps);
        printf("st16    n=%7llu  %8.2f us  %6.2f Gops/s\n", m, ms * 1e3, m / (ms / 1e3) / 1e9);
        ms = time_it([&] { CHK(hipMemsetAsync(t, 0, 4 << 20)); }, reps);
        printf("memset 4MiB        %8.2f us\n", ms * 1e3);
    }
    CHK(hipFree(t));
    return 0;
}
