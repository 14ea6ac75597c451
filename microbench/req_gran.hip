// req_gran.hip — can a random 32-B slot read leave L2 as less than a 128-B memory request?
//
// The hashmap read role sits at a random-line floor of ~44.7 G requests/s, every request a
// 128-B line (profiles/r01_rdreq_size.txt, profiles/r04_read_floor.txt). If the L2 could fetch
// 64 B (or 32 B) per random slot instead, the same request floor would carry half the bytes,
// or the rate might rise. This measures Get-shaped lookups (key streamed, 32-B slot {key, val,
// st[2]} at mix64(key) >> 38 of 2^26 slots = 2 GiB, value + found stored) under:
//   alloc 0  hipMalloc (coarse-grained, the product's table)
//   alloc 1  hipExtMallocWithFlags(hipDeviceMallocUncached)
//   alloc 2  hipExtMallocWithFlags(hipDeviceMallocFinegrained)
//   load  0  plain global loads
//   load  1  __builtin_nontemporal_load
//   load  2  buffer loads with sc0|sc1 (system scope: bypass / write-through L2 policy)
//   load  3  buffer loads with nt
// Usage: req_gran ALLOC LOAD [gets]   (one configuration per process, for per-pass PMC)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                       \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct __attribute__((aligned(32))) Slot {
    u64 key, val, st[2];
};

__device__ __host__ inline u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

constexpr int TPB = 256;
constexpr int SHIFT = 64 - 26;

__device__ inline __amdgpu_buffer_rsrc_t make_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

template <int LOAD>
__device__ inline void load_slot(const Slot* t, u64 s, u64x2& kv, u64& st) {
    if constexpr (LOAD == 0) {
        kv = *(const u64x2*)&t[s];
        st = t[s].st[0];
    } else if constexpr (LOAD == 1) {
        kv = __builtin_nontemporal_load((const u64x2*)&t[s]);
        st = __builtin_nontemporal_load(&t[s].st[0]);
    } else {
        // the table is 2 GiB: address the slot's 1-GiB half with its own resource
        const char* base = (const char*)t + ((s >> 25) << 30);
        const unsigned off = (unsigned)((s & ((1u << 25) - 1)) * 32);
        __amdgpu_buffer_rsrc_t r = make_rsrc(base);
        constexpr int aux = LOAD == 2 ? (1 | 16) : 2;
        u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, aux);
        u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, aux);
        kv.x = (u64)a.x | ((u64)a.y << 32);
        kv.y = (u64)a.z | ((u64)a.w << 32);
        st = (u64)b.x | ((u64)b.y << 32);
    }
}

template <int LOAD>
__global__ __launch_bounds__(TPB) void gets(const Slot* __restrict__ t, const u64* __restrict__ keys, u64 n,
                                            u64* __restrict__ vals, unsigned char* __restrict__ found) {
    const u64 q = (u64)blockIdx.x * TPB + threadIdx.x;
    if (q >= n) return;
    const u64 k = keys[q];
    u64x2 w;
    u64 st;
    load_slot<LOAD>(t, mix64(k) >> SHIFT, w, st);
    const bool f = w.x == k && st != 0;
    vals[q] = f ? w.y : 0;
    found[q] = f;
}

__global__ void fill(Slot* t, u64 slots) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < slots; i += (u64)gridDim.x * blockDim.x) {
        Slot s;
        s.key = i;
        s.val = i + 1;
        s.st[0] = s.st[1] = 1;
        t[i] = s;
    }
}

template <int LOAD>
void run(const Slot* t, u64* const* keys, u64 n, u64* vals, unsigned char* found, hipStream_t st, int alloc) {
    const unsigned grid = (unsigned)((n + TPB - 1) / TPB);
    for (int i = 0; i < 16; i++) gets<LOAD><<<grid, TPB, 0, st>>>(t, keys[i & 15], n, vals, found);
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const int L = 64;
    CHK(hipEventRecord(a, st));
    for (int i = 0; i < L; i++) gets<LOAD><<<grid, TPB, 0, st>>>(t, keys[i & 15], n, vals, found);
    CHK(hipEventRecord(b, st));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / L;
    printf("alloc=%d load=%d  %8.2f us per launch  %7.2f G gets/s\n", alloc, LOAD, us, n / us / 1e3);
}

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: req_gran ALLOC LOAD [gets]\n");
        return 2;
    }
    const int alloc = atoi(argv[1]), load = atoi(argv[2]);
    const u64 n = argc > 3 ? strtoull(argv[3], 0, 10) : 900000ull;
    const u64 slots = 1ull << 26;
    Slot* t;
    if (alloc == 0)
        CHK(hipMalloc((void**)&t, slots * sizeof(Slot)));
    else
        CHK(hipExtMallocWithFlags((void**)&t, slots * sizeof(Slot),
                                  alloc == 1 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
    fill<<<4096, 256>>>(t, slots);
    u64* keys[16];
    u64* h = (u64*)malloc(n * 8);
    for (int b = 0; b < 16; b++) {
        for (u64 i = 0; i < n; i++) h[i] = mix64(0x9e3779b97f4a7c15ull * (b * n + i + 1)) % 10000000ull;
        CHK(hipMalloc((void**)&keys[b], n * 8));
        CHK(hipMemcpy(keys[b], h, n * 8, hipMemcpyHostToDevice));
    }
    free(h);
    u64* vals;
    unsigned char* found;
    CHK(hipMalloc((void**)&vals, n * 8));
    CHK(hipMalloc((void**)&found, n));
    hipStream_t st;
    CHK(hipStreamCreate(&st));
    CHK(hipDeviceSynchronize());
    switch (load) {
        case 0: run<0>(t, keys, n, vals, found, st, alloc); break;
        case 1: run<1>(t, keys, n, vals, found, st, alloc); break;
        case 2: run<2>(t, keys, n, vals, found, st, alloc); break;
        default: run<3>(t, keys, n, vals, found, st, alloc); break;
    }
    CHK(hipStreamSynchronize(st));
    for (int b = 0; b < 16; b++) CHK(hipFree(keys[b]));
    CHK(hipFree(vals));
    CHK(hipFree(found));
    CHK(hipFree(t));
    return 0;
}
