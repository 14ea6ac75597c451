// line_floor.hip — the random-line floor of the hashmap read role.
//
// Get-shaped lookups over the replica's layout: 2^26 slots of 32 B {key, val, st[2]} = 2 GiB,
// the slot from mix64(key) >> 38 as table_home does. Each Get loads its key from a streamed
// array, then the slot's {key, val} (16 B) and, with STAMP, its stamp word (8 B of the same
// 128-B line), and stores the value and a found byte. K Gets per thread, all their loads in
// flight together: K = 1 is the read role's shape (RPT = 1); K = 2, 4, 8 put 2x, 4x, 8x as many
// random lines in flight per wave. If the Gets/s stop rising with K, the memory side (not
// latency or occupancy) sets the rate and the read role's rate is the floor.
// Key batches rotate over 16 arrays so no launch re-reads the last one's lines from the
// 256-MB Infinity Cache. Usage: line_floor [gets_per_launch]   (default 900000, B1's Gets)
#include <hip/hip_runtime.h>

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

template <int K, bool STAMP>
__global__ __launch_bounds__(TPB) void gets(const Slot* __restrict__ t, const u64* __restrict__ keys, u64 n,
                                            u64* __restrict__ vals, unsigned char* __restrict__ found) {
    const u64 q0 = (u64)blockIdx.x * TPB * K + threadIdx.x;
    u64 k[K];
#pragma unroll
    for (int r = 0; r < K; r++) {
        const u64 q = q0 + (u64)r * TPB;
        k[r] = q < n ? keys[q] : 0;
    }
    u64x2 w[K];
    u64 st[K];
#pragma unroll
    for (int r = 0; r < K; r++) {
        const u64 s = mix64(k[r]) >> SHIFT;
        w[r] = *(const u64x2*)&t[s];
        st[r] = STAMP ? t[s].st[0] : 1;
    }
#pragma unroll
    for (int r = 0; r < K; r++) {
        const u64 q = q0 + (u64)r * TPB;
        if (q >= n) continue;
        const bool f = w[r].x == k[r] && st[r] != 0;
        vals[q] = f ? w[r].y : 0;
        found[q] = f;
    }
}

__global__ void fill(Slot* t, u64 slots) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < slots; i += (u64)gridDim.x * blockDim.x) {
        Slot s;
        s.key = i;  // (not the hashed layout: the loads, not the hits, are measured)
        s.val = i + 1;
        s.st[0] = s.st[1] = 1;
        t[i] = s;
    }
}

template <int K, bool STAMP>
void run(const Slot* t, u64* const* keys, u64 n, u64* vals, unsigned char* found, hipStream_t st) {
    const unsigned grid = (unsigned)((n + (u64)TPB * K - 1) / ((u64)TPB * K));
    for (int i = 0; i < 16; i++) gets<K, STAMP><<<grid, TPB, 0, st>>>(t, keys[i & 15], n, vals, found);
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    const int L = 64;
    CHK(hipEventRecord(a, st));
    for (int i = 0; i < L; i++) gets<K, STAMP><<<grid, TPB, 0, st>>>(t, keys[i & 15], n, vals, found);
    CHK(hipEventRecord(b, st));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / L;
    printf("K=%d stamp=%d  %8.2f us per launch  %7.2f G gets/s  %6.2f TB/s of 128-B lines  grid %u\n", K, (int)STAMP,
           us, n / us / 1e3, n * 128.0 / us / 1e6, grid);
    CHK(hipEventDestroy(a));
    CHK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
    const u64 n = argc > 1 ? strtoull(argv[1], 0, 10) : 900000ull;
    const u64 slots = 1ull << 26;
    Slot* t;
    CHK(hipMalloc((void**)&t, slots * sizeof(Slot)));
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
    printf("line_floor: %llu Gets per launch over 2^26 x 32-B slots (2 GiB), 16 rotating key batches\n",
           (unsigned long long)n);
    run<1, true>(t, keys, n, vals, found, st);
    run<2, true>(t, keys, n, vals, found, st);
    run<4, true>(t, keys, n, vals, found, st);
    run<8, true>(t, keys, n, vals, found, st);
    run<1, false>(t, keys, n, vals, found, st);
    run<4, false>(t, keys, n, vals, found, st);
    CHK(hipStreamSynchronize(st));
    for (int b = 0; b < 16; b++) CHK(hipFree(keys[b]));
    CHK(hipFree(vals));
    CHK(hipFree(found));
    CHK(hipFree(t));
    return 0;
}
