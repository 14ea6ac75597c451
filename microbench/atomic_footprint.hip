// atomic_footprint.hip — what does a device-scope 64-bit atomicMax cost as a function of the
// footprint it lands in? The stamp rounds' index pass issues one per distinct key of a block
// into the 2-GiB table (5.9 us of B1's 34.7-us round, profiles/r04_b1_ablation.txt). If atomics
// into a footprint the 256-MB Infinity Cache holds ran much faster, a compact election array
// would pay; this measures it. N random atomics per launch (splitmix-random offsets), footprints
// 8 MB .. 2 GiB, returning (value used) and non-returning forms, 16 rotating seeds.
// Usage: atomic_footprint [N]   (default 100000, B1's Puts)
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

__device__ inline u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// one atomic per thread; stride 4 words = one per 32-B slot, as the table's stamps
template <bool RET>
__global__ __launch_bounds__(256) void amax(u64* a, u64 mask, u64 n, u64 seed, u64* sink) {
    const u64 i = (u64)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const u64 slot = mix64(seed + i) & mask;
    const u64 v = (seed << 32) | (i + 1);
    if (RET) {
        const u64 old = atomicMax(&a[slot * 4], v);
        if (old == 0x12345) sink[0] = old;
    } else {
        (void)__hip_atomic_fetch_max(&a[slot * 4], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <bool RET>
static void run(u64* a, u64 bytes, u64 n, u64* sink, hipStream_t st) {
    const u64 slots = bytes / 32, mask = slots - 1;
    const unsigned grid = (unsigned)((n + 255) / 256);
    for (int i = 0; i < 8; i++) amax<RET><<<grid, 256, 0, st>>>(a, mask, n, 1000 + i, sink);
    hipEvent_t b0, b1;
    CHK(hipEventCreate(&b0));
    CHK(hipEventCreate(&b1));
    const int L = 64;
    CHK(hipEventRecord(b0, st));
    for (int i = 0; i < L; i++) amax<RET><<<grid, 256, 0, st>>>(a, mask, n, 2000 + (i & 15), sink);
    CHK(hipEventRecord(b1, st));
    CHK(hipEventSynchronize(b1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, b0, b1));
    const double us = ms * 1e3 / L;
    printf("footprint %6llu MB  ret=%d  %8.2f us per launch  %6.2f G atomics/s\n", bytes >> 20, (int)RET, us,
           n / us / 1e3);
    CHK(hipEventDestroy(b0));
    CHK(hipEventDestroy(b1));
}

int main(int argc, char** argv) {
    const u64 n = argc > 1 ? strtoull(argv[1], 0, 10) : 100000ull;
    const u64 maxb = 2ull << 30;
    u64 *a, *sink;
    CHK(hipMalloc((void**)&a, maxb));
    CHK(hipMemset(a, 0, maxb));
    CHK(hipMalloc((void**)&sink, 64));
    hipStream_t st;
    CHK(hipStreamCreate(&st));
    printf("atomic_footprint: %llu random 64-bit atomicMax per launch, one per 32-B slot\n", n);
    for (u64 b = 8ull << 20; b <= maxb; b <<= 2) {
        run<true>(a, b, n, sink, st);
        run<false>(a, b, n, sink, st);
    }
    CHK(hipStreamSynchronize(st));
    CHK(hipFree(a));
    CHK(hipFree(sink));
    return 0;
}
