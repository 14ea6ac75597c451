// Cold instruction fetch cost on gfx950 (diagnostic; run on the GPU box).
//
// Same VALU work, executed once per block by 489 blocks of 256 threads (the stack replay's
// launch shape), laid out as ~32 KB of straight-line code (unrolled) or as a ~100 B loop.
// Build: hipcc -O3 --offload-arch=gfx950 microbench/icache.hip -o microbench/icache
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 1024;

template <bool UNROLL>
__global__ __launch_bounds__(256) void work(float* out, float a, float b) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    if constexpr (UNROLL) {
#pragma unroll
        for (int i = 0; i < ITERS; i++) {
            x0 = x0 * a + b;
            x1 = x1 * a + b;
            x2 = x2 * a + b;
            x3 = x3 * a + b;
            a += 1e-7f;  // keeps every step a distinct instruction stream
        }
    } else {
#pragma unroll 1
        for (int i = 0; i < ITERS; i++) {
            x0 = x0 * a + b;
            x1 = x1 * a + b;
            x2 = x2 * a + b;
            x3 = x3 * a + b;
            a += 1e-7f;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3;
}

template <bool U>
static float run(float* d, int blocks, int reps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 5; i++) work<U><<<blocks, 256>>>(d, 1.0001f, 0.5f);
    hipEventRecord(e0);
    for (int i = 0; i < reps; i++) work<U><<<blocks, 256>>>(d, 1.0001f, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1000.f / reps;
}

int main() {
    float* d;
    if (hipMalloc(&d, 4096 * 256 * 4) != hipSuccess) return 1;
    for (int blocks : {256, 489, 2048}) {
        const float u = run<true>(d, blocks, 200), l = run<false>(d, blocks, 200);
        printf("blocks=%d  straight-line %.2f us   loop %.2f us  (%d x 5 VALU per thread)\n", blocks, u, l, ITERS);
    }
    hipFree(d);
    return 0;
}
