// Back-to-back launch period on one stream for kernels of different shapes (no work inside):
// how much of a round's time a kernel boundary costs on MI355X. Prints us per launch.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int LDS_WORDS>
__global__ __launch_bounds__(512) void k_empty(unsigned* out, unsigned n) {
    __shared__ unsigned s[LDS_WORDS];
    s[threadIdx.x % LDS_WORDS] = threadIdx.x;
    __syncthreads();
    if (s[(threadIdx.x + 1) % LDS_WORDS] == 0xFFFFFFFFu && n == 12345u) out[blockIdx.x] = 1;  // never
}
// writes `per` bytes per thread of fresh data (the next kernel's boundary then has dirty lines)
__global__ __launch_bounds__(512) void k_write(unsigned* out, unsigned per) {
    unsigned* p = out + (size_t)(blockIdx.x * 512 + threadIdx.x) * per;
    for (unsigned i = 0; i < per; i++) p[i] = i;
}

template <typename F>
float period(F launch, int iters) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 20; i++) launch();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < iters; i++) launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1000.f / iters;
}

int main() {
    unsigned* buf;
    if (hipMalloc(&buf, 256u << 20) != hipSuccess) return 1;
    const int it = 500;
    printf("1 WG, no LDS:           %.2f us\n", period([&] { hipLaunchKernelGGL((k_empty<64>), 1, 512, 0, 0, buf, 0u); }, it));
    printf("512 WG, 1 KB LDS:       %.2f us\n", period([&] { hipLaunchKernelGGL((k_empty<256>), 512, 512, 0, 0, buf, 0u); }, it));
    printf("512 WG, 48 KB LDS:      %.2f us\n", period([&] { hipLaunchKernelGGL((k_empty<12288>), 512, 512, 0, 0, buf, 0u); }, it));
    printf("978 WG, 51 KB LDS:      %.2f us\n", period([&] { hipLaunchKernelGGL((k_empty<13056>), 978, 512, 0, 0, buf, 0u); }, it));
    printf("4300 WG, 1 KB LDS:      %.2f us\n", period([&] { hipLaunchKernelGGL((k_empty<256>), 4300, 512, 0, 0, buf, 0u); }, it));
    for (unsigned per : {1u, 16u, 64u}) {
        const double mb = 512.0 * 512 * per * 4 / 1e6;
        printf("512 WG writing %.0f MB: %.2f us\n", mb, period([&] { hipLaunchKernelGGL(k_write, 512, 512, 0, 0, buf, per); }, 200));
    }
    return 0;
}
