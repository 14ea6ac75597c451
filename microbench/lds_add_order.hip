// Does a returning LDS add hand conflicting lanes of one instruction their old values in lane
// order? (The synthetic partition's NRG_SYP_ADD variant ranks touches that way.) Every wave runs
// trials of random keys over K packed u16 counters and compares each lane's returned count with
// the number of lower lanes holding the same key. Prints the violations per K.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(512) void order_kernel(uint32_t K, uint32_t trials, unsigned long long* bad,
                                                    unsigned long long* checked) {
    __shared__ unsigned short cnt[8][512];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    unsigned long long nbad = 0, nchk = 0;
    for (uint32_t t = 0; t < trials; t++) {
        for (int i = lane; i < 512; i += 64) cnt[w][i] = 0;
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        // five instructions per trial, as the partition's five touches per op round
        for (int r = 0; r < 5; r++) {
            const uint32_t key = mix(blockIdx.x * 0x9E3779B9u + t * 131u + r * 7u + w * 1000003u + lane) % K;
            uint32_t before = 0;
            for (int l = 0; l < 64; l++) {
                const uint32_t kl = __shfl(key, l, 64);
                if (l < lane && kl == key) before++;
            }
            // counts of earlier instructions of this trial for the key
            uint32_t prior = cnt[w][key];
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            const uint32_t sh = (key & 1u) * 16u;
            const uint32_t old = (atomicAdd((uint32_t*)&cnt[w][key & ~1u], 1u << sh) >> sh) & 0xFFFFu;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            nbad += old != prior + before;
            nchk++;
        }
    }
    atomicAdd(bad, nbad);
    atomicAdd(checked, nchk);
}

int main() {
    unsigned long long *d, h[2];
    if (hipMalloc(&d, 16) != hipSuccess) return 1;
    const uint32_t Ks[] = {2, 8, 64, 512};
    for (uint32_t K : Ks) {
        (void)hipMemset(d, 0, 16);
        hipLaunchKernelGGL(order_kernel, dim3(1024), dim3(512), 0, 0, K, 200u, d, d + 1);
        if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
        (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("K=%u lanes checked %llu, out of lane order %llu\n", K, h[1], h[0]);
    }
    return 0;
}
