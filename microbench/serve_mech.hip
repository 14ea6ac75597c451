// Diagnostic: the round server's host <-> device hand-off alone (no hashmap work). A resident
// workgroup polls `posted` in mapped host memory, answers each round with `served` (and a word
// per round, like the combiner's error word), and exits on `stop` or after 100 ms idle.
// Variants: argv[1] = 0 host and device words on one line, 1 on separate 128-B lines.
// Build: hipcc --offload-arch=gfx950 -O2 microbench/serve_mech.hip -o microbench/serve_mech
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>

struct Ctl {
    alignas(128) uint64_t posted;
    uint32_t stop;
    alignas(128) uint64_t served;
    uint64_t exited;
};

__device__ __forceinline__ void host_put(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

__global__ __launch_bounds__(1024) void serve(Ctl* c, uint64_t* served_alt, uint32_t* words, uint64_t idle) {
    __shared__ int cmd;
    __shared__ uint64_t sk;
    if (threadIdx.x == 0) sk = 0;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (;;) {
        if (wave == 0) {  // wave-uniform: the poll loop is not an exec-masked region
            const uint64_t k = sk;
            const uint64_t t0 = wall_clock64();
            int x = 0;
            for (;;) {
                const uint64_t p = __hip_atomic_load(&c->posted, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
                if ((((uint64_t)hi << 32) | lo) > k) {
                    x = 1;
                    break;
                }
                if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&c->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))) break;
                if (wall_clock64() - t0 > idle) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (threadIdx.x == 0) cmd = x;
        }
        __syncthreads();
        if (!cmd) break;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            *(volatile uint32_t*)&words[sk % 8] = 7;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            sk = sk + 1;
            host_put(served_alt, sk);
        }
    }
    if (threadIdx.x == 0) host_put(&c->exited, 1);
}

__global__ void clk(uint64_t* out) {
    out[0] = wall_clock64();
    for (int i = 0; i < 1000; i++) __builtin_amdgcn_s_sleep(100);
    out[1] = wall_clock64();
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    const int sep = argc > 1 ? std::atoi(argv[1]) : 1;
    {
        uint64_t* d;
        uint64_t h[2];
        (void)hipMalloc(&d, 16);
        const auto a = std::chrono::steady_clock::now();
        clk<<<1, 64>>>(d);
        (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
        std::printf("wall_clock64 ticks %llu over <= %.1f host us\n", (unsigned long long)(h[1] - h[0]), us);
    }
    Ctl* c = nullptr;
    uint32_t* words = nullptr;
    if (hipHostMalloc((void**)&c, sizeof(Ctl), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
    if (hipHostMalloc((void**)&words, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 1;
    *c = Ctl{};
    uint64_t* served = sep ? &c->served : (uint64_t*)((char*)&c->posted + 32);  // 0: on the posted line
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    serve<<<1, 1024, 0, s>>>(c, served, words, 10000000ull);
    std::printf("launched: %s\n", hipGetErrorString(hipGetLastError()));
    int ok = 0;
    for (uint64_t k = 0; k < 20; k++) {
        words[k % 8] = 0;
        __atomic_store_n(&c->posted, k + 1, __ATOMIC_SEQ_CST);
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(served, __ATOMIC_SEQ_CST) < k + 1 &&
               std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(300)) {
        }
        const bool got = __atomic_load_n(served, __ATOMIC_SEQ_CST) >= k + 1;
        std::printf("round %llu: served %llu word %u %s\n", (unsigned long long)k,
                    (unsigned long long)__atomic_load_n(served, __ATOMIC_SEQ_CST), *(volatile uint32_t*)&words[k % 8],
                    got ? "ok" : "TIMEOUT");
        if (!got) {
            std::printf("  stream query: %s, posted %llu\n", hipGetErrorString(hipStreamQuery(s)),
                        (unsigned long long)c->posted);
            break;
        }
        ok++;
    }
    __atomic_store_n(&c->stop, 1u, __ATOMIC_SEQ_CST);
    std::printf("stop set\n");
    for (int i = 0; i < 50 && hipStreamQuery(s) == hipErrorNotReady; i++) usleep(20000);
    std::printf("after 1 s: stream %s exited %llu\n", hipGetErrorString(hipStreamQuery(s)), (unsigned long long)c->exited);
    const hipError_t e = hipStreamSynchronize(s);
    std::printf("sep %d: %d rounds ok, exited %llu, sync %s\n", sep, ok, (unsigned long long)c->exited, hipGetErrorString(e));
    return ok == 20 ? 0 : 2;
}
