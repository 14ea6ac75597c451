// workload.hip — seeded synthetic op streams generated on device (bench inputs and tests).
//
// The reference generates its op streams with unseeded thread_rng (benches/hashmap.rs:131-162,
// benches/stack.rs:87-102); here every stream is a seeded splitmix64 sequence with the same
// definitions as oracle/nr_oracle.c, so the CPU oracle reproduces device-generated inputs:
//   uniform   keys[i] = mulhi64(splitmix64_at(seed, i), span)          (orc_gen_uniform)
//   raw       splitmix64_at(seed, i)                                   (orc_gen_raw)
//   zipf      Gray et al. (SIGMOD'94) inverse-CDF over ranks 1..N      (orc_gen_zipf)
//   stack ops op = r & 1 (1 = Push), val = r >> 32                     (orc_gen_stack_ops)
// The Zipf stream evaluates one double pow per key on device; ocml's pow and glibc's may
// differ in the last ulp, which can move a rare key to a neighbouring rank. It is therefore
// statistically, not bit-for-bit, the oracle's stream; parity tests feed oracle-generated
// keys instead (tests/test_gpu_hashmap.py).
#include "internal.hpp"

namespace nrg {

constexpr int GEN_TPB = 256;

static inline unsigned gen_grid(u64 n) {
    u64 g = (n + GEN_TPB - 1) / GEN_TPB;
    if (g < 1) g = 1;
    if (g > 8192) g = 8192;
    return (unsigned)g;
}

__global__ void gen_uniform_kernel(u64* out, u64 n, u64 seed, u64 span) {
    for (u64 i = blockIdx.x * (u64)GEN_TPB + threadIdx.x; i < n; i += (u64)gridDim.x * GEN_TPB)
        out[i] = mulhi64(sm64_at(seed, i), span);
}
__global__ void gen_raw_kernel(u64* out, u64 n, u64 seed) {
    for (u64 i = blockIdx.x * (u64)GEN_TPB + threadIdx.x; i < n; i += (u64)gridDim.x * GEN_TPB)
        out[i] = sm64_at(seed, i);
}
__global__ void gen_puts_kernel(nrg_put* out, const u64* k, const u64* v, u64 n) {
    for (u64 i = blockIdx.x * (u64)GEN_TPB + threadIdx.x; i < n; i += (u64)gridDim.x * GEN_TPB) {
        nrg_put p;
        p.key = k[i];
        p.val = v[i];
        out[i] = p;
    }
}
__global__ void gen_zipf_kernel(u64* out, u64 n, u64 seed, u64 N, double zetan, double half_pow, double eta,
                                double alpha, int scramble) {
    for (u64 i = blockIdx.x * (u64)GEN_TPB + threadIdx.x; i < n; i += (u64)gridDim.x * GEN_TPB) {
        const double u = (double)(sm64_at(seed, i) >> 11) * (1.0 / 9007199254740992.0);
        const double uz = u * zetan;
        u64 rank;
        if (uz < 1.0)
            rank = 1;
        else if (uz < half_pow)
            rank = 2;
        else
            rank = 1 + (u64)((double)N * pow(eta * u - eta + 1.0, alpha));
        if (rank > N) rank = N;
        out[i] = scramble ? mix64(rank) % N : rank - 1;
    }
}
__global__ void gen_stack_ops_kernel(nrg_stack_op* out, u64 n, u64 seed) {
    for (u64 i = blockIdx.x * (u64)GEN_TPB + threadIdx.x; i < n; i += (u64)gridDim.x * GEN_TPB) {
        const u64 r = sm64_at(seed, i);
        nrg_stack_op o;
        o.val = (uint32_t)(r >> 32);
        o.op = (uint32_t)(r & 1);
        out[i] = o;
    }
}

hipError_t gen_uniform(nrg_ctx* c, u64* d, u64 n, u64 seed, u64 span) {
    gen_uniform_kernel<<<gen_grid(n), GEN_TPB, 0, c->stream>>>(d, n, seed, span);
    return hipGetLastError();
}
hipError_t gen_raw(nrg_ctx* c, u64* d, u64 n, u64 seed) {
    gen_raw_kernel<<<gen_grid(n), GEN_TPB, 0, c->stream>>>(d, n, seed);
    return hipGetLastError();
}
hipError_t gen_puts(nrg_ctx* c, nrg_put* d, const u64* k, const u64* v, u64 n) {
    gen_puts_kernel<<<gen_grid(n), GEN_TPB, 0, c->stream>>>(d, k, v, n);
    return hipGetLastError();
}
hipError_t gen_stack_ops(nrg_ctx* c, nrg_stack_op* d, u64 n, u64 seed) {
    gen_stack_ops_kernel<<<gen_grid(n), GEN_TPB, 0, c->stream>>>(d, n, seed);
    return hipGetLastError();
}

// Host part of the Zipf generator: zeta(N, theta) summed in the oracle's order (i = 1..N),
// cached per (N, theta) in the context.
hipError_t gen_zipf(nrg_ctx* c, u64* d, u64 n, u64 seed, u64 N, double theta, int scramble) {
    if (N == 0 || !(theta > 0.0) || theta == 1.0) return hipErrorInvalidValue;
    if (c->zipf_n != N || c->zipf_theta != theta) {
        double z = 0.0;
        for (u64 i = 1; i <= N; i++) z += pow((double)i, -theta);
        c->zipf_n = N;
        c->zipf_theta = theta;
        c->zipf_zetan = z;
    }
    const double zetan = c->zipf_zetan;
    const double zeta2 = 1.0 + pow(2.0, -theta);
    const double alpha = 1.0 / (1.0 - theta);
    const double eta = (1.0 - pow(2.0 / (double)N, 1.0 - theta)) / (1.0 - zeta2 / zetan);
    const double half_pow = 1.0 + pow(0.5, theta);
    gen_zipf_kernel<<<gen_grid(n), GEN_TPB, 0, c->stream>>>(d, n, seed, N, zetan, half_pow, eta, alpha, scramble);
    return hipGetLastError();
}

}  // namespace nrg
