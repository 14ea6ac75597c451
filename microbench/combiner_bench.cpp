// Native client threads against the flat combiner (nrg_combiner_*), B1's table and stream.
//
// T std::threads each loop on synchronous calls of B ops for a fixed time: one call in ten a
// Put batch (Replica::execute_mut), the others Get batches (Replica::execute), keys uniform over
// 10M on a 2^26-slot table prefilled with [0, 2^23) -> k+1 (benches/hashmap.rs:77-122 with
// nr/src/replica.rs's synchronous per-thread API). Prints ops/s, GPU rounds and ops per round.
// The stack cases (benches/stack.rs: 50/50 push/pop, 50,000 initial elements) follow.
// Build: g++ -O2 -std=c++17 -pthread microbench/combiner_bench.cpp -o microbench/combiner_bench \
//            -Lnode-replication_amd/lib -lnrgpu -Wl,-rpath,$ORIGIN/../node-replication_amd/lib
// Run:   ./microbench/combiner_bench [seconds [threads ops/call kind(0 hashmap, 1 stack)] ...]
#include <sched.h>
#include <sys/resource.h>

#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/nrgpu.h"
#include "../include/nrgpu_testing.h"

static uint64_t sm64(uint64_t& s) {  // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int run(int threads, int batch, double secs, bool stack, int spin, int depth) {
    nrg_config cfg;
    nrg_config_default(&cfg, stack ? NRG_DS_STACK : NRG_DS_HASHMAP);
    cfg.log2_slots = 26;
    cfg.max_batch = cfg.max_reads = 1u << 16;
    cfg.stack_capacity = 1u << 26;
    nrg_ctx* ctx = nullptr;
    if (int r = nrg_open(0, &cfg, &ctx)) return r;
    if (stack) {
        std::vector<uint32_t> init(50000);
        for (uint32_t i = 0; i < 50000; i++) init[i] = i;
        if (int r = nrg_stack_init(ctx, init.data(), init.size())) return r;
    } else if (int r = nrg_hashmap_prefill_range(ctx, 1ull << 23, 1)) {
        return r;
    }
    if (spin >= 0)
        if (int r = nrg_test_set_knob(ctx, NRG_KNOB_COMB_SPIN, (uint64_t)spin)) return r;
    if (depth > 0)
        if (int r = nrg_test_set_knob(ctx, NRG_KNOB_COMB_DEPTH, (uint64_t)depth)) return r;
    if (const char* g = std::getenv("CB_GATHER"))  // (this tool's own setting: the gather window, us)
        if (int r = nrg_test_set_knob(ctx, NRG_KNOB_COMB_GATHER, std::strtoull(g, nullptr, 10))) return r;
    if (const char* g = std::getenv("CB_SERVE"))  // (this tool's own setting: the round server on / off)
        if (int r = nrg_test_set_knob(ctx, NRG_KNOB_COMB_SERVE, std::strtoull(g, nullptr, 10))) return r;
    nrg_combiner* comb = nullptr;
    if (int r = nrg_combiner_open(ctx, (uint32_t)threads, &comb)) return r;
    std::atomic<bool> stop{false};
    std::atomic<int> err{0};
    std::vector<uint64_t> done(threads, 0);
    std::atomic<uint64_t> usr_us{0}, sys_us{0};  // client threads' CPU time (getrusage per thread)
    std::vector<std::thread> th;
    for (int i = 0; i < threads; i++)
        th.emplace_back([&, i] {
            uint32_t tok = 0;
            if (nrg_combiner_register(comb, &tok)) {
                err = 1;
                return;
            }
            uint64_t s = 1000 + i, k[32], v[32], out[32];
            uint8_t f[32];
            nrg_stack_op so[32];
            uint64_t calls = 0, n = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                int r;
                if (stack) {  // benches/stack.rs:87-102: push or pop with equal odds
                    for (int j = 0; j < batch; j++) {
                        const uint64_t x = sm64(s);
                        so[j] = nrg_stack_op{(uint32_t)(x >> 32), (uint32_t)(x & 1)};
                    }
                    r = nrg_combiner_execute_mut(comb, tok, so, batch, out, f);
                } else {
                    for (int j = 0; j < batch; j++) {
                        k[j] = sm64(s) % 10000000ull;
                        v[j] = k[j] + 7;
                    }
                    r = calls++ % 10 == 0 ? nrg_combiner_put(comb, tok, k, v, batch, out, f)
                                          : nrg_combiner_get(comb, tok, k, batch, out, f);
                }
                if (r) {
                    err = r;
                    return;
                }
                n += batch;
            }
            done[i] = n;
            rusage ru;
            if (getrusage(RUSAGE_THREAD, &ru) == 0) {
                usr_us += (uint64_t)ru.ru_utime.tv_sec * 1000000 + ru.ru_utime.tv_usec;
                sys_us += (uint64_t)ru.ru_stime.tv_sec * 1000000 + ru.ru_stime.tv_usec;
            }
        });
    const auto t0 = std::chrono::steady_clock::now();
    std::this_thread::sleep_for(std::chrono::duration<double>(secs));
    stop = true;
    for (auto& x : th) x.join();
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t rounds = 0, ops = 0, tot = 0;
    nrg_combiner_stats(comb, &rounds, &ops);
    for (uint64_t d : done) tot += d;
    std::printf("%s threads %4d ops/call %3d spin %3d depth %d: %9.3f Mops/s  rounds %7llu  ops/round %7.1f  round rate %6.1f k/s%s\n",
                stack ? "stack  " : "hashmap", threads, batch, spin, depth, tot / dt / 1e6, (unsigned long long)rounds,
                rounds ? (double)ops / rounds : 0.0, rounds / dt / 1e3, err ? "  ERROR" : "");
    std::printf("        clients' CPU: user %.2f s, system %.2f s\n", usr_us.load() / 1e6, sys_us.load() / 1e6);
    uint64_t tm[4] = {0, 0, 0, 0};
    if (nrg_test_combiner_times(comb, tm) == 0 && tm[0])
        std::printf("        per round (us): gather %.2f  seal->enqueued %.2f  enqueued->done %.2f\n", tm[1] / 1e3 / tm[0],
                    tm[2] / 1e3 / tm[0], tm[3] / 1e3 / tm[0]);
    std::fflush(stdout);
    nrg_combiner_close(comb);
    nrg_close(ctx);
    return err.load();
}

// cgroup v2 cpu.stat: CPU time used and how often the group's quota throttled it
struct Throttle {
    bool ok = false;
    unsigned long long usage_us = 0, nr_periods = 0, nr_throttled = 0, throttled_us = 0;
};
static Throttle throttle() {
    Throttle t;
    FILE* f = std::fopen("/sys/fs/cgroup/cpu.stat", "r");
    if (!f) return t;
    char k[64];
    unsigned long long v;
    while (std::fscanf(f, "%63s %llu", k, &v) == 2) {
        if (!std::strcmp(k, "usage_usec")) t.usage_us = v, t.ok = true;
        if (!std::strcmp(k, "nr_periods")) t.nr_periods = v;
        if (!std::strcmp(k, "nr_throttled")) t.nr_throttled = v;
        if (!std::strcmp(k, "throttled_usec")) t.throttled_us = v;
    }
    std::fclose(f);
    return t;
}

static void show_cpus() {  // what the host gives this process: affinity and cgroup CPU quota
    cpu_set_t set;
    const int aff = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : -1;
    char q[64] = "none";
    const char* files[] = {"/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"};
    for (const char* fn : files)
        if (FILE* f = std::fopen(fn, "r")) {
            if (!std::fgets(q, sizeof(q), f)) q[0] = 0;
            std::fclose(f);
            break;
        }
    std::printf("cpus: hardware %u affinity %d cgroup quota %s\n", std::thread::hardware_concurrency(), aff, q);
}

int main(int argc, char** argv) {
    // combiner_bench [seconds [threads ops/call kind spin depth] ...]  (kind 0 hashmap, 1 stack;
    // spin -1 and depth 0: the library's defaults); without cases: the default set
    const double secs = argc > 1 ? std::atof(argv[1]) : 2.0;
    show_cpus();
    std::vector<std::array<int, 5>> cases = {{8, 1, 0, -1, 0},   {8, 32, 0, -1, 0},  {16, 32, 0, -1, 0},
                                             {64, 1, 0, -1, 0},  {64, 32, 0, -1, 0}, {128, 32, 0, -1, 0},
                                             {256, 32, 0, -1, 0}, {16, 32, 1, -1, 0}, {64, 32, 1, -1, 0},
                                             {256, 32, 1, -1, 0}};
    if (argc > 6) {
        cases.clear();
        for (int i = 2; i + 4 < argc; i += 5)
            cases.push_back({std::atoi(argv[i]), std::atoi(argv[i + 1]), std::atoi(argv[i + 2]), std::atoi(argv[i + 3]),
                             std::atoi(argv[i + 4])});
    }
    for (auto& c : cases) {
        const Throttle t0 = throttle();
        if (int r = run(c[0], c[1], secs, c[2] != 0, c[3], c[4])) {
            std::printf("error %d (%s)\n", r, nrg_strerror(r));
            return 1;
        }
        const Throttle t1 = throttle();
        if (t0.ok && t1.ok)
            std::printf("        cgroup: throttled %llu of %llu periods, %.1f ms throttled, %.2f CPU-s used\n",
                        (unsigned long long)(t1.nr_throttled - t0.nr_throttled), (unsigned long long)(t1.nr_periods - t0.nr_periods),
                        (t1.throttled_us - t0.throttled_us) / 1e3, (t1.usage_us - t0.usage_us) / 1e6);
    }
    return 0;
}
