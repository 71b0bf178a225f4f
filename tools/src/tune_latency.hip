/*
 * tune_latency.hip - A/B harness for the small-step floor of the staged
 * combine (not part of the product libraries): one small device-resident
 * combine launched, then the host waits for it, by each of
 *
 *   sync      hipStreamSynchronize (what ucg_builtin_dev_stage_end does)
 *   query     spin on hipStreamQuery
 *   event     hipEventRecord + hipEventSynchronize
 *   flag      spin on a pinned host word that the kernel's last workgroup
 *             writes (agent-scope counter, system-scope release store)
 *   graph     the same kernel as a one-node hipGraph, hipGraphLaunch + sync
 *   empty     an empty kernel + hipStreamSynchronize (launch + wait only)
 *   launch    launches only, one sync at the end (per-launch host cost)
 *
 *   hipcc -O3 --offload-arch=gfx950 -I../../include tune_latency.hip -o tune
 *   ./tune_latency [bytes=4096] [iters=2000] [rounds=7]
 *
 * Methods are interleaved over rounds; median us per step is printed.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "dev_kernels.h"

using namespace ucgdev;

#define CHECK(x)                                                               \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,          \
                    hipGetErrorString(e_));                                    \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

__global__ void __launch_bounds__(64) k_empty() {}

/* the product's combine shape (one wave per workgroup, one 16-B vector per
 * lane), plus a completion word: every workgroup releases its stores at
 * agent scope and counts itself; the last one resets the counter and
 * publishes `seq` to pinned host memory with a system-scope release */
__global__ void __launch_bounds__(64)
k_combine_flag(float *dst, const float *src, size_t nvec, unsigned *counter,
               unsigned *host_flag, unsigned seq)
{
    const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (i < nvec) {
        const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
        u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
        st16<1>(d4 + i, vapply<float, 0>(ld16<1>(s4 + i), ld16<1>(d4 + i)));
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) {
            __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   /* system scope */
            /* the compiler may drop the wait after the write-back when the
             * scoreboard looks empty (MI355X_MICROARCH.md, compiler hazard) */
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(host_flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

/* a one-workgroup kernel queued behind any stream work (a combine, a D2H
 * copy): stream order means everything before it has completed; the
 * system-scope release makes the pinned word the host's completion signal */
__global__ void __launch_bounds__(64) k_signal(unsigned *host_flag, unsigned seq)
{
    if (threadIdx.x == 0) {
        __hip_atomic_store(host_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static void spin_flag(volatile unsigned *flag, unsigned s, hipStream_t st, const char *who)
{
    long spins = 0;
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != s) {
        if (++spins == (1L << 28)) {   /* seconds, not microseconds */
            fprintf(stderr, "%s: flag %u never arrived\n", who, s);
            (void)hipStreamSynchronize(st);
            exit(2);
        }
    }
}

static double now_us()
{
    return std::chrono::duration<double, std::micro>(
        std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Method {
    std::string name;
    std::function<void()> step;
    std::vector<double> us;
};

int main(int argc, char **argv)
{
    const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 0) : 4096;
    const int iters    = argc > 2 ? atoi(argv[2]) : 2000;
    const int rounds   = argc > 3 ? atoi(argv[3]) : 7;
    const size_t nvec  = bytes / 16;
    const unsigned grid = (unsigned)((nvec + 63) / 64);
    float *src, *dst;
    unsigned *counter, *flag;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMemset(src, 0, bytes));
    CHECK(hipMemset(dst, 0, bytes));
    CHECK(hipMalloc(&counter, sizeof(unsigned)));
    CHECK(hipMemset(counter, 0, sizeof(unsigned)));
    CHECK(hipHostMalloc((void**)&flag, sizeof(unsigned), hipHostMallocDefault));
    *flag = 0;
    void *hbuf;
    CHECK(hipHostMalloc(&hbuf, 256, hipHostMallocDefault));
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t ev;
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    unsigned seq = 0;

    auto launch = [&]() {
        hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, 64>), dim3(grid), dim3(64), 0, st,
                           dst, (const float*)src, (size_t)0, nvec, (size_t)0);
    };
    hipGraph_t graph;
    hipGraphExec_t gexec;
    CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    launch();
    CHECK(hipStreamEndCapture(st, &graph));
    CHECK(hipGraphInstantiate(&gexec, graph, nullptr, nullptr, 0));

    std::vector<Method> ms;
    ms.push_back({"sync   (launch + hipStreamSynchronize)", [&]() {
        launch();
        CHECK(hipStreamSynchronize(st));
    }, {}});
    ms.push_back({"query  (launch + spin hipStreamQuery)", [&]() {
        launch();
        while (hipStreamQuery(st) == hipErrorNotReady) {
        }
    }, {}});
    ms.push_back({"event  (launch + record + hipEventSynchronize)", [&]() {
        launch();
        CHECK(hipEventRecord(ev, st));
        CHECK(hipEventSynchronize(ev));
    }, {}});
    ms.push_back({"flag   (launch + spin on pinned completion word)", [&]() {
        const unsigned s = ++seq;
        hipLaunchKernelGGL(k_combine_flag, dim3(grid), dim3(64), 0, st, dst,
                           (const float*)src, nvec, counter, flag, s);
        long spins = 0;
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != s) {
            if (++spins == (1L << 28)) {   /* seconds, not microseconds */
                fprintf(stderr, "flag %u never arrived\n", s);
                CHECK(hipStreamSynchronize(st));
                exit(2);
            }
        }
    }, {}});
    ms.push_back({"sig    (launch + 1-WG signal kernel + spin on word)", [&]() {
        const unsigned s = ++seq;
        launch();
        hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, st, flag, s);
        spin_flag(flag, s, st, "sig");
    }, {}});
    ms.push_back({"wv32   (launch + hipStreamWriteValue32 + spin on word)", [&]() {
        const unsigned s = ++seq;
        launch();
        CHECK(hipStreamWriteValue32(st, flag, s, 0));
        spin_flag(flag, s, st, "wv32");
    }, {}});
    ms.push_back({"d2hsig (launch + 256-B D2H + signal kernel + spin)", [&]() {
        const unsigned s = ++seq;
        launch();
        CHECK(hipMemcpyAsync(hbuf, dst, 256, hipMemcpyDeviceToHost, st));
        hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, st, flag, s);
        spin_flag(flag, s, st, "d2hsig");
    }, {}});
    ms.push_back({"d2hsyn (launch + 256-B D2H + hipStreamSynchronize)", [&]() {
        launch();
        CHECK(hipMemcpyAsync(hbuf, dst, 256, hipMemcpyDeviceToHost, st));
        CHECK(hipStreamSynchronize(st));
    }, {}});
    ms.push_back({"graph  (hipGraphLaunch + hipStreamSynchronize)", [&]() {
        CHECK(hipGraphLaunch(gexec, st));
        CHECK(hipStreamSynchronize(st));
    }, {}});
    ms.push_back({"empty  (empty kernel + hipStreamSynchronize)", [&]() {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
        CHECK(hipStreamSynchronize(st));
    }, {}});
    ms.push_back({"launch (launch only; one sync per round)", [&]() {
        launch();
    }, {}});

    for (int r = 0; r < rounds; r++) {
        for (auto &m : ms) {
            for (int i = 0; i < 50; i++) {
                m.step();
            }
            CHECK(hipStreamSynchronize(st));
            const double t0 = now_us();
            for (int i = 0; i < iters; i++) {
                m.step();
            }
            CHECK(hipStreamSynchronize(st));
            m.us.push_back((now_us() - t0) / iters);
        }
    }
    CHECK(hipStreamSynchronize(st));
    printf("bytes=%zu grid=%u iters=%d rounds=%d\n", bytes, grid, iters, rounds);
    for (auto &m : ms) {
        std::sort(m.us.begin(), m.us.end());
        printf("%-52s med %7.2f us  min %7.2f  max %7.2f\n", m.name.c_str(),
               m.us[m.us.size() / 2], m.us.front(), m.us.back());
    }
    CHECK(hipGraphExecDestroy(gexec));
    CHECK(hipGraphDestroy(graph));
    return 0;
}
