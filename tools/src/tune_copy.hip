/*
 * tune_copy.hip - A/B of the all-gather's row copy (copy_row in
 * dev_combine.hip, k_gather_multi's in-phase path) against the same copy with
 * the next tile's first lines loaded ahead (the combine's PF form, issued
 * before or after the tile's own load).
 *
 *   tune_copy [log2 bytes per row = 26] [rounds = 9]
 *
 * 8 rows in one allocation, the gather's grid: workgroup b copies tile b / 8
 * of row b % 8 (dealt round-robin over the rows, so row r runs on XCD r and a
 * row's next tile is its own XCD's). Output checked bit for bit, then the
 * variants run interleaved over rounds, 20 launches per sample, HIP events;
 * 2 x the bytes moved per launch.
 *
 * Built by `make -C tools/src` into tools/ (not part of the product).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dev_kernels.h"

using namespace ucgdev;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr unsigned kRows = 8;

/* PF 0: the product's aligned row copy; PF > 0: lanes 63 .. 64 - PF also load
 * the first PF lines of the row's tile D ahead (temporal, discarded), FIRST
 * = 1 before the tile's own load */
template <int PF, int D, int FIRST>
__global__ void __launch_bounds__(kReduceBlock)
k_copy_rows(char *dst, const char *src, size_t row_bytes)
{
    const unsigned r  = blockIdx.x % kRows;
    const size_t wg   = blockIdx.x / kRows;
    const size_t nvec = row_bytes / 16;
    const size_t i    = wg * kReduceBlock + threadIdx.x;
    const u32x4 *s4   = reinterpret_cast<const u32x4*>(src + (size_t)r * row_bytes);
    u32x4 *o4         = reinterpret_cast<u32x4*>(dst + (size_t)r * row_bytes);
    const size_t ic   = i < nvec ? i : nvec - 1;
    u32x4 v, pf;
    if constexpr (PF > 0) {
        const unsigned k  = kReduceBlock - 1 - threadIdx.x;
        const size_t want = (i - threadIdx.x + (size_t)D * kReduceBlock) + (size_t)k * 8;
        const u32x4 *at   = s4 + (k < (unsigned)PF && want < nvec ? want : nvec - 1);
        if constexpr (FIRST) {
            pf = ld16<0>(at);
            __builtin_amdgcn_sched_barrier(0);
            v  = ld16<1>(s4 + ic);
        } else {
            v  = ld16<1>(s4 + ic);
            __builtin_amdgcn_sched_barrier(0);
            pf = ld16<0>(at);
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" :: "v"(pf[0]));
    } else {
        v = ld16<1>(s4 + ic);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (i < nvec) {
        st16<1>(o4 + i, v);
    }
}

struct Variant {
    std::string name;
    void (*f)(char *, const char *, size_t, hipStream_t);
    std::vector<float> ms;
};

template <int PF, int D, int FIRST>
static void run(char *d, const char *s, size_t rb, hipStream_t q)
{
    const size_t tiles = (rb / 16 + kReduceBlock - 1) / kReduceBlock;
    hipLaunchKernelGGL((k_copy_rows<PF, D, FIRST>), dim3((unsigned)(tiles * kRows)),
                       dim3(kReduceBlock), 0, q, d, s, rb);
}

__global__ void k_init(uint32_t *p, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        p[i] = (uint32_t)(i * 2654435761u);
    }
}

int main(int argc, char **argv)
{
    const int lg     = argc > 1 ? atoi(argv[1]) : 26;
    const int rounds = argc > 2 ? atoi(argv[2]) : 9;
    const int iters  = 20;
    const size_t rb = (size_t)1 << lg, total = rb * kRows;
    std::vector<Variant> vs = {
        {"product row copy (no prefetch)", run<0, 1, 0>, {}},
        {"PF1 next tile, after", run<1, 1, 0>, {}},
        {"PF1 next tile, first", run<1, 1, 1>, {}},
        {"PF3 next tile, after", run<3, 1, 0>, {}},
        {"PF3 next tile, first", run<3, 1, 1>, {}},
        {"PF1 2 tiles ahead, first", run<1, 2, 1>, {}},
        {"PF3 2 tiles ahead, first", run<3, 2, 1>, {}},
    };
    char *arena;
    CHECK(hipMalloc(&arena, 2 * total));
    char *src = arena, *dst = arena + total;
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipLaunchKernelGGL(k_init, dim3((unsigned)((total / 4 + 255) / 256)), dim3(256), 0, st,
                       reinterpret_cast<uint32_t*>(src), total / 4);
    CHECK(hipStreamSynchronize(st));
    {
        std::vector<char> hs(total), hd(total);
        CHECK(hipMemcpy(hs.data(), src, total, hipMemcpyDeviceToHost));
        for (auto &v : vs) {
            CHECK(hipMemset(dst, 0, total));
            v.f(dst, src, rb, st);
            CHECK(hipStreamSynchronize(st));
            CHECK(hipMemcpy(hd.data(), dst, total, hipMemcpyDeviceToHost));
            if (memcmp(hs.data(), hd.data(), total) != 0) {
                printf("MISMATCH %s\n", v.name.c_str());
                return 3;
            }
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (auto &v : vs) {
        for (int i = 0; i < 3; i++) {
            v.f(dst, src, rb, st);
        }
    }
    for (int r = 0; r < rounds; r++) {
        for (auto &v : vs) {
            v.f(dst, src, rb, st);
            CHECK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; i++) {
                v.f(dst, src, rb, st);
            }
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms / iters);
        }
    }
    printf("row copy, %u rows of %zu MiB (the gather's grid), %d rounds x %d\n", kRows,
           rb >> 20, rounds, iters);
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2];
        printf("%-34s median %8.2f us  min %8.2f  %5.1f%% of 8 TB/s\n", v.name.c_str(),
               med * 1e3, v.ms.front() * 1e3, 100.0 * 2.0 * total / (med * 1e-3) / 8e12);
    }
    return 0;
}
