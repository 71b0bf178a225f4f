/*
 * tune_copy.hip - A/B of the device copy (copy_row in dev_combine.hip: the
 * engine's init and final copies, the all-gather and the push copies): one
 * 16-B non-temporal vector per lane per wave (the product) against U vectors
 * per lane (more bytes in flight per wave), and the runtime's
 * hipMemcpyAsync D2D. Every variant's output is checked against the source.
 *
 *   tune_copy [log2 bytes = 28] [rounds = 5]
 *
 * Built by `make -C tools/src` into tools/ (not part of the product).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "dev_kernels.h"

using namespace ucgdev;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <int U, int NTL, int NTS>
__global__ void __launch_bounds__(64)
k_copy_var(u32x4 *dst, const u32x4 *src, size_t nvec)
{
    const size_t base = (size_t)blockIdx.x * 64 * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        if (base + u * 64 < nvec) {
            v[u] = ld16<NTL>(src + base + u * 64);
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        if (base + u * 64 < nvec) {
            st16<NTS>(dst + base + u * 64, v[u]);
        }
    }
}

struct Variant {
    std::string name;
    std::function<void(u32x4*, const u32x4*, size_t, hipStream_t)> run;
    std::vector<float> us;
};

int main(int argc, char **argv)
{
    const int lg     = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int iters  = 20;
    const size_t bytes = (size_t)1 << lg, nvec = bytes / 16;
    char *pair;
    /* source and destination as the two halves of one allocation (the
     * bench's layout for the combine) */
    CHECK(hipMalloc(&pair, 2 * bytes));
    u32x4 *src = reinterpret_cast<u32x4*>(pair), *dst = reinterpret_cast<u32x4*>(pair + bytes);
    hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                       (void*)src, 1, 7ull, bytes / 4);
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    CHECK(hipDeviceSynchronize());

    std::vector<Variant> vs;
#define VAR(U, NTL, NTS, W)                                                              \
    vs.push_back({"copy U" #U " ntl" #NTL " nts" #NTS " cap" #W,                          \
                  [=](u32x4 *d, const u32x4 *s, size_t nv, hipStream_t q) {              \
        const size_t lds = (W) ? (size_t)163840 / (W) / 512 * 512 : 0;                    \
        hipLaunchKernelGGL((k_copy_var<U, NTL, NTS>), dim3((unsigned)((nv + 64 * (U) - 1) / (64 * (U)))), \
                           dim3(64), lds, q, d, s, nv);                                  \
    }, {}})
    VAR(1, 1, 1, 0);
    VAR(2, 1, 1, 0);
    VAR(4, 1, 1, 0);
    VAR(2, 1, 1, 16);
    VAR(2, 1, 1, 24);
    VAR(4, 1, 1, 8);
    VAR(4, 1, 1, 16);
    VAR(1, 0, 1, 0);
    VAR(2, 0, 1, 0);
#undef VAR
    vs.push_back({"hipMemcpyAsync D2D", [=](u32x4 *d, const u32x4 *s, size_t nv, hipStream_t q) {
        (void)hipMemcpyAsync(d, s, nv * 16, hipMemcpyDeviceToDevice, q);
    }, {}});

    std::vector<uint32_t> want(bytes / 4), got(bytes / 4);
    CHECK(hipMemcpy(want.data(), src, bytes, hipMemcpyDeviceToHost));
    for (auto &v : vs) {
        CHECK(hipMemset(dst, 0, bytes));
        v.run(dst, src, nvec, st);
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpy(got.data(), dst, bytes, hipMemcpyDeviceToHost));
        if (memcmp(got.data(), want.data(), bytes) != 0) {
            printf("MISMATCH %s\n", v.name.c_str());
            return 3;
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; r++) {
        for (auto &v : vs) {
            v.run(dst, src, nvec, st);
            CHECK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; i++) {
                v.run(dst, src, nvec, st);
            }
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            v.us.push_back(1000.f * ms / iters);
        }
    }
    printf("copy of %zu MiB (2x bytes moved), %d rounds x %d iters\n", bytes >> 20, rounds, iters);
    for (auto &v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double med = v.us[v.us.size() / 2];
        printf("%-34s median %9.2f us  %7.0f GB/s  %5.1f%% of 8 TB/s\n", v.name.c_str(), med,
               2.0 * bytes / (med * 1e-6) / 1e9, 100.0 * 2.0 * bytes / (med * 1e-6) / 8e12);
    }
    return 0;
}
