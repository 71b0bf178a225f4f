/*
 * tune_alloc.hip - is the headline kernel's throughput a property of the
 * allocation? Times the product combine on fresh operand pairs of several
 * sizes, allocated with plain hipMalloc and with hipDeviceMallocContiguous,
 * several trials each (interleaved), median of 20 launches per pair.
 *
 *   tune_alloc [trials = 4]
 *
 * Built by `make -C xucg_amd/csrc tune` into tools/ (not part of the product).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dev_kernels.h"

using namespace ucgdev;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static float time_pair(float *d, const float *s, size_t n, hipStream_t st)
{
    const size_t nvec = n / 4;
    const unsigned g = (unsigned)((nvec + kReduceBlock - 1) / kReduceBlock);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int r = 0; r < 5; r++) {
        hipLaunchKernelGGL((k_reduce<float, 0, kReduceU, 1, kReduceBlock>), dim3(g),
                           dim3(kReduceBlock), 0, st, d, s, (size_t)0, nvec, (size_t)0);
        CHECK(hipEventRecord(e0, st));
        for (int i = 0; i < 20; i++) {
            hipLaunchKernelGGL((k_reduce<float, 0, kReduceU, 1, kReduceBlock>), dim3(g),
                               dim3(kReduceBlock), 0, st, d, s, (size_t)0, nvec, (size_t)0);
        }
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float t;
        CHECK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t / 20);
    }
    std::sort(ms.begin(), ms.end());
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return ms[ms.size() / 2];
}

int main(int argc, char **argv)
{
    const int trials = argc > 1 ? atoi(argv[1]) : 4;
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    const size_t sizes[] = {(size_t)1 << 26, (size_t)1 << 28};   /* elements */
    const unsigned flags[] = {hipDeviceMallocDefault, hipDeviceMallocContiguous};
    const char *fname[] = {"hipMalloc", "contiguous"};
    for (int t = 0; t < trials; t++) {
        for (size_t n : sizes) {
            for (int f = 0; f < 2; f++) {
                float *s = nullptr, *d = nullptr;
                if (hipExtMallocWithFlags((void**)&s, n * 4, flags[f]) != hipSuccess ||
                    hipExtMallocWithFlags((void**)&d, n * 4, flags[f]) != hipSuccess) {
                    printf("trial %d %4zu MiB %-10s allocation failed\n", t, n * 4 >> 20,
                           fname[f]);
                    (void)hipGetLastError();
                    if (s) (void)hipFree(s);
                    continue;
                }
                CHECK(hipMemset(s, 0, n * 4));
                CHECK(hipMemset(d, 0, n * 4));
                const float ms = time_pair(d, s, n, st);
                printf("trial %d %4zu MiB %-10s %8.1f us  %5.1f%% of 8 TB/s\n", t,
                       n * 4 >> 20, fname[f], ms * 1e3, 100.0 * 3 * n * 4 / (ms * 1e-3) / 8e12);
                CHECK(hipFree(s));
                CHECK(hipFree(d));
            }
        }
    }
    return 0;
}
