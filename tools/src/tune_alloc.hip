/*
 * tune_alloc.hip - is the headline kernel's throughput a property of the
 * allocation? Times the product combine on fresh operand pairs of several
 * sizes, allocated with plain hipMalloc and with hipDeviceMallocContiguous,
 * several trials each (interleaved), median of 20 launches per pair.
 *
 *   tune_alloc [trials = 4]
 *
 * Built by `make -C tools/src` into tools/ (not part of the product).
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

/* VMM allocation: one physical chunk of `bytes` (rounded to the minimum
 * granularity) mapped into a fresh VA range */
static void *vmm_alloc(size_t bytes, size_t *mapped)
{
    hipMemAllocationProp prop = {};
    prop.type          = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id   = 0;
    size_t gran = 0;
    CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    const size_t sz = (bytes + gran - 1) / gran * gran;
    hipMemGenericAllocationHandle_t h;
    CHECK(hipMemCreate(&h, sz, &prop, 0));
    void *va = nullptr;
    CHECK(hipMemAddressReserve(&va, sz, 0, nullptr, 0));
    CHECK(hipMemMap(va, sz, 0, h, 0));
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags    = hipMemAccessFlagsProtReadWrite;
    CHECK(hipMemSetAccess(va, sz, &acc, 1));
    CHECK(hipMemRelease(h));      /* the mapping keeps it alive */
    *mapped = sz;
    return va;
}

static void vmm_free(void *va, size_t sz)
{
    CHECK(hipMemUnmap(va, sz));
    CHECK(hipMemAddressFree(va, sz));
}

/* scenario mode (argv[1] = "scen"): the same 256 MiB pair shape allocated
 * after different histories of the device heap, interleaved over trials */
static int scenarios(int trials)
{
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    const size_t n = (size_t)1 << 26, nb = n * 4;
    for (int t = 0; t < trials; t++) {
        float *s, *d;
        /* S1: fresh hipMalloc */
        CHECK(hipMalloc(&s, nb));
        CHECK(hipMalloc(&d, nb));
        CHECK(hipMemset(s, 0, nb));
        CHECK(hipMemset(d, 0, nb));
        printf("trial %d S1 fresh hipMalloc          %5.1f%%\n", t,
               100.0 * 3 * nb / (time_pair(d, s, n, st) * 1e-3) / 8e12);
        CHECK(hipFree(s));
        CHECK(hipFree(d));
        /* S2: after a freed 1 GiB pair */
        {
            float *a, *b;
            CHECK(hipMalloc(&a, nb * 4));
            CHECK(hipMalloc(&b, nb * 4));
            CHECK(hipMemset(a, 0, nb * 4));
            CHECK(hipMemset(b, 0, nb * 4));
            CHECK(hipFree(a));
            CHECK(hipFree(b));
        }
        CHECK(hipMalloc(&s, nb));
        CHECK(hipMalloc(&d, nb));
        CHECK(hipMemset(s, 0, nb));
        CHECK(hipMemset(d, 0, nb));
        printf("trial %d S2 after freed 1 GiB pair   %5.1f%%\n", t,
               100.0 * 3 * nb / (time_pair(d, s, n, st) * 1e-3) / 8e12);
        CHECK(hipFree(s));
        CHECK(hipFree(d));
        /* S3: a heap with holes: 96 x 8 MiB, every other one freed */
        {
            std::vector<void*> v(96);
            for (auto &p : v) CHECK(hipMalloc(&p, 8u << 20));
            for (size_t i = 0; i < v.size(); i += 2) CHECK(hipFree(v[i]));
            CHECK(hipMalloc(&s, nb));
            CHECK(hipMalloc(&d, nb));
            CHECK(hipMemset(s, 0, nb));
            CHECK(hipMemset(d, 0, nb));
            printf("trial %d S3 heap with 8 MiB holes    %5.1f%%\n", t,
                   100.0 * 3 * nb / (time_pair(d, s, n, st) * 1e-3) / 8e12);
            CHECK(hipFree(s));
            CHECK(hipFree(d));
            for (size_t i = 1; i < v.size(); i += 2) CHECK(hipFree(v[i]));
        }
        /* S4: VMM physical chunks */
        {
            size_t ms_, md_;
            s = (float*)vmm_alloc(nb, &ms_);
            d = (float*)vmm_alloc(nb, &md_);
            CHECK(hipMemset(s, 0, nb));
            CHECK(hipMemset(d, 0, nb));
            printf("trial %d S4 VMM hipMemCreate/Map     %5.1f%%\n", t,
                   100.0 * 3 * nb / (time_pair(d, s, n, st) * 1e-3) / 8e12);
            vmm_free(s, ms_);
            vmm_free(d, md_);
        }
        /* S5: contiguous flag */
        CHECK(hipExtMallocWithFlags((void**)&s, nb, hipDeviceMallocContiguous));
        CHECK(hipExtMallocWithFlags((void**)&d, nb, hipDeviceMallocContiguous));
        CHECK(hipMemset(s, 0, nb));
        CHECK(hipMemset(d, 0, nb));
        printf("trial %d S5 hipDeviceMallocContiguous %5.1f%%\n", t,
               100.0 * 3 * nb / (time_pair(d, s, n, st) * 1e-3) / 8e12);
        CHECK(hipFree(s));
        CHECK(hipFree(d));
    }
    return 0;
}

int main(int argc, char **argv)
{
    if (argc > 1 && argv[1][0] == 's') {
        return scenarios(argc > 2 ? atoi(argv[2]) : 4);
    }
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
