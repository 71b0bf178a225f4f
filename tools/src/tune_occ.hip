/*
 * tune_occ.hip - occupancy A/B for the multi-operand kernels: how many
 * one-wave workgroups per CU the one-shot combines (k_reduce_multi, N
 * operands) and the tree fan-in (k_reduce_tree, n operands) should run with.
 * The cap is dynamic LDS the kernels do not use (160 KiB per CU, so at most
 * W workgroups fit). Every capped launch is checked bit for bit against the
 * uncapped one. Operands: 16 separate allocations of S bytes, fp32 SUM.
 *
 *   tune_occ [log2 elements per operand = 24] [rounds = 5]
 *
 * Built by `make -C tools/src` into tools/ (not part of the product).
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "dev_kernels.h"

using namespace ucgdev;

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static size_t lds_for(int w)
{
    return w ? (size_t)163840 / w / 512 * 512 : 0;
}

template <int N>
static void run_multi(float *d, const SrcList &s, size_t nv, size_t lds, hipStream_t q)
{
    const unsigned g = (unsigned)((nv + kReduceBlock - 1) / kReduceBlock);
    hipLaunchKernelGGL((k_reduce_multi<float, 0, N>), dim3(g), dim3(kReduceBlock), lds, q,
                       d, s, 0u, (size_t)0, nv, (size_t)0);
}

template <int NMAX>
static void run_tree(float *d, const SrcList &s, unsigned n, size_t nv, size_t lds,
                     hipStream_t q)
{
    const unsigned g = (unsigned)((nv + kReduceBlock - 1) / kReduceBlock);
    hipLaunchKernelGGL((k_reduce_tree<float, 0, NMAX>), dim3(g), dim3(kReduceBlock), lds, q,
                       d, s, n, (size_t)0, nv, (size_t)0);
}

struct Case {
    std::string name;
    int ops;                        /* operands read */
    int w;                          /* waves per CU cap, 0 = none */
    std::function<void(float*, size_t, hipStream_t)> run;
    std::vector<float> us;
};

int main(int argc, char **argv)
{
    const int lg     = argc > 1 ? atoi(argv[1]) : 24;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int iters  = 10;
    const size_t n = (size_t)1 << lg, nvec = n / 4;
    std::vector<float*> bufs(kMaxMulti);
    for (int m = 0; m < kMaxMulti; m++) {
        CHECK(hipMalloc(&bufs[m], n * 4));
        hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                           (void*)bufs[m], 0, 100ull + m, n);   /* "exact" values */
    }
    SrcList all;
    for (int m = 0; m < kMaxMulti; m++) {
        all.p[m] = bufs[m];
    }
    float *out, *ref;
    CHECK(hipMalloc(&out, n * 4));
    CHECK(hipMalloc(&ref, n * 4));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    CHECK(hipDeviceSynchronize());

    std::vector<Case> cs;
    /* TUNE_OCC_PMC=1: only N = 8 uncapped and at 8 waves per CU, for the
     * rocprofv3 counter passes (scripts/occ_pmc.sh) */
    const bool pmc = getenv("TUNE_OCC_PMC") != nullptr;
    if (pmc) {
        for (int w : {0, 8}) {
            const size_t lds = lds_for(w);
            cs.push_back({"multi N=8", 8, w, [=](float *d, size_t nv, hipStream_t q) { run_multi<8>(d, all, nv, lds, q); }, {}});
        }
        for (int r = 0; r < rounds; r++) {
            for (auto &c : cs) {
                c.run(out, nvec, st);
            }
        }
        CHECK(hipStreamSynchronize(st));
        printf("pmc mode: %d rounds of N=8 uncapped, then capped at 8\n", rounds);
        return 0;
    }
    const int caps[] = {0, 4, 6, 8, 10, 12, 14, 16, 20, 24, 28};
    for (int w : caps) {
        const size_t lds = lds_for(w);
        cs.push_back({"multi N=2", 2, w, [=](float *d, size_t nv, hipStream_t q) { run_multi<2>(d, all, nv, lds, q); }, {}});
        cs.push_back({"multi N=4", 4, w, [=](float *d, size_t nv, hipStream_t q) { run_multi<4>(d, all, nv, lds, q); }, {}});
        cs.push_back({"multi N=8", 8, w, [=](float *d, size_t nv, hipStream_t q) { run_multi<8>(d, all, nv, lds, q); }, {}});
        cs.push_back({"multi N=16", 16, w, [=](float *d, size_t nv, hipStream_t q) { run_multi<16>(d, all, nv, lds, q); }, {}});
        cs.push_back({"tree n=3 (NMAX 4)", 3, w, [=](float *d, size_t nv, hipStream_t q) { run_tree<4>(d, all, 3, nv, lds, q); }, {}});
        cs.push_back({"tree n=6 (NMAX 8)", 6, w, [=](float *d, size_t nv, hipStream_t q) { run_tree<8>(d, all, 6, nv, lds, q); }, {}});
        cs.push_back({"tree n=8 (NMAX 8)", 8, w, [=](float *d, size_t nv, hipStream_t q) { run_tree<8>(d, all, 8, nv, lds, q); }, {}});
        cs.push_back({"tree n=12 (NMAX 16)", 12, w, [=](float *d, size_t nv, hipStream_t q) { run_tree<16>(d, all, 12, nv, lds, q); }, {}});
    }

    std::vector<uint32_t> want(n), got(n);
    /* bits: each capped launch against the uncapped launch of the same kernel */
    int bad = 0;
    for (size_t base = 0; base < 8; base++) {
        CHECK(hipMemset(ref, 0, n * 4));
        cs[base].run(ref, nvec, st);
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpy(want.data(), ref, n * 4, hipMemcpyDeviceToHost));
        for (size_t k = base + 8; k < cs.size(); k += 8) {
            CHECK(hipMemset(out, 0, n * 4));
            cs[k].run(out, nvec, st);
            CHECK(hipStreamSynchronize(st));
            CHECK(hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost));
            if (got != want) {
                printf("MISMATCH %s cap %d\n", cs[k].name.c_str(), cs[k].w);
                bad = 1;
            }
        }
    }
    if (bad) {
        return 3;
    }

    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; r++) {
        for (auto &c : cs) {
            c.run(out, nvec, st);
            CHECK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; i++) {
                c.run(out, nvec, st);
            }
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            c.us.push_back(1000.f * ms / iters);
        }
    }
    printf("%zu MiB per operand, fp32 SUM, %% of 8 TB/s on (operands + 1) * S bytes\n",
           n * 4 >> 20);
    printf("%-22s", "kernel \\ waves/CU cap");
    for (int w : caps) {
        printf(w ? "%7d" : "   none", w);
    }
    printf("\n");
    for (size_t base = 0; base < 8; base++) {
        printf("%-22s", cs[base].name.c_str());
        for (size_t k = base; k < cs.size(); k += 8) {
            auto v = cs[k].us;
            std::sort(v.begin(), v.end());
            const double med = v[v.size() / 2];
            const double bytes = (double)(cs[k].ops + 1) * n * 4;
            printf("%7.1f", 100.0 * bytes / (med * 1e-6) / 8e12);
        }
        printf("\n");
    }
    return 0;
}
