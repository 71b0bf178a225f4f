/*
 * tune_multi.hip - A/B harness for the one-shot multi-operand combine
 * (k_reduce_multi, N = 8 fp32 SUM, the C4 one-shot reduce-scatter shape) on
 * one GPU: every variant reads the same N local operands and writes one
 * output; runs are interleaved over rounds; every variant's output is
 * checked bit for bit against the product kernel's.
 *
 *   tune_multi [log2 elements per operand = 26] [rounds = 5]
 *
 * Built by `make -C xucg_amd/csrc tune` into tools/ (not part of the product).
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

constexpr int N = 8;

/* U vectors per lane; CONTIG = 1 gives a lane U adjacent vectors, else the
 * lane's vectors are BS apart; NTL = non-temporal loads */
template <int U, int BS, int NTL, int CONTIG>
__global__ void __launch_bounds__(BS)
k_multi_var(float *dst, SrcList srcs, unsigned self, size_t nvec)
{
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    u32x4 val[U][N];
    size_t idx[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        idx[u] = CONTIG ? ((size_t)blockIdx.x * BS + threadIdx.x) * U + u
                        : (size_t)blockIdx.x * BS * U + (size_t)u * BS + threadIdx.x;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        if (idx[u] < nvec) {
#pragma unroll
            for (int m = 0; m < N; m++) {
                val[u][m] = ld16<NTL>(reinterpret_cast<const u32x4*>(srcs.p[self ^ m]) + idx[u]);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        if (idx[u] < nvec) {
            st16<1>(reinterpret_cast<u32x4*>(dst) + idx[u], rd_tree<N>(val[u], fv));
        }
    }
}

struct Variant {
    std::string name;
    std::function<void(float*, SrcList, size_t, hipStream_t)> run;
    std::vector<float> ms;
};

int main(int argc, char **argv)
{
    const int lg     = argc > 1 ? atoi(argv[1]) : 26;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int iters  = 10;
    const size_t n = (size_t)1 << lg, nvec = n / 4;
    SrcList srcs;
    std::vector<float*> bufs(N);
    for (int m = 0; m < N; m++) {
        CHECK(hipMalloc(&bufs[m], n * 4));
        std::vector<float> h(n);
        for (size_t i = 0; i < n; i++) {
            h[i] = (float)((int)((i * 2654435761u + m * 40503u) % 2049) - 1024);
        }
        CHECK(hipMemcpy(bufs[m], h.data(), n * 4, hipMemcpyHostToDevice));
    }
    for (int m = 0; m < kMaxMulti; m++) {
        srcs.p[m] = m < N ? bufs[m] : nullptr;
    }
    float *out, *ref;
    CHECK(hipMalloc(&out, n * 4));
    CHECK(hipMalloc(&ref, n * 4));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));

    std::vector<Variant> vs;
    vs.push_back({"product k_reduce_multi<f32,SUM,8> (bs64 U1 NT)",
                  [=](float *d, SrcList s, size_t nv, hipStream_t q) {
        unsigned g = (unsigned)((nv + kReduceBlock - 1) / kReduceBlock);
        hipLaunchKernelGGL((k_reduce_multi<float, 0, N>), dim3(g), dim3(kReduceBlock), 0, q,
                           d, s, 0u, (size_t)0, nv, (size_t)0);
    }, {}});
#define VAR(U, BS, NTL, CONTIG)                                                       \
    vs.push_back({"var U" #U " BS" #BS " NTL" #NTL " CONTIG" #CONTIG,                 \
                  [=](float *d, SrcList s, size_t nv, hipStream_t q) {                \
        unsigned g = (unsigned)((nv + (BS) * (U) - 1) / ((BS) * (U)));                \
        hipLaunchKernelGGL((k_multi_var<U, BS, NTL, CONTIG>), dim3(g), dim3(BS), 0, q, \
                           d, s, 0u, nv);                                             \
    }, {}})
    VAR(1, 64, 1, 0);
    VAR(2, 64, 1, 0);
    VAR(2, 64, 1, 1);
    VAR(1, 256, 1, 0);
    VAR(2, 256, 1, 0);
    VAR(1, 64, 0, 0);
    VAR(4, 64, 1, 0);
#undef VAR

    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    vs[0].run(ref, srcs, nvec, st);
    CHECK(hipStreamSynchronize(st));
    std::vector<float> hr(n), ho(n);
    CHECK(hipMemcpy(hr.data(), ref, n * 4, hipMemcpyDeviceToHost));
    for (auto &v : vs) {
        CHECK(hipMemset(out, 0, n * 4));
        v.run(out, srcs, nvec, st);
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpy(ho.data(), out, n * 4, hipMemcpyDeviceToHost));
        if (ho != hr) {
            printf("MISMATCH %s\n", v.name.c_str());
            return 3;
        }
    }
    for (int r = 0; r < rounds; r++) {
        for (auto &v : vs) {
            v.run(out, srcs, nvec, st);
            CHECK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; i++) {
                v.run(out, srcs, nvec, st);
            }
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms / iters);
        }
    }
    const double bytes = (double)(N + 1) * n * 4;
    printf("N=%d, %zu MiB per operand, (N+1)*S = %.0f MiB per launch\n", N, n * 4 >> 20,
           bytes / 1048576.0);
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        float med = v.ms[v.ms.size() / 2];
        printf("%-48s median %8.2f us  %7.1f GB/s  %5.1f%% of 8 TB/s\n", v.name.c_str(),
               med * 1e3, bytes / (med * 1e-3) / 1e9, 100.0 * bytes / (med * 1e-3) / 8e12);
    }
    return 0;
}
