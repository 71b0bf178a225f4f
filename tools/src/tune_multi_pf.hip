/*
 * tune_multi_pf.hip - A/B harness for the next-tile prefetch (k_reduce's PF
 * form) in the in-phase multi-operand kernels: k_reduce_multi
 * (the C4/C5 one-shot reduce-scatter's local fold, recursive-doubling
 * association) and k_reduce_tree (the tree plan's fan-in at its root).
 *
 *   tune_multi_pf multi N [log2 elements per operand = 24] [rounds = 5]
 *   tune_multi_pf tree  n [log2 elements per operand = 24] [rounds = 5]
 *
 * The operands and the output sit in one allocation, S apart (bench.py's
 * one_shot_shape layout). Every variant's output is checked bit for bit
 * against the round-4 product form's before timing; the variants then run
 * interleaved over rounds, 10 launches per sample, HIP events on the stream.
 * (N + 1) * S algorithmic bytes per launch.
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

struct Variant {
    std::string name;
    std::function<void(float*, SrcList, size_t, hipStream_t)> run;
    bool checked;
    std::vector<float> ms;
};

static unsigned tiles(size_t nvec) { return (unsigned)((nvec + kReduceBlock - 1) / kReduceBlock); }

/* the N operands read, nothing stored (the read ceiling of the same streams) */
template <int N>
__global__ void __launch_bounds__(kReduceBlock)
k_read_only(float *dst, SrcList srcs, size_t nvec)
{
    UCG_MULTI_CAP_CLOBBER();
    const size_t i = (size_t)blockIdx.x * kReduceBlock + threadIdx.x;
    if (i >= nvec) {
        return;
    }
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < N; m++) {
        acc ^= ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[m]) + i);
    }
    if (acc[0] == 0x7fc00123u && acc[1] == 0x7fc00321u) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + i, acc);
    }
}

template <int N>
static void add_multi(std::vector<Variant> &vs)
{
#define MV(label, XM, CAP, PF, PFM, CHK, ...)                                          \
    vs.push_back({label, [](float *d, SrcList s, size_t nv, hipStream_t q) {           \
        hipLaunchKernelGGL((k_reduce_multi<float, 0, N, XM, CAP, PF, PFM __VA_OPT__(,) __VA_ARGS__>), \
                           dim3(tiles(nv)), \
                           dim3(kReduceBlock), 0, q, d, s, 0u, (size_t)0, nv, (size_t)0); \
    }, CHK, {}})
    MV("round-4 product (capped, identity map)", 0, 1, 0, 0, true);
    MV("capped, XCD map, no prefetch", 1, 1, 0, 0, true);
    MV("PF1, all operands", 1, 1, 1, N, true);
    MV("PF2, all operands", 1, 1, 2, N, true);
    MV("PF3, all operands", 1, 1, 3, N, true);
    MV("PF3, half the operands", 1, 1, 3, (N / 2 > 0 ? N / 2 : 1), true);
    MV("PF3, operand 0 only", 1, 1, 3, 1, true);
    MV("PF1, operand 0 only", 1, 1, 1, 1, true);
    MV("PF1, half the operands", 1, 1, 1, (N / 2 > 0 ? N / 2 : 1), true);
    MV("PF1, two operands", 1, 1, 1, (N >= 2 ? 2 : 1), true);
    MV("PF1, all operands, 2 tiles ahead", 1, 1, 1, N, true, 2);
    MV("PF1, all operands, 4 tiles ahead", 1, 1, 1, N, true, 4);
    MV("PF1, operand 0 only, 2 tiles ahead", 1, 1, 1, 1, true, 2);
    MV("PF3, all operands, uncapped", 1, 0, 3, N, true);
    MV("PF1, all operands, uncapped", 1, 0, 1, N, true);
#undef MV
    vs.push_back({"ceiling: read the N operands, no store (N*S bytes)",
                  [](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL((k_read_only<N>), dim3(tiles(nv)), dim3(kReduceBlock), 0, q, d, s, nv);
    }, false, {}});
}

template <int NMAX>
static void add_tree(std::vector<Variant> &vs, unsigned n)
{
#define TV(label, XM, CAP, PF, PFM, ...)                                                \
    vs.push_back({label, [n](float *d, SrcList s, size_t nv, hipStream_t q) {           \
        hipLaunchKernelGGL((k_reduce_tree<float, 0, NMAX, XM, CAP, PF, PFM __VA_OPT__(,) __VA_ARGS__>), \
                           dim3(tiles(nv)), \
                           dim3(kReduceBlock), 0, q, d, s, n, (size_t)0, nv, (size_t)0); \
    }, true, {}})
    constexpr int C = NMAX >= 8;    /* the product caps NMAX 8 and 16 */
    TV("round-4 product (identity map)", 0, C, 0, 0);
    TV("XCD map, no prefetch", 1, C, 0, 0);
    TV("PF1, all operands", 1, C, 1, NMAX);
    TV("PF3, all operands", 1, C, 3, NMAX);
    TV("PF3, first half", 1, C, 3, NMAX / 2);
    TV("PF3, operand 0 only", 1, C, 3, 1);
    TV("PF1, operand 0 only", 1, C, 1, 1);
    TV("PF1, first half", 1, C, 1, NMAX / 2);
    TV("PF1, all operands, 2 tiles ahead", 1, C, 1, NMAX, 2);
    TV("PF1, all operands, 4 tiles ahead", 1, C, 1, NMAX, 4);
    TV("PF1, operand 0 only, 2 tiles ahead", 1, C, 1, 1, 2);
#undef TV
}

int main(int argc, char **argv)
{
    if (argc < 3 || (strcmp(argv[1], "multi") && strcmp(argv[1], "tree"))) {
        fprintf(stderr, "usage: tune_multi_pf multi|tree N [lg=24] [rounds=5] [stagger=0]\n");
        return 2;
    }
    const bool tree  = !strcmp(argv[1], "tree");
    const unsigned N = (unsigned)atoi(argv[2]);
    const int lg     = argc > 3 ? atoi(argv[3]) : 24;
    const int rounds = argc > 4 ? atoi(argv[4]) : 5;
    /* operand m starts m * stagger bytes past m * S (a multiple of 256 B):
     * do operands a power of two apart meet in the same HBM channels? */
    const size_t stagger = argc > 5 ? (size_t)atol(argv[5]) & ~(size_t)255 : 0;
    const int iters  = 10;
    if ((!tree && (N != 2 && N != 4 && N != 8 && N != 16)) || (tree && (N < 2 || N > 16))) {
        fprintf(stderr, "N: multi 2/4/8/16, tree 2..16\n");
        return 2;
    }
    const size_t n = (size_t)1 << lg, nvec = n / 4, S = n * 4;
    char *arena;
    const size_t slot = S + stagger;
    CHECK(hipMalloc(&arena, (N + 2) * slot));
    SrcList srcs;
    for (unsigned m = 0; m < (unsigned)kMaxMulti; m++) {
        srcs.p[m] = m < N ? arena + m * slot : nullptr;
    }
    {
        std::vector<float> h(n);
        for (unsigned m = 0; m < N; m++) {
            for (size_t i = 0; i < n; i++) {   /* rounded values: association matters */
                const uint32_t x = (uint32_t)(i * 2654435761u) ^ (m * 0x9e3779b9u);
                h[i] = (float)((int)(x % 200003) - 100001) * 0.0137f;
            }
            CHECK(hipMemcpy(const_cast<void*>(srcs.p[m]), h.data(), S, hipMemcpyHostToDevice));
        }
    }
    float *out = reinterpret_cast<float*>(arena + N * slot);
    float *ref = reinterpret_cast<float*>(arena + (N + 1) * slot);
    hipStream_t st;
    CHECK(hipStreamCreate(&st));

    std::vector<Variant> vs;
    if (!tree) {
        switch (N) {
        case 2:  add_multi<2>(vs); break;
        case 4:  add_multi<4>(vs); break;
        case 8:  add_multi<8>(vs); break;
        default: add_multi<16>(vs); break;
        }
    } else if (N <= 4) {
        add_tree<4>(vs, N);
    } else if (N <= 8) {
        add_tree<8>(vs, N);
    } else {
        add_tree<16>(vs, N);
    }

    vs[0].run(ref, srcs, nvec, st);
    CHECK(hipStreamSynchronize(st));
    std::vector<float> hr(n), ho(n);
    CHECK(hipMemcpy(hr.data(), ref, S, hipMemcpyDeviceToHost));
    for (auto &v : vs) {
        if (!v.checked) {
            continue;
        }
        CHECK(hipMemset(out, 0, S));
        v.run(out, srcs, nvec, st);
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpy(ho.data(), out, S, hipMemcpyDeviceToHost));
        if (memcmp(ho.data(), hr.data(), S) != 0) {
            printf("MISMATCH %s\n", v.name.c_str());
            return 3;
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (auto &v : vs) {          /* warm: clocks up */
        for (int i = 0; i < 5; i++) {
            v.run(out, srcs, nvec, st);
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
    const double bytes = (double)(N + 1) * S;
    printf("%s %u, %zu MiB per operand, (N+1)*S = %.0f MiB per launch, %d rounds x %d, "
           "stagger %zu B\n", tree ? "tree n =" : "multi N =", N, S >> 20, bytes / 1048576.0,
           rounds, iters, stagger);
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2];
        const double b = v.checked ? bytes : bytes * N / (N + 1);
        printf("%-52s median %8.2f us  min %8.2f  %7.1f GB/s  %5.1f%% of 8 TB/s\n",
               v.name.c_str(), med * 1e3, v.ms.front() * 1e3, b / (med * 1e-3) / 1e9,
               100.0 * b / (med * 1e-3) / 8e12);
    }
    return 0;
}
