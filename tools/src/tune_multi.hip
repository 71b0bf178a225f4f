/*
 * tune_multi.hip - A/B harness for the one-shot multi-operand combine
 * (k_reduce_multi, N = 8 fp32 SUM, the C4 one-shot reduce-scatter shape) on
 * one GPU: every variant reads the same N local operands and writes one
 * output; runs are interleaved over rounds; every variant's output is
 * checked bit for bit against the product kernel's.
 *
 *   tune_multi [log2 elements per operand = 26] [rounds = 5]
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

/* store policy and persistent-grid A/B: NTS = non-temporal store; G > 0:
 * a grid of G workgroups looping over the tiles (tile b, b + G, ...) */
template <int NTS>
__global__ void __launch_bounds__(64)
k_multi_loop(float *dst, SrcList srcs, unsigned self, size_t nvec, unsigned loop)
{
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    const size_t step = loop ? (size_t)gridDim.x * 64 : nvec;
    for (size_t i = (size_t)blockIdx.x * 64 + threadIdx.x; i < nvec; i += step) {
        u32x4 val[N];
#pragma unroll
        for (int m = 0; m < N; m++) {
            val[m] = ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[self ^ m]) + i);
        }
        st16<NTS>(reinterpret_cast<u32x4*>(dst) + i, rd_tree<N>(val, fv));
    }
}

/* load-order A/B: waves of odd workgroups issue their N loads last operand
 * first, so that at any instant the waves in flight spread over all N
 * buffers instead of all starting on operand 0 (same tree, same bits) */
__global__ void __launch_bounds__(64)
k_multi_alt_order(float *dst, SrcList srcs, unsigned self, size_t nvec)
{
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= nvec) {
        return;
    }
    u32x4 val[N];
    if (blockIdx.x & 1) {
#pragma unroll
        for (int m = N - 1; m >= 0; m--) {
            val[m] = ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[self ^ m]) + i);
        }
    } else {
#pragma unroll
        for (int m = 0; m < N; m++) {
            val[m] = ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[self ^ m]) + i);
        }
    }
    st16<1>(reinterpret_cast<u32x4*>(dst) + i, rd_tree<N>(val, fv));
}

/* the N loads and one store with no combine (an XOR fold; not checked): how
 * much of the loss is the store itself */
__global__ void __launch_bounds__(64)
k_multi_xor_store(float *dst, SrcList srcs, unsigned self, size_t nvec)
{
    const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= nvec) {
        return;
    }
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < N; m++) {
        acc ^= ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[self ^ m]) + i);
    }
    st16<1>(reinterpret_cast<u32x4*>(dst) + i, acc);
}

/* ceiling probe: the same N loads, no combine and a store only where the
 * (never true) data test passes, so the loads cannot be dropped */
template <int BS>
__global__ void __launch_bounds__(BS)
k_multi_readonly(float *dst, SrcList srcs, unsigned self, size_t nvec)
{
    const size_t i = (size_t)blockIdx.x * BS + threadIdx.x;
    if (i >= nvec) {
        return;
    }
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < N; m++) {
        acc ^= ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[self ^ m]) + i);
    }
    if (acc[0] == 0x7fc00123u && acc[1] == 0x7fc00321u) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + i, acc);
    }
}

/* operand-major: a wave streams U KiB of one operand at a time (U vectors
 * per lane, 64 lanes apart, so each load instruction covers 1 KiB) with the
 * next operand's loads in flight while it combines the current one, and
 * keeps a stack of log2 N partials: operand m's vectors are folded into the
 * partials as a binary counter carries, later group first, which is exactly
 * rd_tree's association (level h: val[m] = f(val[m + h], val[m])). Fewer
 * registers than holding all N operands, and U times longer contiguous runs
 * per operand per wave. nvec must be a multiple of 64 U. */
template <int U>
__global__ void __launch_bounds__(64)
k_multi_opmajor(float *dst, SrcList srcs, unsigned self, size_t nvec)
{
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    constexpr int L = 3;                      /* log2 N */
    const size_t base = (size_t)blockIdx.x * 64 * U + threadIdx.x;
    if (base >= nvec) {
        return;
    }
    u32x4 part[L][U], cur[U], nxt[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        cur[u] = ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[self]) + base + u * 64);
    }
#pragma unroll
    for (int m = 0; m < N; m++) {
        if (m + 1 < N) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                nxt[u] = ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[self ^ (m + 1)]) +
                                 base + u * 64);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        int lvl = 0;
#pragma unroll
        for (int l = 0; l < L; l++) {
            if (((m >> l) & 1) && lvl == l) {
#pragma unroll
                for (int u = 0; u < U; u++) {
                    cur[u] = fv(cur[u], part[l][u]);
                }
                lvl = l + 1;
            }
        }
        if (m + 1 < N) {
#pragma unroll
            for (int u = 0; u < U; u++) {
                part[lvl][u] = cur[u];
                cur[u] = nxt[u];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + base + u * 64, cur[u]);
    }
}

/* L lanes per vector (verdict item 5's suggestion): the N = 8 operands of
 * one 16-B vector are split over L lanes of a wave (N / L each, lanes 64 / L
 * apart), each lane folds its operands as the subtree rd_tree builds for them,
 * and the partials meet over lane exchanges (xor 32, then 16): the same
 * association, so the same bits. A wave covers 64 / L vectors per operand. */
template <int L>
__global__ void __launch_bounds__(64)
k_multi_lanes(float *dst, SrcList srcs, unsigned self, size_t nvec)
{
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    constexpr int K = N / L;                 /* operands per lane */
    constexpr int W = 64 / L;                /* vectors per wave */
    const unsigned part = threadIdx.x / W;   /* which K operands */
    const size_t i = (size_t)blockIdx.x * W + (threadIdx.x % W);
    u32x4 val[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        val[k] = ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[self ^ (part * K + k)]) + i);
    }
    u32x4 acc = rd_tree<K>(val, fv);
    /* level log2 K + 1 ...: the partial of the higher group is the src */
#pragma unroll
    for (int w = 1; w < L; w <<= 1) {
        u32x4 other;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            other[c] = __shfl_xor(acc[c], w * W, 64);
        }
        if ((part & w) == 0) {
            acc = fv(other, acc);
        }
    }
    if (part == 0 && i < nvec) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + i, acc);
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
    const bool occ = getenv("TUNE_OCC") != nullptr;
    if (occ) {
        /* occupancy A/B: dynamic LDS the kernel does not use caps the
         * one-wave workgroups per CU at W (160 KiB of LDS per CU): fewer
         * operand streams in flight at once */
        for (int W : {4, 6, 8, 12, 16, 20, 24, 28}) {
            const size_t lds = (size_t)163840 / W / 512 * 512;
            vs.push_back({"product, <= " + std::to_string(W) + " waves per CU",
                          [=](float *d, SrcList s, size_t nv, hipStream_t q) {
                unsigned g = (unsigned)((nv + kReduceBlock - 1) / kReduceBlock);
                hipLaunchKernelGGL((k_reduce_multi<float, 0, N>), dim3(g), dim3(kReduceBlock),
                                   lds, q, d, s, 0u, (size_t)0, nv, (size_t)0);
            }, {}});
        }
    }
    std::vector<char*> stag;
    if (!occ) {
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
    vs.push_back({"2 lanes per vector (4 operands each, xor-32 exchange)",
                  [=](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL((k_multi_lanes<2>), dim3((unsigned)(nv / 32)), dim3(64), 0, q,
                           d, s, 0u, nv);
    }, {}});
    vs.push_back({"4 lanes per vector (2 operands each, xor-32/16 exchange)",
                  [=](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL((k_multi_lanes<4>), dim3((unsigned)(nv / 16)), dim3(64), 0, q,
                           d, s, 0u, nv);
    }, {}});
#define OPM(U)                                                                        \
    vs.push_back({"operand-major, " #U " KiB per operand per wave, stack of partials",  \
                  [=](float *d, SrcList s, size_t nv, hipStream_t q) {                \
        hipLaunchKernelGGL((k_multi_opmajor<U>), dim3((unsigned)(nv / (64 * (U)))),    \
                           dim3(64), 0, q, d, s, 0u, nv);                             \
    }, {}})
    OPM(2);
    OPM(4);
    OPM(8);
#undef OPM
    vs.push_back({"temporal stores (U1 BS64)", [=](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL((k_multi_loop<0>), dim3((unsigned)((nv + 63) / 64)), dim3(64), 0, q,
                           d, s, 0u, nv, 0u);
    }, {}});
    for (unsigned w : {4u, 8u, 16u, 32u}) {
        vs.push_back({"persistent grid 256 CUs x " + std::to_string(w) + " waves, NT stores",
                      [=](float *d, SrcList s, size_t nv, hipStream_t q) {
            hipLaunchKernelGGL((k_multi_loop<1>), dim3(256 * w), dim3(64), 0, q, d, s, 0u, nv, 1u);
        }, {}});
    }
    /* the operands at staggered offsets inside one allocation: operand m at
     * m * (S + pad); tests whether N streams at equal offsets of 2^k-sized
     * buffers collide in the HBM channel/bank map */
    for (size_t pad : {(size_t)4096, (size_t)65536, (size_t)(1 << 20) + 4096, (size_t)(2 << 20) + 256 * 1024 + 4096}) {
        char *big;
        CHECK(hipMalloc(&big, N * (n * 4 + pad)));
        stag.push_back(big);
        SrcList ss;
        for (int m = 0; m < kMaxMulti; m++) {
            ss.p[m] = nullptr;
        }
        for (int m = 0; m < N; m++) {
            ss.p[m] = big + m * (n * 4 + pad);
            CHECK(hipMemcpy(const_cast<void*>(ss.p[m]), bufs[m], n * 4, hipMemcpyDeviceToDevice));
        }
        vs.push_back({"product kernel, operands staggered by S+" + std::to_string(pad),
                      [=](float *d, SrcList, size_t nv, hipStream_t q) {
            unsigned g = (unsigned)((nv + kReduceBlock - 1) / kReduceBlock);
            hipLaunchKernelGGL((k_reduce_multi<float, 0, N>), dim3(g), dim3(kReduceBlock), 0, q,
                               d, ss, 0u, (size_t)0, nv, (size_t)0);
        }, {}});
    }
    vs.push_back({"product with the XCD-aware tile map (XM=1)",
                  [=](float *d, SrcList s, size_t nv, hipStream_t q) {
        unsigned g = (unsigned)((nv + kReduceBlock - 1) / kReduceBlock);
        hipLaunchKernelGGL((k_reduce_multi<float, 0, N, 1>), dim3(g), dim3(kReduceBlock), 0, q,
                           d, s, 0u, (size_t)0, nv, (size_t)0);
    }, {}});
    vs.push_back({"odd waves load the operands in reverse order",
                  [=](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL(k_multi_alt_order, dim3((unsigned)((nv + 63) / 64)), dim3(64), 0, q,
                           d, s, 0u, nv);
    }, {}});
    }
    const size_t nvariants_checked = vs.size();
    if (!occ) {
    /* operands AND dst in one allocation (dst after the 8 operands, each
     * S + pad apart): the product kernel on the one-allocation layout that
     * avoids operand aliasing for the 2-operand combine;
     * timing only (the same kernel as the product, other pointers) */
    for (size_t pad : {(size_t)0, (size_t)4096}) {
        char *big;
        CHECK(hipMalloc(&big, (N + 1) * (n * 4 + pad)));
        stag.push_back(big);
        SrcList ss;
        for (int m = 0; m < kMaxMulti; m++) {
            ss.p[m] = m < N ? big + m * (n * 4 + pad) : nullptr;
        }
        for (int m = 0; m < N; m++) {
            CHECK(hipMemcpy(const_cast<void*>(ss.p[m]), bufs[m], n * 4, hipMemcpyDeviceToDevice));
        }
        float *jd = reinterpret_cast<float*>(big + N * (n * 4 + pad));
        vs.push_back({"product, operands and dst in one allocation, S+" + std::to_string(pad) +
                      " apart (unchecked)",
                      [=](float *, SrcList, size_t nv, hipStream_t q) {
            unsigned g = (unsigned)((nv + kReduceBlock - 1) / kReduceBlock);
            hipLaunchKernelGGL((k_reduce_multi<float, 0, N>), dim3(g), dim3(kReduceBlock), 0, q,
                               jd, ss, 0u, (size_t)0, nv, (size_t)0);
        }, {}});
    }
    vs.push_back({"N loads + 1 store, XOR fold (unchecked)",
                  [=](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL(k_multi_xor_store, dim3((unsigned)((nv + 63) / 64)), dim3(64), 0, q,
                           d, s, 0u, nv);
    }, {}});
    /* the 2-operand combine on operands 0 and 1 (3 streams), same process */
    }
    vs.push_back({"2-operand k_reduce on two of the buffers (3*S bytes)",
                  [=](float *d, SrcList s, size_t nv, hipStream_t q) {
        unsigned g = (unsigned)((nv + kReduceBlock - 1) / kReduceBlock);
        hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock>), dim3(g), dim3(kReduceBlock),
                           0, q, d, static_cast<const float*>(s.p[1]), (size_t)0, nv,
                           (size_t)0);
    }, {}});
    vs.push_back({"ceiling: read the N operands, no store (N*S bytes)",
                  [=](float *d, SrcList s, size_t nv, hipStream_t q) {
        unsigned g = (unsigned)((nv + 63) / 64);
        hipLaunchKernelGGL((k_multi_readonly<64>), dim3(g), dim3(64), 0, q, d, s, 0u, nv);
    }, {}});

    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    vs[0].run(ref, srcs, nvec, st);
    CHECK(hipStreamSynchronize(st));
    std::vector<float> hr(n), ho(n);
    CHECK(hipMemcpy(hr.data(), ref, n * 4, hipMemcpyDeviceToHost));
    for (size_t k = 0; k < nvariants_checked; k++) {
        auto &v = vs[k];
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
        const double b = v.name.rfind("ceiling", 0) == 0 ? bytes * N / (N + 1) :
                         v.name.rfind("2-operand", 0) == 0 ? 3.0 * n * 4 : bytes;
        printf("%-56s median %8.2f us  %7.1f GB/s  %5.1f%% of 8 TB/s\n", v.name.c_str(),
               med * 1e3, b / (med * 1e-3) / 1e9, 100.0 * b / (med * 1e-3) / 8e12);
    }
    return 0;
}
