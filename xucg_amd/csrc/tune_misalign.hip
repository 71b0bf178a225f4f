/*
 * tune_misalign.hip - operands out of dst's 16-B phase: the product realigns
 * them in registers (k_reduce_shift / k_reduce_multi_shift: aligned 16-B
 * loads, the next vector from the next lane, a funnel shift). The
 * alternative here is the plain kernel fed the misaligned pointer: every
 * lane's 16-B load straddles two 16-B words (gfx950 runs with unaligned
 * access enabled), and the wave's 64 loads still cover one contiguous span.
 * fp32 SUM, 2^26 elements (2 x 256 MiB) and N = 8 operands of 64 MiB, src 4 B
 * past dst's phase; every form checked bit for bit against the product's.
 *
 *   tune_misalign [rounds = 5]
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

/* the aligned kernel's body with the src pointer taken as given */
__global__ void __launch_bounds__(kReduceBlock)
k_plain_misaligned(float *dst, const float *src, size_t nvec)
{
    const size_t i = (size_t)blockIdx.x * kReduceBlock + threadIdx.x;
    if (i < nvec) {
        const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + i);
        const u32x4 b = __builtin_nontemporal_load(reinterpret_cast<u32x4*>(dst) + i);
        __builtin_nontemporal_store(vapply<float, 0>(a, b), reinterpret_cast<u32x4*>(dst) + i);
    }
}

template <int N>
__global__ void __launch_bounds__(kReduceBlock)
k_multi_plain_misaligned(float *dst, SrcList srcs, size_t nvec)
{
    UCG_MULTI_CAP_CLOBBER();
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    const size_t i = (size_t)blockIdx.x * kReduceBlock + threadIdx.x;
    if (i < nvec) {
        u32x4 val[N];
#pragma unroll
        for (int m = 0; m < N; m++) {
            val[m] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(srcs.p[m]) + i);
        }
        __builtin_nontemporal_store(rd_tree<N>(val, fv), reinterpret_cast<u32x4*>(dst) + i);
    }
}

/* the all-gather row copy of a source 4 B out of phase: the product's
 * realignment (copy_row in dev_combine.hip), and the plain misaligned load */
__global__ void __launch_bounds__(kReduceBlock)
k_copy_shift(u32x4 *out, const float *src, size_t nvec)
{
    const size_t i = (size_t)blockIdx.x * kReduceBlock + threadIdx.x;
    const char *sp = reinterpret_cast<const char*>(src);
    const unsigned rs = (unsigned)((uintptr_t)sp & 15);
    const u32x4 *a4 = reinterpret_cast<const u32x4*>(sp - rs);
    const bool last_lane = threadIdx.x == kReduceBlock - 1;
    const u32x4 lo = ld16<1>(a4 + (i < nvec ? i : nvec));
    const u32x4 ex = ld16<1>(a4 + (last_lane && i < nvec ? i + 1 : nvec));
    u32x4 hi;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        hi[k] = from_next_lane(lo[k]);
    }
    if (last_lane) {
        hi = ex;
    }
    if (i < nvec) {
        st16<1>(out + i, funnel16(lo, hi, rs));
    }
}

__global__ void __launch_bounds__(kReduceBlock)
k_copy_plain_misaligned(u32x4 *out, const float *src, size_t nvec)
{
    const size_t i = (size_t)blockIdx.x * kReduceBlock + threadIdx.x;
    if (i < nvec) {
        st16<1>(out + i, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + i));
    }
}

struct Case {
    std::string name;
    double bytes;
    std::function<void()> run;
    std::vector<float> us;
};

int main(int argc, char **argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    const size_t n = (size_t)1 << 26, nvec = n / 4;
    const size_t nm = (size_t)1 << 24, nvm = nm / 4;
    float *src, *dst, *ref;
    CHECK(hipMalloc(&src, n * 4 + 4096));
    CHECK(hipMalloc(&dst, n * 4));
    CHECK(hipMalloc(&ref, n * 4));
    const float *s4 = src + 1;                        /* 4 B past dst's phase */
    std::vector<float*> ops(8);
    SrcList sl, sl_al;
    for (int m = 0; m < 8; m++) {
        CHECK(hipMalloc(&ops[m], nm * 4 + 4096));
        hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                           (void*)ops[m], 0, 50ull + m, nm + 1024);
        sl.p[m] = ops[m] + 1;
        sl_al.p[m] = ops[m];
    }
    for (int m = 8; m < kMaxMulti; m++) {
        sl.p[m] = sl_al.p[m] = nullptr;
    }
    hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                       (void*)src, 1, 7ull, n + 1024);
    hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                       (void*)dst, 1, 8ull, n);
    hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                       (void*)ref, 1, 9ull, n);
    CHECK(hipDeviceSynchronize());
    const unsigned g2 = (unsigned)(nvec / kReduceBlock), gm = (unsigned)(nvm / kReduceBlock);

    std::vector<Case> cs = {
        {"2-op aligned k_reduce", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock>), dim3(g2),
                                dim3(kReduceBlock), 0, 0, dst, (const float*)src, (size_t)0,
                                nvec, (size_t)0); }, {}},
        {"2-op shift (product)", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce_shift<float, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0,
                                dst, s4, (size_t)0, nvec, (size_t)0, 0u); }, {}},
        {"2-op plain misaligned", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL(k_plain_misaligned, dim3(g2), dim3(kReduceBlock), 0, 0,
                                dst, s4, nvec); }, {}},
        {"copy aligned", 2.0 * n * 4, [&] {
             hipLaunchKernelGGL(k_copy_plain_misaligned, dim3(g2), dim3(kReduceBlock), 0, 0,
                                reinterpret_cast<u32x4*>(dst), (const float*)src, nvec); }, {}},
        {"copy shift (product's copy_row)", 2.0 * n * 4, [&] {
             hipLaunchKernelGGL(k_copy_shift, dim3(g2), dim3(kReduceBlock), 0, 0,
                                reinterpret_cast<u32x4*>(dst), s4, nvec); }, {}},
        {"copy plain misaligned", 2.0 * n * 4, [&] {
             hipLaunchKernelGGL(k_copy_plain_misaligned, dim3(g2), dim3(kReduceBlock), 0, 0,
                                reinterpret_cast<u32x4*>(dst), s4, nvec); }, {}},
        {"N=8 aligned (capped)", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_multi<float, 0, 8, 0, 1>), dim3(gm), dim3(kReduceBlock),
                                0, 0, dst, sl_al, 0u, (size_t)0, nvm, (size_t)0); }, {}},
        {"N=8 shift (product)", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_multi_shift<float, 0, 8>), dim3(gm), dim3(kReduceBlock),
                                0, 0, dst, sl, 0u, (size_t)0, nvm, (size_t)0); }, {}},
        {"N=8 shift, VGPR-capped", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_multi_shift<float, 0, 8, 1>), dim3(gm), dim3(kReduceBlock),
                                0, 0, dst, sl, 0u, (size_t)0, nvm, (size_t)0); }, {}},
        {"N=8 plain misaligned (capped)", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_multi_plain_misaligned<8>), dim3(gm), dim3(kReduceBlock), 0, 0,
                                dst, sl, nvm); }, {}},
    };

    /* bits: the misaligned forms against the product's realigning forms */
    std::vector<uint32_t> a(n), b(n);
    const int pairs[][2] = {{1, 2}, {4, 5}, {7, 8}, {7, 9}};
    for (const auto &pr : pairs) {
        for (int k = 0; k < 2; k++) {
            CHECK(hipMemcpy(dst, ref, n * 4, hipMemcpyDeviceToDevice));   /* same start */
            cs[pr[k]].run();
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(k ? b.data() : a.data(), dst, n * 4, hipMemcpyDeviceToHost));
        }
        const size_t cmp = pr[0] == 7 ? nm : n;
        if (!std::equal(a.begin(), a.begin() + cmp, b.begin())) {
            printf("MISMATCH %s vs %s\n", cs[pr[0]].name.c_str(), cs[pr[1]].name.c_str());
            return 3;
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; r++) {
        for (auto &c : cs) {
            c.run();
            CHECK(hipEventRecord(e0, 0));
            for (int i = 0; i < 20; i++) {
                c.run();
            }
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            c.us.push_back(1000.f * ms / 20);
        }
    }
    printf("fp32 SUM, src 4 B past dst's 16-B phase; %% of 8 TB/s, median of %d rounds\n",
           rounds);
    for (auto &c : cs) {
        auto v = c.us;
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2];
        printf("%-32s %9.2f us %6.1f %%\n", c.name.c_str(), med,
               100.0 * c.bytes / (med * 1e-6) / 8e12);
    }
    return 0;
}
