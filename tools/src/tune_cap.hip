/*
 * tune_cap.hip - how to cap the occupancy of the multi-operand combines
 * without dynamic LDS (the LDS cap is suspected in the zeroed
 * allocations). Three forms of k_reduce_multi (N operands, recursive-doubling
 * association) at the same waves per CU:
 *   none  one tile of 64 16-B vectors per one-wave workgroup, grid = tiles
 *   lds   the same grid, at most W workgroups per CU through unused LDS
 *   loop  grid = W x 256 CUs, each workgroup looping over tiles t, t + grid..
 *   pipe  the loop with the next tile's loads issued before this tile's store
 *   vgpr  the `none` grid, at most W waves per CU through the kernel's VGPR
 *         allocation (a clobbered high register)
 * Every form is checked bit for bit against `none`. Operands are separate
 * allocations of S bytes, fp32 SUM, "exact" values.
 *
 *   tune_cap [log2 elements per operand = 24] [rounds = 5] [joint]
 *
 * `joint`: operands and output carved out of one allocation, back to back
 * (bench.py's one_shot_shape layout) instead of one allocation each.
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

template <int N, int PIPE>
__global__ void __launch_bounds__(kReduceBlock)
k_multi_loop(float *dst, SrcList srcs, size_t nvec)
{
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    const size_t ntiles = (nvec + kReduceBlock - 1) / kReduceBlock;
    const size_t G = gridDim.x;
    u32x4 *d4 = reinterpret_cast<u32x4*>(dst);
    size_t t = blockIdx.x;
    if (!PIPE) {
        for (; t < ntiles; t += G) {
            const size_t i = t * kReduceBlock + threadIdx.x;
            if (i < nvec) {
                u32x4 val[N];
#pragma unroll
                for (int m = 0; m < N; m++) {
                    val[m] = ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[m]) + i);
                }
                st16<1>(d4 + i, rd_tree<N>(val, fv));
            }
        }
        return;
    }
    if (t >= ntiles) {
        return;
    }
    size_t i = t * kReduceBlock + threadIdx.x;
    u32x4 cur[N];
#pragma unroll
    for (int m = 0; m < N; m++) {
        cur[m] = ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[m]) + (i < nvec ? i : nvec - 1));
    }
    for (; t < ntiles; t += G) {
        const size_t in = (t + G) * kReduceBlock + threadIdx.x;
        const bool more = t + G < ntiles;
        u32x4 nxt[N];
#pragma unroll
        for (int m = 0; m < N; m++) {
            nxt[m] = more ? ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[m]) +
                                    (in < nvec ? in : nvec - 1))
                          : cur[m];
        }
        if (i < nvec) {
            st16<1>(d4 + i, rd_tree<N>(cur, fv));
        }
#pragma unroll
        for (int m = 0; m < N; m++) {
            cur[m] = nxt[m];
        }
        i = in;
    }
}

/* k_reduce_multi with its VGPR allocation forced up by a clobber of the
 * highest register: 512 VGPRs per SIMD lane on CDNA, so `VG` registers give
 * floor(512 / VG) waves per SIMD, 4x that per CU (no LDS) */
#define CLOBBER_(r) asm volatile("" ::: #r)
template <int N, int W>
__global__ void __launch_bounds__(kReduceBlock)
k_multi_vgpr(float *dst, SrcList srcs, size_t nvec)
{
    if constexpr (W == 8)  CLOBBER_(v255);
    if constexpr (W == 12) CLOBBER_(v167);
    if constexpr (W == 16) CLOBBER_(v127);
    if constexpr (W == 20) CLOBBER_(v95);
    if constexpr (W == 24) CLOBBER_(v79);
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    const size_t i = (size_t)blockIdx.x * kReduceBlock + threadIdx.x;
    if (i < nvec) {
        u32x4 val[N];
#pragma unroll
        for (int m = 0; m < N; m++) {
            val[m] = ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[m]) + i);
        }
        st16<1>(reinterpret_cast<u32x4*>(dst) + i, rd_tree<N>(val, fv));
    }
}

/* two adjacent tiles per one-wave workgroup, every load of both issued
 * before the first combine: twice the bytes in flight per wave, half the
 * workgroups (U = 2), optionally also VGPR-capped */
template <int N, int CAP>
__global__ void __launch_bounds__(kReduceBlock)
k_multi_u2(float *dst, SrcList srcs, size_t nvec)
{
    if constexpr (CAP) {
        UCG_MULTI_CAP_CLOBBER();
    }
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    const size_t i0 = (size_t)blockIdx.x * 2 * kReduceBlock + threadIdx.x;
    const size_t i1 = i0 + kReduceBlock;
    u32x4 a[N], b[N];
#pragma unroll
    for (int m = 0; m < N; m++) {
        const u32x4 *p = reinterpret_cast<const u32x4*>(srcs.p[m]);
        a[m] = ld16<1>(p + (i0 < nvec ? i0 : nvec - 1));
        b[m] = ld16<1>(p + (i1 < nvec ? i1 : nvec - 1));
    }
    if (i0 < nvec) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + i0, rd_tree<N>(a, fv));
    }
    if (i1 < nvec) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + i1, rd_tree<N>(b, fv));
    }
}

template <int N>
static void run_vgpr(int w, float *d, const SrcList &s, size_t nv, unsigned tiles, hipStream_t q)
{
    switch (w) {
    case 8:  hipLaunchKernelGGL((k_multi_vgpr<N, 8>), dim3(tiles), dim3(kReduceBlock), 0, q, d, s, nv); break;
    case 12: hipLaunchKernelGGL((k_multi_vgpr<N, 12>), dim3(tiles), dim3(kReduceBlock), 0, q, d, s, nv); break;
    case 16: hipLaunchKernelGGL((k_multi_vgpr<N, 16>), dim3(tiles), dim3(kReduceBlock), 0, q, d, s, nv); break;
    case 20: hipLaunchKernelGGL((k_multi_vgpr<N, 20>), dim3(tiles), dim3(kReduceBlock), 0, q, d, s, nv); break;
    default: hipLaunchKernelGGL((k_multi_vgpr<N, 24>), dim3(tiles), dim3(kReduceBlock), 0, q, d, s, nv); break;
    }
}

static size_t lds_for(int w)
{
    return w ? (size_t)163840 / w / 512 * 512 : 0;
}

template <int N>
static void run(int form, int w, float *d, const SrcList &s, size_t nv, hipStream_t q)
{
    const unsigned tiles = (unsigned)((nv + kReduceBlock - 1) / kReduceBlock);
    if (form <= 1) {
        hipLaunchKernelGGL((k_reduce_multi<float, 0, N>), dim3(tiles), dim3(kReduceBlock),
                           form == 1 ? lds_for(w) : 0, q, d, s, 0u, (size_t)0, nv, (size_t)0);
        return;
    }
    if (form == 4) {
        run_vgpr<N>(w, d, s, nv, tiles, q);
        return;
    }
    if (form == 5 || form == 6) {
        const unsigned g2 = (tiles + 1) / 2;
        if (form == 5)
            hipLaunchKernelGGL((k_multi_u2<N, 0>), dim3(g2), dim3(kReduceBlock), 0, q, d, s, nv);
        else
            hipLaunchKernelGGL((k_multi_u2<N, 1>), dim3(g2), dim3(kReduceBlock), 0, q, d, s, nv);
        return;
    }
    unsigned g = (unsigned)(256 * w);
    if (g > tiles) g = tiles;
    if (form == 2)
        hipLaunchKernelGGL((k_multi_loop<N, 0>), dim3(g), dim3(kReduceBlock), 0, q, d, s, nv);
    else
        hipLaunchKernelGGL((k_multi_loop<N, 1>), dim3(g), dim3(kReduceBlock), 0, q, d, s, nv);
}

struct Case {
    std::string name;
    int ops, form, w;
    std::function<void(float*, size_t, hipStream_t)> fn;
    std::vector<float> us;
};

int main(int argc, char **argv)
{
    const int lg     = argc > 1 ? atoi(argv[1]) : 24;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int iters  = 10;
    const size_t n = (size_t)1 << lg, nvec = n / 4;
    const bool joint = argc > 3 && strcmp(argv[3], "joint") == 0;
    std::vector<float*> bufs(kMaxMulti);
    SrcList all;
    float *arena = nullptr;
    if (joint) {
        CHECK(hipMalloc(&arena, (size_t)(kMaxMulti + 2) * n * 4));
    }
    for (int m = 0; m < kMaxMulti; m++) {
        if (joint) {
            bufs[m] = arena + (size_t)m * n;
        } else {
            CHECK(hipMalloc(&bufs[m], n * 4));
        }
        hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                           (void*)bufs[m], 0, 100ull + m, n);
        all.p[m] = bufs[m];
    }
    float *out, *ref;
    if (joint) {
        out = arena + (size_t)kMaxMulti * n;
        ref = out + n;
    } else {
        CHECK(hipMalloc(&out, n * 4));
        CHECK(hipMalloc(&ref, n * 4));
    }
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    CHECK(hipDeviceSynchronize());

    static const char *fname[] = {"none", "lds", "loop", "pipe", "vgpr", "u2", "u2+vgpr"};
    std::vector<Case> cs;
    auto add = [&](int ops, int form, int w) {
        char nm[64];
        snprintf(nm, sizeof(nm), "N=%d %s W=%d", ops, fname[form], w);
        std::function<void(float*, size_t, hipStream_t)> f;
        switch (ops) {
        case 4:  f = [=](float *d, size_t nv, hipStream_t q) { run<4>(form, w, d, all, nv, q); }; break;
        case 8:  f = [=](float *d, size_t nv, hipStream_t q) { run<8>(form, w, d, all, nv, q); }; break;
        default: f = [=](float *d, size_t nv, hipStream_t q) { run<16>(form, w, d, all, nv, q); }; break;
        }
        cs.push_back({nm, ops, form, w, f, {}});
    };
    for (int ops : {4, 8, 16}) {
        add(ops, 0, 0);
        add(ops, 5, 0);
        add(ops, 6, 12);
        for (int w : {6, 8, 10, 12, 16}) {
            for (int form : {1, 4}) {
                if (form == 4 && (w == 6 || w == 10)) continue;   /* not a VGPR step */
                add(ops, form, w);
            }
        }
    }

    std::vector<uint32_t> want(n), got(n);
    int bad = 0;
    for (size_t k = 0; k < cs.size(); k++) {
        float *o = cs[k].form == 0 ? ref : out;
        CHECK(hipMemset(o, 0, n * 4));
        cs[k].fn(o, nvec, st);
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpy(cs[k].form == 0 ? want.data() : got.data(), o, n * 4,
                        hipMemcpyDeviceToHost));
        if (cs[k].form != 0 && got != want) {
            printf("MISMATCH %s\n", cs[k].name.c_str());
            bad = 1;
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
            c.fn(out, nvec, st);
            CHECK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; i++) {
                c.fn(out, nvec, st);
            }
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            c.us.push_back(1000.f * ms / iters);
        }
    }
    printf("%zu MiB per operand (%s), fp32 SUM, %% of 8 TB/s on (operands + 1) * S bytes, "
           "median of %d rounds\n", n * 4 >> 20, joint ? "one allocation" : "separate allocations",
           rounds);
    for (auto &c : cs) {
        auto v = c.us;
        std::sort(v.begin(), v.end());
        const double med = v[v.size() / 2];
        printf("%-20s %9.2f us %6.1f %%\n", c.name.c_str(), med,
               100.0 * (double)(c.ops + 1) * n * 4 / (med * 1e-6) / 8e12);
    }
    return 0;
}
