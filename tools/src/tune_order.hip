/*
 * tune_order.hip - A/B of the issue order of k_reduce's three loads in the PF
 * form (the product's 2-operand combine): src's vector, dst's
 * vector and the next tile's src line. Round 6's config-3 sweep read the
 * pairs whose compiled kernel issues src, prefetch, dst 1.7 points above the
 * pairs issuing src, dst, prefetch (profiles/r06/c3); the compiler picks the
 * order per (dtype, op). ORD 0 = the compiler's order, 1 = src, prefetch,
 * dst, 2 = prefetch, src, dst, 3 = src, dst, prefetch (sched barriers).
 *
 *   tune_order [log2 bytes per operand = 30] [rounds = 7]
 *
 * Both operands in one allocation (the bench's layout). Every variant's
 * result is checked bit for bit against ORD 0's on a 16 MiB prefix first;
 * then the variants run interleaved over rounds, 20 launches per sample, HIP
 * events on one stream; 3 x operand bytes per launch.
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

typedef void (*launch_f)(void *dst, const void *src, size_t nvec, hipStream_t q);

template <typename T, int OP, int ORD>
static void run(void *dst, const void *src, size_t nvec, hipStream_t q)
{
    hipLaunchKernelGGL((k_reduce<T, OP, 1, 1, kReduceBlock, 1, 3, ORD>),
                       dim3((unsigned)((nvec + kReduceBlock - 1) / kReduceBlock)),
                       dim3(kReduceBlock), 0, q, static_cast<T*>(dst),
                       static_cast<const T*>(src), (size_t)0, nvec, (size_t)0);
}

/* the product's form (ORD 2) with dynamic LDS bounding the one-wave
 * workgroups per CU (160 KiB / LDS): does the 2-operand combine gain from
 * an occupancy cap as the multi-operand kernels did? */
template <typename T, int OP, unsigned LDS>
static void run_cap(void *dst, const void *src, size_t nvec, hipStream_t q)
{
    hipLaunchKernelGGL((k_reduce<T, OP, 1, 1, kReduceBlock, 1, 3, 2>),
                       dim3((unsigned)((nvec + kReduceBlock - 1) / kReduceBlock)),
                       dim3(kReduceBlock), LDS, q, static_cast<T*>(dst),
                       static_cast<const T*>(src), (size_t)0, nvec, (size_t)0);
}

/* the product's load order with PF lines of the next tile (the product: 3) */
template <typename T, int OP, int PF>
static void run_pf(void *dst, const void *src, size_t nvec, hipStream_t q)
{
    hipLaunchKernelGGL((k_reduce<T, OP, 1, 1, kReduceBlock, 1, PF, 2>),
                       dim3((unsigned)((nvec + kReduceBlock - 1) / kReduceBlock)),
                       dim3(kReduceBlock), 0, q, static_cast<T*>(dst),
                       static_cast<const T*>(src), (size_t)0, nvec, (size_t)0);
}

/* the PF form's aligned body (no ragged edges: the harness sizes are whole
 * tiles) with the load order of ORD and SLP x 64 cycles of s_sleep between
 * the loads' return and the store - does a later store let HBM batch more
 * reads (int8 LXOR, ~90 VALU ops before its store, reads 2 points above) */
template <typename T, int OP, int ORD, int SLP>
__global__ void __launch_bounds__(kReduceBlock)
k_pf_sleep(T *dst, const T *src, size_t nvec)
{
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
    const size_t i  = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * kReduceBlock +
                      threadIdx.x;
    const size_t ic = i < nvec ? i : nvec - 1;
    const unsigned k = kReduceBlock - 1 - threadIdx.x;
    const size_t want = (i - threadIdx.x + kReduceBlock) + (size_t)k * 8;
    const u32x4 *at   = s4 + (k < 3u && want < nvec ? want : nvec - 1);
    u32x4 a, b, pf;
    if constexpr (ORD == 2) {
        pf = ld16<0>(at);
        __builtin_amdgcn_sched_barrier(0);
        a  = ld16<1>(s4 + ic);
        __builtin_amdgcn_sched_barrier(0);
        b  = ld16<1>(d4 + ic);
    } else {
        a  = ld16<1>(s4 + ic);
        __builtin_amdgcn_sched_barrier(0);
        pf = ld16<0>(at);
        __builtin_amdgcn_sched_barrier(0);
        b  = ld16<1>(d4 + ic);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" :: "v"(pf[0]));
    const u32x4 r = vapply<T, OP>(a, b);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (SLP > 0) {
        __builtin_amdgcn_s_sleep(SLP);
    }
    if (i < nvec) {
        st16<1>(d4 + i, r);
    }
}

/* the same body (ORD 2) on XCD chunks of C tiles (the product: 64) */
template <typename T, int OP, unsigned C>
__global__ void __launch_bounds__(kReduceBlock)
k_pf_chunk(T *dst, const T *src, size_t nvec)
{
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
    const size_t i  = (size_t)xcd_tile<C>(blockIdx.x, gridDim.x) * kReduceBlock + threadIdx.x;
    const size_t ic = i < nvec ? i : nvec - 1;
    const unsigned k = kReduceBlock - 1 - threadIdx.x;
    const size_t want = (i - threadIdx.x + kReduceBlock) + (size_t)k * 8;
    const u32x4 *at   = s4 + (k < 3u && want < nvec ? want : nvec - 1);
    const u32x4 pf = ld16<0>(at);
    __builtin_amdgcn_sched_barrier(0);
    const u32x4 a = ld16<1>(s4 + ic);
    __builtin_amdgcn_sched_barrier(0);
    const u32x4 b = ld16<1>(d4 + ic);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" :: "v"(pf[0]));
    if (i < nvec) {
        st16<1>(d4 + i, vapply<T, OP>(a, b));
    }
}

template <typename T, int OP, unsigned C>
static void run_chunk(void *dst, const void *src, size_t nvec, hipStream_t q)
{
    hipLaunchKernelGGL((k_pf_chunk<T, OP, C>),
                       dim3((unsigned)((nvec + kReduceBlock - 1) / kReduceBlock)),
                       dim3(kReduceBlock), 0, q, static_cast<T*>(dst),
                       static_cast<const T*>(src), nvec);
}

/* the realigning combine's aligned body (src 4 B past dst's phase: Q = 1,
 * rb = 0; no ragged edges) on XCD chunks of C tiles (the product: 64) */
template <typename T, int OP, unsigned C>
__global__ void __launch_bounds__(kReduceBlock)
k_shift_chunk(T *dst, const T *src, size_t nvec)
{
    const u32x4 *a4 = reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(src) + 4 - 4);
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
    const size_t i  = (size_t)xcd_tile<C>(blockIdx.x, gridDim.x) * kReduceBlock + threadIdx.x;
    const bool last_lane = threadIdx.x == kReduceBlock - 1;
    const u32x4 b  = ld16<1>(d4 + (i < nvec ? i : nvec - 1));
    const u32x4 lo = ld16<1>(a4 + (i < nvec ? i : nvec));
    const unsigned k  = kReduceBlock - 1 - threadIdx.x;
    const size_t want = (i - threadIdx.x + kReduceBlock) + (size_t)k * 8;
    const u32x4 ex = ld16<0>(a4 + (k < 3u && want <= nvec ? want : nvec));
    __builtin_amdgcn_sched_barrier(0);
    u32x4 hi;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        hi[q] = from_next_lane(lo[q]);
    }
    if (last_lane) {
        hi = ex;
    }
    if (i < nvec) {
        const uint32_t w[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        u32x4 sv;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            sv[q] = __builtin_amdgcn_alignbyte(w[q + 2], w[q + 1], 0u);
        }
        st16<1>(d4 + i, vapply<T, OP>(sv, b));
    }
}

template <typename T, int OP, unsigned C>
static void run_shift_chunk(void *dst, const void *src, size_t nvec, hipStream_t q)
{
    /* src + 4 B: its aligned vectors A[0..nvec] start at src; one vector fewer */
    hipLaunchKernelGGL((k_shift_chunk<T, OP, C>),
                       dim3((unsigned)((nvec - 1 + kReduceBlock - 1) / kReduceBlock)),
                       dim3(kReduceBlock), 0, q, static_cast<T*>(dst), static_cast<const T*>(src),
                       nvec - 1);
}

template <typename T, int OP, int ORD, int SLP>
static void run_sleep(void *dst, const void *src, size_t nvec, hipStream_t q)
{
    hipLaunchKernelGGL((k_pf_sleep<T, OP, ORD, SLP>),
                       dim3((unsigned)((nvec + kReduceBlock - 1) / kReduceBlock)),
                       dim3(kReduceBlock), 0, q, static_cast<T*>(dst),
                       static_cast<const T*>(src), nvec);
}

struct Variant {
    std::string name;
    int pair;
    launch_f f;
    std::vector<float> ms;
};

/* small integers in every dtype's bit pattern: no NaN, no overflow to inf */
__global__ void k_init(uint32_t *p, size_t n, uint32_t seed)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t x = (uint32_t)(i * 2654435761u) ^ seed;
        p[i] = (x & 0x3fff3fffu) | 0x3c003c00u;   /* fp16/bf16 halves, fp32 ~1-2 */
    }
}

#define PAIR(T, OP, label)                                                  \
    vs.push_back({std::string(label) + " ORD 0 (compiler)", np, run<T, OP, 0>, {}}); \
    vs.push_back({std::string(label) + " ORD 1 src,pf,dst", np, run<T, OP, 1>, {}}); \
    vs.push_back({std::string(label) + " ORD 2 pf,src,dst", np, run<T, OP, 2>, {}}); \
    vs.push_back({std::string(label) + " ORD 3 src,dst,pf", np, run<T, OP, 3>, {}}); \
    np++;

int main(int argc, char **argv)
{
    const int lg     = argc > 1 ? atoi(argv[1]) : 30;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const int iters  = 20;
    const size_t S = (size_t)1 << lg, nvec = S / 16;
    std::vector<Variant> vs;
    int np = 0;
    PAIR(float, UCG_DEV_OP_SUM, "fp32 sum");
    PAIR(int32_t, UCG_DEV_OP_MAX, "int32 max");
    PAIR(double, UCG_DEV_OP_MAX, "fp64 max");
    PAIR(uint32_t, UCG_DEV_OP_MIN, "uint32 min");
    PAIR(int16_t, UCG_DEV_OP_MIN, "int16 min");
    PAIR(int64_t, UCG_DEV_OP_SUM, "int64 sum");
    PAIR(int8_t, UCG_DEV_OP_LXOR, "int8 lxor");
    /* the realigning kernel's XCD chunk (its own pair) */
    vs.push_back({"shift fp32 sum chunk 64 ORD 0", np, run_shift_chunk<float, UCG_DEV_OP_SUM, 64>, {}});
    vs.push_back({"shift fp32 sum chunk 128", np, run_shift_chunk<float, UCG_DEV_OP_SUM, 128>, {}});
    vs.push_back({"shift fp32 sum chunk 256", np, run_shift_chunk<float, UCG_DEV_OP_SUM, 256>, {}});
    np++;
    /* XCD chunk size with the lines first, fp32 SUM (pair 0) */
    vs.push_back({"fp32 sum ORD 2, XCD chunk 16", 0, run_chunk<float, UCG_DEV_OP_SUM, 16>, {}});
    vs.push_back({"fp32 sum ORD 2, XCD chunk 32", 0, run_chunk<float, UCG_DEV_OP_SUM, 32>, {}});
    vs.push_back({"fp32 sum ORD 2, XCD chunk 64", 0, run_chunk<float, UCG_DEV_OP_SUM, 64>, {}});
    vs.push_back({"fp32 sum ORD 2, XCD chunk 128", 0, run_chunk<float, UCG_DEV_OP_SUM, 128>, {}});
    vs.push_back({"fp32 sum ORD 2, XCD chunk 256", 0, run_chunk<float, UCG_DEV_OP_SUM, 256>, {}});
    /* prefetch depth with the lines first, fp32 SUM (pair 0) */
    vs.push_back({"fp32 sum ORD 2, PF 1 line", 0, run_pf<float, UCG_DEV_OP_SUM, 1>, {}});
    vs.push_back({"fp32 sum ORD 2, PF 2 lines", 0, run_pf<float, UCG_DEV_OP_SUM, 2>, {}});
    vs.push_back({"fp32 sum ORD 2, PF 4 lines", 0, run_pf<float, UCG_DEV_OP_SUM, 4>, {}});
    vs.push_back({"fp32 sum ORD 2, PF 5 lines", 0, run_pf<float, UCG_DEV_OP_SUM, 5>, {}});
    vs.push_back({"fp32 sum ORD 2, PF 6 lines", 0, run_pf<float, UCG_DEV_OP_SUM, 6>, {}});
    /* occupancy caps, fp32 SUM (pair 0) */
#define CAPV(W) vs.push_back({"fp32 sum ORD 2, LDS cap " #W " waves/CU", 0, \
                              run_cap<float, UCG_DEV_OP_SUM, 163840u / W>, {}});
    (void)0; /* caps: r06zd (every cap lost) */
#undef CAPV
    /* sleep before the store, fp32 SUM and int32 MAX (pair indices 0, 1) */
#define SLV(T, OP, P, label, ORD, SLP) \
    vs.push_back({std::string(label), P, run_sleep<T, OP, ORD, SLP>, {}});
    SLV(float, UCG_DEV_OP_SUM, 0, "fp32 sum ORD 2, sleep 0", 2, 0);
    SLV(float, UCG_DEV_OP_SUM, 0, "fp32 sum ORD 2, sleep 1", 2, 1);
    SLV(float, UCG_DEV_OP_SUM, 0, "fp32 sum ORD 2, sleep 2", 2, 2);
    SLV(float, UCG_DEV_OP_SUM, 0, "fp32 sum ORD 2, sleep 4", 2, 4);
    SLV(float, UCG_DEV_OP_SUM, 0, "fp32 sum ORD 2, sleep 8", 2, 8);
    SLV(float, UCG_DEV_OP_SUM, 0, "fp32 sum ORD 1, sleep 2", 1, 2);
    SLV(float, UCG_DEV_OP_SUM, 0, "fp32 sum ORD 1, sleep 4", 1, 4);
    SLV(int32_t, UCG_DEV_OP_MAX, 1, "int32 max ORD 2, sleep 0", 2, 0);
    SLV(int32_t, UCG_DEV_OP_MAX, 1, "int32 max ORD 2, sleep 2", 2, 2);
    SLV(int32_t, UCG_DEV_OP_MAX, 1, "int32 max ORD 2, sleep 4", 2, 4);
#undef SLV

    char *arena;
    CHECK(hipMalloc(&arena, 2 * S));
    char *src = arena, *dst = arena + S;
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    const size_t nw = S / 4;
    hipLaunchKernelGGL(k_init, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st,
                       reinterpret_cast<uint32_t*>(src), nw, 0x1234u);
    hipLaunchKernelGGL(k_init, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st,
                       reinterpret_cast<uint32_t*>(dst), nw, 0xabcdu);
    CHECK(hipStreamSynchronize(st));

    /* bit-exact against ORD 0 on a 16 MiB prefix, from the same dst */
    {
        const size_t cb = std::min(S, (size_t)16 << 20), cv = cb / 16;
        char *d0, *d1;
        CHECK(hipMalloc(&d0, cb));
        CHECK(hipMalloc(&d1, cb));
        std::vector<char> h0(cb), h1(cb);
        for (auto &v : vs) {
            if (v.name.find("ORD 0") == std::string::npos) {
                continue;
            }
            CHECK(hipMemcpy(d0, dst, cb, hipMemcpyDeviceToDevice));
            v.f(d0, src, cv, st);
            CHECK(hipStreamSynchronize(st));
            CHECK(hipMemcpy(h0.data(), d0, cb, hipMemcpyDeviceToHost));
            for (auto &w : vs) {
                if (w.pair != v.pair || &w == &v) {
                    continue;
                }
                CHECK(hipMemcpy(d1, dst, cb, hipMemcpyDeviceToDevice));
                w.f(d1, src, cv, st);
                CHECK(hipStreamSynchronize(st));
                CHECK(hipMemcpy(h1.data(), d1, cb, hipMemcpyDeviceToHost));
                if (memcmp(h0.data(), h1.data(), cb) != 0) {
                    printf("MISMATCH %s\n", w.name.c_str());
                    return 3;
                }
            }
        }
        CHECK(hipFree(d0));
        CHECK(hipFree(d1));
    }

    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (auto &v : vs) {
        for (int i = 0; i < 3; i++) {
            v.f(dst, src, nvec, st);
        }
    }
    for (int r = 0; r < rounds; r++) {
        for (auto &v : vs) {
            v.f(dst, src, nvec, st);
            CHECK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; i++) {
                v.f(dst, src, nvec, st);
            }
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms / iters);
        }
    }
    printf("k_reduce PF=3 load order, %zu MiB per operand (one allocation), %d rounds x %d\n",
           S >> 20, rounds, iters);
    const double bytes = 3.0 * S;
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2];
        printf("%-32s median %8.2f us  min %8.2f  %5.1f%% of 8 TB/s\n", v.name.c_str(),
               med * 1e3, v.ms.front() * 1e3, 100.0 * bytes / (med * 1e-3) / 8e12);
    }
    return 0;
}
