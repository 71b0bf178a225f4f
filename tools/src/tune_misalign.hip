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

/* The realigning forms read one 16-B vector past the wave's tile (lane 63's
 * `ex`), the first vector of the next tile: PMC put the realigning kernels at
 * 1.043-1.045 x the algorithmic FETCH_SIZE (r04j/shift), that line fetched
 * twice. Candidates, all on the product's XCD tile map:
 *   EXNT 0   `ex` as a temporal load (the tile loads stay non-temporal)
 *   U 2      a wave realigns two adjacent tiles (128 vectors): tile 0's lane
 *            63 takes tile 1's first vector by readfirstlane, so one extra
 *            vector per 2 KiB instead of per 1 KiB
 * N = 1 is the all-gather row copy, N > 1 the one-shot combine (rd_tree). */
template <int N, int EXNT, int U, int CAP>
__global__ void __launch_bounds__(kReduceBlock)
k_ms(float *dst, SrcList srcs, size_t nvec)
{
    if constexpr (CAP) {
        UCG_MULTI_CAP_CLOBBER();
    }
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    const unsigned ntiles = gridDim.x;
    const size_t base = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, ntiles) * (kReduceBlock * U);
    const bool last_lane = threadIdx.x == kReduceBlock - 1;
    u32x4 lo[U][N], ex[N];
    unsigned r[N];
    const u32x4 *a4[N];
#pragma unroll
    for (int m = 0; m < N; m++) {
        const char *p = reinterpret_cast<const char*>(srcs.p[m]);
        r[m]  = (unsigned)((uintptr_t)p & 15);
        a4[m] = reinterpret_cast<const u32x4*>(p - r[m]);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = base + (size_t)u * kReduceBlock + threadIdx.x;
            lo[u][m] = ld16<1>(a4[m] + (i < nvec ? i : nvec));
        }
        const size_t e = base + (size_t)U * kReduceBlock;
        ex[m] = ld16<EXNT>(a4[m] + (last_lane && e <= nvec ? e : nvec));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < U; u++) {
        u32x4 val[N];
#pragma unroll
        for (int m = 0; m < N; m++) {
            u32x4 hi;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                hi[k] = from_next_lane(lo[u][m][k]);
            }
            if (u + 1 < U) {
                u32x4 nx;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    nx[k] = __builtin_amdgcn_readfirstlane(lo[u + 1 < U ? u + 1 : u][m][k]);
                }
                if (last_lane) hi = nx;
            } else if (last_lane) {
                hi = ex[m];
            }
            val[m] = funnel16(lo[u][m], hi, r[m]);
        }
        const size_t i = base + (size_t)u * kReduceBlock + threadIdx.x;
        if (i < nvec) {
            st16<1>(reinterpret_cast<u32x4*>(dst) + i, N == 1 ? val[0] : rd_tree<N>(val, fv));
        }
    }
}

template <int N, int EXNT, int U, int CAP>
static void run_ms(float *dst, const SrcList &s, size_t nvec)
{
    const unsigned g = (unsigned)((nvec + kReduceBlock * U - 1) / (kReduceBlock * U));
    hipLaunchKernelGGL((k_ms<N, EXNT, U, CAP>), dim3(g), dim3(kReduceBlock), 0, 0, dst, s, nvec);
}

/* The all-gather of 8 rows whose sources are all 4 B out of dst's phase
 * (k_gather_multi's case). The product deals workgroups round-robin over the
 * rows (MAP 0: row = b % 8, tile = b / 8, so row r runs on XCD r); MAP 1
 * walks the rows one after another on the XCD tile map of k_ms (a row's
 * tiles in runs of 64 per XCD). Both realign as k_ms<1, EXNT, 1>. PMC put
 * the product at 1.047 x the algorithmic FETCH_SIZE with either ex policy
 * (r04j, r04l), against 1.002 x for the one-source copy with a temporal ex. */
template <int EXNT, int MAP>
__global__ void __launch_bounds__(kReduceBlock)
k_gather_ms(char *dst, SrcList srcs, size_t row_bytes, size_t nvec)
{
    const unsigned tpr = (unsigned)((nvec + kReduceBlock - 1) / kReduceBlock);
    unsigned r, t;
    if (MAP == 0) {
        r = blockIdx.x % 8;
        t = blockIdx.x / 8;
    } else {
        const unsigned g = xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x);
        r = g / tpr;
        t = g % tpr;
    }
    const char *p = static_cast<const char*>(srcs.p[r]);
    const unsigned rs = (unsigned)((uintptr_t)p & 15);
    const u32x4 *a4 = reinterpret_cast<const u32x4*>(p - rs);
    const size_t i = (size_t)t * kReduceBlock + threadIdx.x;
    const bool last_lane = threadIdx.x == kReduceBlock - 1;
    const u32x4 lo = ld16<1>(a4 + (i < nvec ? i : nvec));
    const u32x4 ex = ld16<EXNT>(a4 + (last_lane && i < nvec ? i + 1 : nvec));
    u32x4 hi;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        hi[k] = from_next_lane(lo[k]);
    }
    if (last_lane) {
        hi = ex;
    }
    if (i < nvec) {
        st16<1>(reinterpret_cast<u32x4*>(dst + (size_t)r * row_bytes) + i, funnel16(lo, hi, rs));
    }
}

/* round 6: k_gather_ms<0, 0> with two consecutive tiles of its row per wave:
 * tile 0's lane 63 takes tile 1's first vector from tile 1's own load
 * (readfirstlane), so one extra vector per 2 KiB */
template <int U>
__global__ void __launch_bounds__(kReduceBlock)
k_gather_msu(char *dst, SrcList srcs, size_t row_bytes, size_t nvec)
{
    const unsigned r = blockIdx.x % 8, t = blockIdx.x / 8;
    const char *p = static_cast<const char*>(srcs.p[r]);
    const unsigned rs = (unsigned)((uintptr_t)p & 15);
    const u32x4 *a4 = reinterpret_cast<const u32x4*>(p - rs);
    const size_t i0 = (size_t)t * U * kReduceBlock + threadIdx.x;
    const bool last_lane = threadIdx.x == kReduceBlock - 1;
    u32x4 lo[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = i0 + (size_t)u * kReduceBlock;
        lo[u] = ld16<1>(a4 + (i < nvec ? i : nvec));
    }
    const size_t il = i0 + (size_t)(U - 1) * kReduceBlock;
    u32x4 ex = {0, 0, 0, 0};
    if (rs) {
        ex = ld16<0>(a4 + (last_lane && il < nvec ? il + 1 : nvec));
    }
    __builtin_amdgcn_sched_barrier(0);
    u32x4 *o = reinterpret_cast<u32x4*>(dst + (size_t)r * row_bytes);
#pragma unroll
    for (int u = 0; u < U; u++) {
        u32x4 v = lo[u];
        if (rs) {
            u32x4 hi, nx;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                hi[k] = from_next_lane(lo[u][k]);
                nx[k] = __builtin_amdgcn_readfirstlane(lo[u + 1 < U ? u + 1 : u][k]);
            }
            if (last_lane) {
                hi = u + 1 < U ? nx : ex;
            }
            v = funnel16(lo[u], hi, rs);
        }
        const size_t i = i0 + (size_t)u * kReduceBlock;
        if (i < nvec) {
            st16<1>(o + i, v);
        }
    }
}

/* In-phase operands (round 4, r04o): the realigning kernel fed in-phase
 * operands read 84.8 % where k_reduce_multi read 79.9 % (capped, N = 8). What
 * of the realigning kernel does it? All forms capped, on the XCD tile map:
 *   MODE 0  clamped unmasked loads + sched barrier, nothing else
 *   MODE 1  as 0, plus the temporal loads of the realigning kernel (lane 63
 *           the next tile's first vector, the other lanes the operand's last),
 *           kept alive and unused
 *   MODE 2  as 0, plus lane 63's next-tile load alone (masked) */
template <int N, int MODE>
__global__ void __launch_bounds__(kReduceBlock)
k_mx(float *dst, SrcList srcs, size_t nvec)
{
    UCG_MULTI_CAP_CLOBBER();
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    const size_t i = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * kReduceBlock +
                     threadIdx.x;
    const bool last_lane = threadIdx.x == kReduceBlock - 1;
    u32x4 val[N], ex[N];
#pragma unroll
    for (int m = 0; m < N; m++) {
        const u32x4 *a4 = reinterpret_cast<const u32x4*>(srcs.p[m]);
        val[m] = ld16<1>(a4 + (i < nvec ? i : nvec - 1));
        if (MODE == 1) {
            ex[m] = ld16<0>(a4 + (last_lane && i + 1 < nvec ? i + 1 : nvec - 1));
        } else if (MODE == 2) {
            if (last_lane && i + 1 < nvec) {
                ex[m] = ld16<0>(a4 + i + 1);
            } else {
                ex[m] = u32x4{0, 0, 0, 0};
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (MODE != 0) {
#pragma unroll
        for (int m = 0; m < N; m++) {
            asm volatile("" :: "v"(ex[m][0]));
        }
    }
    if (i < nvec) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + i, rd_tree<N>(val, fv));
    }
}

/* The 2-operand combine (the headline kernel, k_reduce<.., XM=0>), in phase,
 * with the pieces of the realigning kernel that sped the 8-operand form:
 *   MODE 0  clamped unmasked loads + sched barrier
 *   MODE 1  + a temporal load of src: lane 63 the next tile's first vector,
 *           the other lanes src's last vector (as k_reduce_shift's `ex`)
 *   MODE 2  + the same for dst
 *   MODE 3  + only the other lanes' load (every lane src's last vector)
 * XMAP 1: the XCD tile map. */
template <int MODE, int XMAP, unsigned C = kXcdChunk>
__global__ void __launch_bounds__(kReduceBlock)
k2x(float *dst, const float *src, size_t nvec)
{
    const size_t tile = XMAP ? xcd_tile<C>(blockIdx.x, gridDim.x) : blockIdx.x;
    const size_t i = tile * kReduceBlock + threadIdx.x;
    const bool last_lane = threadIdx.x == kReduceBlock - 1;
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4 = reinterpret_cast<u32x4*>(dst);
    const size_t ic = i < nvec ? i : nvec - 1;
    const u32x4 a = ld16<1>(s4 + ic);
    const u32x4 b = ld16<1>(d4 + ic);
    u32x4 e0 = {0, 0, 0, 0}, e1 = {0, 0, 0, 0};
    const size_t nx = (MODE != 3 && last_lane && i + 1 < nvec) ? i + 1 : nvec - 1;
    if (MODE >= 1) {
        e0 = ld16<0>(s4 + nx);
    }
    if (MODE == 2) {
        e1 = ld16<0>(d4 + nx);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (MODE >= 1) {
        asm volatile("" :: "v"(e0[0]), "v"(e1[0]));
    }
    if (i < nvec) {
        st16<1>(d4 + i, vapply<float, 0>(a, b));
    }
}

/* More of the PF idea (2-operand combine, XCD map): the last K lanes each
 * load one line of tile + DIST (lane 63 its first line, lane 62 its second,
 * ...) temporally and discard it; DST also does so for dst. */
template <int K, int DST, int DIST, unsigned C = kXcdChunk, int EDGE = 1>
__global__ void __launch_bounds__(kReduceBlock)
k2p(float *dst, const float *src, size_t nvec)
{
    const size_t tile = xcd_tile<C>(blockIdx.x, gridDim.x);
    const unsigned lane = threadIdx.x;
    /* EDGE 0: no prefetch by the last tile of an XCD's chunk (its neighbour
     * runs on another XCD, which would fetch the lines again) */
    const bool edge = EDGE == 0 && (tile % C) == C - 1;
    const size_t i = tile * kReduceBlock + lane;
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4 = reinterpret_cast<u32x4*>(dst);
    const size_t ic = i < nvec ? i : nvec - 1;
    const u32x4 a = ld16<1>(s4 + ic);
    const u32x4 b = ld16<1>(d4 + ic);
    const unsigned k = kReduceBlock - 1 - lane;          /* 0 for lane 63 */
    const size_t want = (tile + DIST) * kReduceBlock + (size_t)k * 8;
    const size_t nx = (k < (unsigned)K && want < nvec && !edge) ? want : nvec - 1;
    const u32x4 e0 = ld16<0>(s4 + nx);
    u32x4 e1 = {0, 0, 0, 0};
    if (DST) {
        e1 = ld16<0>(d4 + nx);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" :: "v"(e0[0]), "v"(e1[0]));
    if (i < nvec) {
        st16<1>(d4 + i, vapply<float, 0>(a, b));
    }
}

/* Round 6: the headline's PF form (XCD map, the first PF lines of the next
 * tile's src temporally) with its loads and store issued as buffer
 * instructions carrying explicit cache-policy bits (1 sc0, 2 nt, 16 sc1;
 * the product uses nt for both). Offsets 32-bit: < 4 GiB per operand. */
template <int LAUX, int SAUX, int PF = 3>
__global__ void __launch_bounds__(kReduceBlock)
k2buf(float *dst, const float *src, size_t nvec)
{
    const size_t i  = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * kReduceBlock +
                      threadIdx.x;
    const size_t ic = i < nvec ? i : nvec - 1;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), 0,
                                                                  0xffffffffu, 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0xffffffffu,
                                                                  0x00020000);
    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(ic * 16), 0, LAUX);
    const u32x4 b = __builtin_amdgcn_raw_buffer_load_b128(rd, (unsigned)(ic * 16), 0, LAUX);
    const unsigned k  = kReduceBlock - 1 - threadIdx.x;
    const size_t want = (i - threadIdx.x + kReduceBlock) + (size_t)k * 8;
    const u32x4 pf = ld16<0>(reinterpret_cast<const u32x4*>(src) +
                             (k < (unsigned)PF && want < nvec ? want : nvec - 1));
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" :: "v"(pf[0]));
    if (i < nvec) {
        __builtin_amdgcn_raw_buffer_store_b128(vapply<float, 0>(a, b), rd, (unsigned)(i * 16), 0,
                                               SAUX);
    }
}

struct Case {
    std::string name;
    double bytes;
    std::function<void()> run;
    std::vector<float> us;
    bool flushed = false;   /* each launch timed alone after a 3 GiB stream */
};

int main(int argc, char **argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    const size_t n = (size_t)1 << 26, nvec = n / 4;
    const size_t nm = (size_t)1 << 24, nvm = nm / 4;
    /* dst holds the largest output: n elements, or the gather's 8 rows of nm */
    const size_t nd = std::max(n, 8 * nm);
    float *src, *dst, *ref;
    CHECK(hipMalloc(&src, n * 4 + 4096));
    CHECK(hipMalloc(&dst, nd * 4));
    CHECK(hipMalloc(&ref, nd * 4));
    const float *s4 = src + 1;                        /* 4 B past dst's phase */
    /* the north-star size: 2 x 1 GiB, in phase */
    const size_t ng = (size_t)1 << 28, nvg = ng / 4;
    const unsigned gg = (unsigned)(nvg / kReduceBlock);
    float *srcg, *dstg;
    CHECK(hipMalloc(&srcg, ng * 4));
    CHECK(hipMalloc(&dstg, ng * 4));
    hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                       (void*)srcg, 1, 11ull, ng);
    hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                       (void*)dstg, 1, 12ull, ng);
    const unsigned gg0 = (unsigned)(((ng / 4) + kReduceBlock - 1) / kReduceBlock);
    auto flush = [&] {
        hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock>), dim3(gg0),
                           dim3(kReduceBlock), 0, 0, dstg, (const float*)srcg, (size_t)0,
                           ng / 4, (size_t)0);
    };
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
                       (void*)ref, 1, 9ull, nd);
    CHECK(hipDeviceSynchronize());
    const unsigned g2 = (unsigned)(nvec / kReduceBlock), gm = (unsigned)(nvm / kReduceBlock);
    SrcList s1 = sl_al;
    s1.p[0] = s4;

    std::vector<Case> cs = {
        {"2-op aligned k_reduce (round 3's form)", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock>), dim3(g2),
                                dim3(kReduceBlock), 0, 0, dst, (const float*)src, (size_t)0,
                                nvec, (size_t)0); }, {}},
        {"2-op shift, 1 line ahead (round 4 r04l-r04w)", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce_shift<float, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0,
                                dst, s4, (size_t)0, nvec, (size_t)0, 0u); }, {}},
        {"2-op shift, 4 lines ahead", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce_shift<float, 0, 1, 4>), dim3(g2), dim3(kReduceBlock), 0, 0,
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
        {"gather 8 rows, round-robin, ex nt", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_ms<1, 0>), dim3(8 * gm), dim3(kReduceBlock), 0, 0,
                                (char*)dst, sl, nm * 4, nvm); }, {}},
        {"gather 8 rows, round-robin, ex temporal", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_ms<0, 0>), dim3(8 * gm), dim3(kReduceBlock), 0, 0,
                                (char*)dst, sl, nm * 4, nvm); }, {}},
        {"gather 8 rows, XCD map, ex temporal", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_ms<0, 1>), dim3(8 * gm), dim3(kReduceBlock), 0, 0,
                                (char*)dst, sl, nm * 4, nvm); }, {}},
        /* round 6: the same layout with every source in
         * phase (the aligned path), and the out-of-phase rows with fewer
         * waves per CU (dynamic LDS bounding the one-wave workgroups) */
        {"gather 8 rows in phase, round-robin", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_ms<0, 0>), dim3(8 * gm), dim3(kReduceBlock), 0, 0,
                                (char*)dst, sl_al, nm * 4, nvm); }, {}},
        {"gather 8 rows, round-robin, ex temporal, 16 waves/CU", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_ms<0, 0>), dim3(8 * gm), dim3(kReduceBlock), 10240, 0,
                                (char*)dst, sl, nm * 4, nvm); }, {}},
        {"gather 8 rows, round-robin, ex temporal, 12 waves/CU", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_ms<0, 0>), dim3(8 * gm), dim3(kReduceBlock), 13653, 0,
                                (char*)dst, sl, nm * 4, nvm); }, {}},
        {"gather 8 rows, round-robin, ex temporal, 8 waves/CU", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_ms<0, 0>), dim3(8 * gm), dim3(kReduceBlock), 20480, 0,
                                (char*)dst, sl, nm * 4, nvm); }, {}},
        {"gather 8 rows, round-robin, 2 tiles per wave", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_msu<2>), dim3(8 * ((gm + 1) / 2)), dim3(kReduceBlock), 0, 0,
                                (char*)dst, sl, nm * 4, nvm); }, {}},
        {"gather 8 rows, round-robin, 4 tiles per wave", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_msu<4>), dim3(8 * ((gm + 3) / 4)), dim3(kReduceBlock), 0, 0,
                                (char*)dst, sl, nm * 4, nvm); }, {}},
        {"gather 8 rows in phase, 1 tile per wave (msu)", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_msu<1>), dim3(8 * gm), dim3(kReduceBlock), 0, 0,
                                (char*)dst, sl_al, nm * 4, nvm); }, {}},
        {"gather 8 rows in phase, 2 tiles per wave", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_msu<2>), dim3(8 * ((gm + 1) / 2)), dim3(kReduceBlock), 0, 0,
                                (char*)dst, sl_al, nm * 4, nvm); }, {}},
        {"gather 8 rows in phase, 4 tiles per wave", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_msu<4>), dim3(8 * ((gm + 3) / 4)), dim3(kReduceBlock), 0, 0,
                                (char*)dst, sl_al, nm * 4, nvm); }, {}},
        {"gather 8 rows, round-robin, 1 tile per wave (msu)", 2.0 * 8 * nm * 4, [&] {
             hipLaunchKernelGGL((k_gather_msu<1>), dim3(8 * gm), dim3(kReduceBlock), 0, 0,
                                (char*)dst, sl, nm * 4, nvm); }, {}},
        {"N=8 aligned capped, XCD map", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_multi<float, 0, 8, 1, 1>), dim3(gm), dim3(kReduceBlock),
                                0, 0, dst, sl_al, 0u, (size_t)0, nvm, (size_t)0); }, {}},
        {"N=4 aligned capped", 5.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_multi<float, 0, 4, 0, 1>), dim3(gm), dim3(kReduceBlock),
                                0, 0, dst, sl_al, 0u, (size_t)0, nvm, (size_t)0); }, {}},
        {"N=4 aligned capped, XCD map", 5.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_multi<float, 0, 4, 1, 1>), dim3(gm), dim3(kReduceBlock),
                                0, 0, dst, sl_al, 0u, (size_t)0, nvm, (size_t)0); }, {}},
        {"tree n=8 aligned capped", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_tree<float, 0, 8, 0, 1>), dim3(gm), dim3(kReduceBlock),
                                0, 0, dst, sl_al, 8u, (size_t)0, nvm, (size_t)0); }, {}},
        {"tree n=8 aligned capped, XCD map", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_tree<float, 0, 8, 1, 1>), dim3(gm), dim3(kReduceBlock),
                                0, 0, dst, sl_al, 8u, (size_t)0, nvm, (size_t)0); }, {}},
        {"N=8 aligned via the shift kernel (capped)", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_multi_shift<float, 0, 8, 1>), dim3(gm),
                                dim3(kReduceBlock), 0, 0, dst, sl_al, 0u, (size_t)0, nvm,
                                (size_t)0); }, {}},
        {"N=4 aligned via the shift kernel (capped)", 5.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_multi_shift<float, 0, 4, 1>), dim3(gm),
                                dim3(kReduceBlock), 0, 0, dst, sl_al, 0u, (size_t)0, nvm,
                                (size_t)0); }, {}},
        {"tree n=8 aligned via the shift kernel (capped)", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_reduce_tree_shift<float, 0, 8, 1>), dim3(gm),
                                dim3(kReduceBlock), 0, 0, dst, sl_al, 8u, (size_t)0, nvm,
                                (size_t)0); }, {}},
        {"N=8 aligned, clamp + barrier", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_mx<8, 0>), dim3(gm), dim3(kReduceBlock), 0, 0, dst, sl_al,
                                nvm); }, {}},
        {"N=8 aligned, + temporal extra loads", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_mx<8, 1>), dim3(gm), dim3(kReduceBlock), 0, 0, dst, sl_al,
                                nvm); }, {}},
        {"N=8 aligned, + lane-63 next-tile load", 9.0 * nm * 4, [&] {
             hipLaunchKernelGGL((k_mx<8, 2>), dim3(gm), dim3(kReduceBlock), 0, 0, dst, sl_al,
                                nvm); }, {}},
        {"2-op product: k_reduce PF=3 (next tile's first 3 lines)", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock, 1, 3>), dim3(g2),
                                dim3(kReduceBlock), 0, 0, dst, (const float*)src, (size_t)0,
                                nvec, (size_t)0); }, {}},
        {"2-op buffer ld/st nt (= product)", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2buf<2, 2>), dim3(g2), dim3(kReduceBlock), 0, 0, dst,
                                (const float*)src, nvec); }, {}},
        {"2-op buffer ld nt, st sc0 sc1 nt", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2buf<2, 19>), dim3(g2), dim3(kReduceBlock), 0, 0, dst,
                                (const float*)src, nvec); }, {}},
        {"2-op buffer ld nt, st nt sc1", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2buf<2, 18>), dim3(g2), dim3(kReduceBlock), 0, 0, dst,
                                (const float*)src, nvec); }, {}},
        {"2-op buffer ld nt, st sc0 nt", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2buf<2, 3>), dim3(g2), dim3(kReduceBlock), 0, 0, dst,
                                (const float*)src, nvec); }, {}},
        {"2-op buffer ld sc1 nt, st nt", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2buf<18, 2>), dim3(g2), dim3(kReduceBlock), 0, 0, dst,
                                (const float*)src, nvec); }, {}},
        {"2-op buffer ld sc0 sc1 nt, st nt", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2buf<19, 2>), dim3(g2), dim3(kReduceBlock), 0, 0, dst,
                                (const float*)src, nvec); }, {}},
        {"2-op buffer ld default, st nt", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2buf<0, 2>), dim3(g2), dim3(kReduceBlock), 0, 0, dst,
                                (const float*)src, nvec); }, {}},
        {"2-op buffer ld nt, st sc1", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2buf<2, 16>), dim3(g2), dim3(kReduceBlock), 0, 0, dst,
                                (const float*)src, nvec); }, {}},
        {"2-op k_reduce PF=4 (next tile's first 4 lines)", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock, 1, 4>), dim3(g2),
                                dim3(kReduceBlock), 0, 0, dst, (const float*)src, (size_t)0,
                                nvec, (size_t)0); }, {}},
        {"2-op k_reduce PF=1 (next-tile first line)", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock, 1, 1>), dim3(g2),
                                dim3(kReduceBlock), 0, 0, dst, (const float*)src, (size_t)0,
                                nvec, (size_t)0); }, {}},
        {"1 GiB: round 3's k_reduce", 3.0 * ng * 4, [&] {
             hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock>), dim3(gg),
                                dim3(kReduceBlock), 0, 0, dstg, (const float*)srcg, (size_t)0,
                                nvg, (size_t)0); }, {}},
        {"1 GiB: k_reduce PF=1", 3.0 * ng * 4, [&] {
             hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock, 1, 1>), dim3(gg),
                                dim3(kReduceBlock), 0, 0, dstg, (const float*)srcg, (size_t)0,
                                nvg, (size_t)0); }, {}},
        {"1 GiB: PF, chunk 128", 3.0 * ng * 4, [&] {
             hipLaunchKernelGGL((k2x<1, 1, 128>), dim3(gg), dim3(kReduceBlock), 0, 0, dstg,
                                srcg, nvg); }, {}},
        {"1 GiB: PF, chunk 32", 3.0 * ng * 4, [&] {
             hipLaunchKernelGGL((k2x<1, 1, 32>), dim3(gg), dim3(kReduceBlock), 0, 0, dstg,
                                srcg, nvg); }, {}},
        {"256 MiB: PF, chunk 128", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2x<1, 1, 128>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src,
                                nvec); }, {}},
        {"256 MiB: PF, chunk 32", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2x<1, 1, 32>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src,
                                nvec); }, {}},
        {"256 MiB cache-flushed: round 3's k_reduce", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock>), dim3(g2),
                                dim3(kReduceBlock), 0, 0, dst, (const float*)src, (size_t)0,
                                nvec, (size_t)0); }, {}, true},
        {"256 MiB cache-flushed: product (PF)", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce<float, 0, 1, 1, kReduceBlock, 1, 1>), dim3(g2),
                                dim3(kReduceBlock), 0, 0, dst, (const float*)src, (size_t)0,
                                nvec, (size_t)0); }, {}, true},
        {"256 MiB cache-flushed: realigning kernel, src 4 B off", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce_shift<float, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0,
                                dst, s4, (size_t)0, nvec, (size_t)0, 0u); }, {}, true},
        {"PF: 2 lines of the next tile", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<2, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"PF: 4 lines of the next tile", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<4, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"PF: src and dst line of the next tile", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<1, 1, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"PF: first line two tiles ahead", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<1, 0, 2>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"PF: 8 lines (the whole next tile)", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<8, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"PF: 4 lines of src and of dst", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<4, 1, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"PF: 2 lines, chunk 128", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<2, 0, 1, 128>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"PF: 4 lines, chunk 128", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<4, 0, 1, 128>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"1 GiB: PF 2 lines", 3.0 * ng * 4, [&] {
             hipLaunchKernelGGL((k2p<2, 0, 1>), dim3(gg), dim3(kReduceBlock), 0, 0, dstg, srcg, nvg); }, {}},
        {"1 GiB: PF 4 lines", 3.0 * ng * 4, [&] {
             hipLaunchKernelGGL((k2p<4, 0, 1>), dim3(gg), dim3(kReduceBlock), 0, 0, dstg, srcg, nvg); }, {}},
        {"1 GiB: PF 4 lines, chunk 128", 3.0 * ng * 4, [&] {
             hipLaunchKernelGGL((k2p<4, 0, 1, 128>), dim3(gg), dim3(kReduceBlock), 0, 0, dstg, srcg, nvg); }, {}},
        {"256 MiB cache-flushed: PF 4 lines", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<4, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}, true},
        {"PF: 3 lines", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<3, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"PF: 5 lines", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<5, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"PF: 6 lines", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<6, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"PF: 4 lines, none at chunk edges", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<4, 0, 1, kXcdChunk, 0>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"1 GiB: PF 4 lines, none at chunk edges", 3.0 * ng * 4, [&] {
             hipLaunchKernelGGL((k2p<4, 0, 1, kXcdChunk, 0>), dim3(gg), dim3(kReduceBlock), 0, 0, dstg, srcg, nvg); }, {}},
        {"1 GiB: PF 3 lines", 3.0 * ng * 4, [&] {
             hipLaunchKernelGGL((k2p<3, 0, 1>), dim3(gg), dim3(kReduceBlock), 0, 0, dstg, srcg, nvg); }, {}},
        {"256 MiB cache-flushed: PF 3 lines", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<3, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}, true},
        {"1 GiB: PF 6 lines", 3.0 * ng * 4, [&] {
             hipLaunchKernelGGL((k2p<6, 0, 1>), dim3(gg), dim3(kReduceBlock), 0, 0, dstg, srcg, nvg); }, {}},
        {"PF: 1 line (k2p)", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2p<1, 0, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"2-op clamp + barrier", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2x<0, 0>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"2-op + temporal src extra", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2x<1, 0>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"2-op + temporal src, dst extra", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2x<2, 0>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"2-op + uniform last-vector load", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2x<3, 0>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"2-op + temporal src extra, XCD map", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k2x<1, 1>), dim3(g2), dim3(kReduceBlock), 0, 0, dst, src, nvec); }, {}},
        {"2-op aligned via the shift kernel", 3.0 * n * 4, [&] {
             hipLaunchKernelGGL((k_reduce_shift<float, 0, 0>), dim3(g2), dim3(kReduceBlock), 0, 0,
                                dst, (const float*)src, (size_t)0, nvec, (size_t)0, 0u); }, {}},
        {"copy shift, ex temporal", 2.0 * n * 4, [&] { run_ms<1, 0, 1, 0>(dst, s1, nvec); }, {}},
        {"copy shift, U=2", 2.0 * n * 4, [&] { run_ms<1, 1, 2, 0>(dst, s1, nvec); }, {}},
        {"copy shift, U=2 ex temporal", 2.0 * n * 4, [&] { run_ms<1, 0, 2, 0>(dst, s1, nvec); }, {}},
        {"N=8 shift capped, ex temporal", 9.0 * nm * 4, [&] { run_ms<8, 0, 1, 1>(dst, sl, nvm); }, {}},
        {"N=8 shift capped, U=2", 9.0 * nm * 4, [&] { run_ms<8, 1, 2, 1>(dst, sl, nvm); }, {}},
        {"N=8 shift capped, U=2 ex temporal", 9.0 * nm * 4, [&] { run_ms<8, 0, 2, 1>(dst, sl, nvm); }, {}},
    };

    /* bits: every form against its reference form, by name; each run starts
     * from the same output contents */
    auto idx = [&](const char *nm_) {
        for (size_t k = 0; k < cs.size(); k++) {
            if (cs[k].name == nm_) return (int)k;
        }
        fprintf(stderr, "no case %s\n", nm_);
        exit(2);
    };
    const char *pairs[][2] = {
        {"2-op shift, 1 line ahead (round 4 r04l-r04w)", "2-op plain misaligned"},
        {"2-op shift, 1 line ahead (round 4 r04l-r04w)", "2-op shift, 4 lines ahead"},
        {"copy shift (product's copy_row)", "copy plain misaligned"},
        {"N=8 shift (product)", "N=8 shift, VGPR-capped"},
        {"N=8 shift (product)", "N=8 plain misaligned (capped)"},
        {"gather 8 rows, round-robin, ex nt", "gather 8 rows, round-robin, ex temporal"},
        {"gather 8 rows, round-robin, ex nt", "gather 8 rows, XCD map, ex temporal"},
        {"gather 8 rows, round-robin, ex nt", "gather 8 rows, round-robin, ex temporal, 16 waves/CU"},
        {"gather 8 rows, round-robin, ex nt", "gather 8 rows, round-robin, ex temporal, 8 waves/CU"},
        {"gather 8 rows, round-robin, ex nt", "gather 8 rows, round-robin, 2 tiles per wave"},
        {"gather 8 rows, round-robin, ex nt", "gather 8 rows, round-robin, 4 tiles per wave"},
        {"gather 8 rows, round-robin, ex nt", "gather 8 rows, round-robin, 1 tile per wave (msu)"},
        {"gather 8 rows in phase, round-robin", "gather 8 rows in phase, 2 tiles per wave"},
        {"gather 8 rows in phase, round-robin", "gather 8 rows in phase, 4 tiles per wave"},
        {"gather 8 rows in phase, round-robin", "gather 8 rows in phase, 1 tile per wave (msu)"},
        {"N=8 aligned (capped)", "N=8 aligned capped, XCD map"},
        {"N=4 aligned capped", "N=4 aligned capped, XCD map"},
        {"tree n=8 aligned capped", "tree n=8 aligned capped, XCD map"},
        {"N=8 aligned (capped)", "N=8 aligned via the shift kernel (capped)"},
        {"N=4 aligned capped", "N=4 aligned via the shift kernel (capped)"},
        {"tree n=8 aligned capped", "tree n=8 aligned via the shift kernel (capped)"},
        {"N=8 aligned (capped)", "N=8 aligned, clamp + barrier"},
        {"N=8 aligned (capped)", "N=8 aligned, + temporal extra loads"},
        {"N=8 aligned (capped)", "N=8 aligned, + lane-63 next-tile load"},
        {"2-op aligned k_reduce (round 3's form)", "2-op k_reduce PF=1 (next-tile first line)"},
        {"2-op aligned k_reduce (round 3's form)", "2-op clamp + barrier"},
        {"2-op aligned k_reduce (round 3's form)", "2-op + temporal src extra"},
        {"2-op aligned k_reduce (round 3's form)", "2-op + temporal src, dst extra"},
        {"2-op aligned k_reduce (round 3's form)", "2-op + uniform last-vector load"},
        {"2-op aligned k_reduce (round 3's form)", "2-op + temporal src extra, XCD map"},
        {"2-op aligned k_reduce (round 3's form)", "2-op aligned via the shift kernel"},
        {"2-op aligned k_reduce (round 3's form)", "256 MiB cache-flushed: product (PF)"},
        {"2-op aligned k_reduce (round 3's form)", "256 MiB: PF, chunk 128"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 2 lines of the next tile"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 4 lines of the next tile"},
        {"2-op aligned k_reduce (round 3's form)", "PF: src and dst line of the next tile"},
        {"2-op aligned k_reduce (round 3's form)", "PF: first line two tiles ahead"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 1 line (k2p)"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 3 lines"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 5 lines"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 6 lines"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 4 lines, none at chunk edges"},
        {"1 GiB: round 3's k_reduce", "1 GiB: PF 4 lines, none at chunk edges"},
        {"1 GiB: round 3's k_reduce", "1 GiB: PF 6 lines"},
        {"1 GiB: round 3's k_reduce", "1 GiB: PF 3 lines"},
        {"2-op aligned k_reduce (round 3's form)", "2-op k_reduce PF=4 (next tile's first 4 lines)"},
        {"2-op aligned k_reduce (round 3's form)", "2-op product: k_reduce PF=3 (next tile's first 3 lines)"},
        {"2-op aligned k_reduce (round 3's form)", "2-op buffer ld/st nt (= product)"},
        {"2-op aligned k_reduce (round 3's form)", "2-op buffer ld nt, st sc0 sc1 nt"},
        {"2-op aligned k_reduce (round 3's form)", "2-op buffer ld sc0 sc1 nt, st nt"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 8 lines (the whole next tile)"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 4 lines of src and of dst"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 2 lines, chunk 128"},
        {"2-op aligned k_reduce (round 3's form)", "PF: 4 lines, chunk 128"},
        {"1 GiB: round 3's k_reduce", "1 GiB: PF 2 lines"},
        {"1 GiB: round 3's k_reduce", "1 GiB: PF 4 lines"},
        {"1 GiB: round 3's k_reduce", "1 GiB: PF 4 lines, chunk 128"},
        {"2-op aligned k_reduce (round 3's form)", "256 MiB: PF, chunk 32"},
        {"1 GiB: round 3's k_reduce", "1 GiB: k_reduce PF=1"},
        {"1 GiB: round 3's k_reduce", "1 GiB: PF, chunk 128"},
        {"1 GiB: round 3's k_reduce", "1 GiB: PF, chunk 32"},
        {"copy shift (product's copy_row)", "copy shift, ex temporal"},
        {"copy shift (product's copy_row)", "copy shift, U=2"},
        {"copy shift (product's copy_row)", "copy shift, U=2 ex temporal"},
        {"N=8 shift (product)", "N=8 shift capped, ex temporal"},
        {"N=8 shift (product)", "N=8 shift capped, U=2"},
        {"N=8 shift (product)", "N=8 shift capped, U=2 ex temporal"},
    };
    std::vector<uint32_t> a(nd), b(nd);
    std::vector<uint32_t> ag, bg;
    for (const auto &pr : pairs) {
        const std::string first = pr[0];
        const bool big = first.rfind("1 GiB", 0) == 0;
        /* N = 8 / 4 and the tree write nm elements, a gather 8 nm, 1 GiB ng,
         * the rest n */
        const size_t cmp = big ? ng
                         : (first.rfind("N=", 0) == 0 || first.rfind("tree", 0) == 0) ? nm
                         : first.rfind("gather", 0) == 0 ? 8 * nm : n;
        if (big && ag.empty()) {
            ag.resize(ng);
            bg.resize(ng);
        }
        for (int k = 0; k < 2; k++) {
            if (big) {
                hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, 0,
                                   (void*)dstg, 1, 12ull, ng);
            } else {
                CHECK(hipMemcpy(dst, ref, nd * 4, hipMemcpyDeviceToDevice));
            }
            cs[idx(pr[k])].run();
            CHECK(hipDeviceSynchronize());
            uint32_t *h = big ? (k ? bg.data() : ag.data()) : (k ? b.data() : a.data());
            CHECK(hipMemcpy(h, big ? dstg : dst, (big ? ng : nd) * 4, hipMemcpyDeviceToHost));
        }
        const bool same = big ? std::equal(ag.begin(), ag.end(), bg.begin())
                              : std::equal(a.begin(), a.begin() + cmp, b.begin());
        if (!same) {
            printf("MISMATCH %s vs %s\n", pr[0], pr[1]);
            return 3;
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; r++) {
        for (auto &c : cs) {
            c.run();
            if (c.flushed) {
                /* the 1 GiB combine between launches streams 3 GiB through
                 * L2 and the 256 MiB Infinity Cache: nothing of the previous
                 * launch's operands is left in either */
                float tot = 0;
                for (int i = 0; i < 20; i++) {
                    flush();
                    CHECK(hipEventRecord(e0, 0));
                    c.run();
                    CHECK(hipEventRecord(e1, 0));
                    CHECK(hipEventSynchronize(e1));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    tot += ms;
                }
                c.us.push_back(1000.f * tot / 20);
                continue;
            }
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
        printf("%-56s %9.2f us %6.1f %%\n", c.name.c_str(), med,
               100.0 * c.bytes / (med * 1e-6) / 8e12);
    }
    return 0;
}
