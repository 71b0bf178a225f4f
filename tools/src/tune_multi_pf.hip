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

/* Round 6: U vectors per lane per operand (a wave's tile is 64 x U vectors of
 * each operand, lane stride 64), XCD tile map over those tiles, PF1 of every
 * operand D tiles ahead - fewer, longer per-operand bursts per wave */
template <int N, int U, int D, int PF, int NTS = 1, int ROT = 0>
__global__ void __launch_bounds__(kReduceBlock)
k_multi_u(float *dst, SrcList srcs, size_t nvec)
{
    UCG_MULTI_CAP_CLOBBER();
    const size_t tile = xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x);
    const size_t base = tile * (kReduceBlock * U) + threadIdx.x;
    const u32x4 *op[N];
    u32x4 val[U][N];
#pragma unroll
    for (int m = 0; m < N; m++) {
        op[m] = reinterpret_cast<const u32x4*>(srcs.p[m]);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * kReduceBlock;
        const size_t ic = i < nvec ? i : nvec - 1;
        if constexpr (ROT) {
            /* the operands in an order rotated by the tile: the waves in
             * flight spread their first loads over all operands */
            const unsigned r = (unsigned)tile % N;
#pragma unroll
            for (int m = 0; m < N; m++) {
                const unsigned mm = (m + r) % N;
                const u32x4 v = ld16<1>(op[mm] + ic);
#pragma unroll
                for (int q = 0; q < N; q++) {
                    if ((unsigned)q == mm) val[u][q] = v;
                }
            }
        } else {
#pragma unroll
            for (int m = 0; m < N; m++) {
                val[u][m] = ld16<1>(op[m] + ic);
            }
        }
    }
    if constexpr (!PF) {
        __builtin_amdgcn_sched_barrier(0);     /* every load issued before any use */
    }
    if constexpr (PF) {
        const unsigned k  = kReduceBlock - 1 - threadIdx.x;
        /* lane 63 - u: the first line of row u of the tile D tiles ahead */
        const size_t want = tile * (kReduceBlock * U) + (size_t)D * kReduceBlock * U +
                            (size_t)k * kReduceBlock;
        const size_t at   = (k < (unsigned)U && want < nvec) ? want : nvec - 1;
        u32x4 pf[N];
#pragma unroll
        for (int m = 0; m < N; m++) {
            pf[m] = ld16<0>(op[m] + at);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < N; m++) {
            asm volatile("" :: "v"(pf[m][0]));
        }
    }
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * kReduceBlock;
        if (i < nvec) {
            st16<NTS>(reinterpret_cast<u32x4*>(dst) + i, rd_tree<N>(val[u], fv));
        }
    }
}

/* Round 6: the XCD tile map, then the superchunks (8 XCD chunks, 8 x 64
 * tiles) visited in a segmented order - superchunk s of G segments goes to
 * (s % G) * (nsc / G) + s / G - so the waves in flight cover G regions far
 * apart in every operand instead of one window (more DRAM banks busy with
 * 9 streams). A ragged remainder of superchunks keeps the identity. */
template <int N, int G, int D>
__global__ void __launch_bounds__(kReduceBlock)
k_multi_seg(float *dst, SrcList srcs, size_t nvec)
{
    UCG_MULTI_CAP_CLOBBER();
    const unsigned ntiles = gridDim.x;
    unsigned t = xcd_tile<kXcdChunk>(blockIdx.x, ntiles);
    constexpr unsigned SC = 8 * kXcdChunk;
    const unsigned nsc = ntiles / SC, full = (nsc / G) * G;
    if (t / SC < full) {
        const unsigned sc = t / SC, per = full / G;
        t = ((sc % G) * per + sc / G) * SC + t % SC;
    }
    const size_t i  = (size_t)t * kReduceBlock + threadIdx.x;
    const size_t ic = i < nvec ? i : nvec - 1;
    const u32x4 *op[N];
    u32x4 val[N];
#pragma unroll
    for (int m = 0; m < N; m++) {
        op[m]  = reinterpret_cast<const u32x4*>(srcs.p[m]);
        val[m] = ld16<1>(op[m] + ic);
    }
    next_tile_lines<1, N, D>(op, i, nvec);
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    if (i < nvec) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + i, rd_tree<N>(val, fv));
    }
}

/* Round 6: the product's PF form (every operand's line D tiles ahead) with
 * the store - and, BUFLD, the operand loads - issued as buffer instructions
 * carrying explicit cache-policy bits (AUX: 1 sc0, 2 nt, 16 sc1; the
 * product's non-temporal store is nt). Offsets are 32-bit: operands < 4 GiB. */
template <int N, int D, int SAUX, int BUFLD = 0, int LAUX = 2>
__global__ void __launch_bounds__(kReduceBlock)
k_multi_buf(float *dst, SrcList srcs, size_t nvec)
{
    UCG_MULTI_CAP_CLOBBER();
    const size_t i  = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * kReduceBlock +
                      threadIdx.x;
    const size_t ic = i < nvec ? i : nvec - 1;
    const u32x4 *op[N];
    u32x4 val[N];
#pragma unroll
    for (int m = 0; m < N; m++) {
        op[m] = reinterpret_cast<const u32x4*>(srcs.p[m]);
        if constexpr (BUFLD) {
            __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<void*>(srcs.p[m]), 0, 0xffffffffu, 0x00020000);
            val[m] = __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(ic * 16), 0, LAUX);
        } else {
            val[m] = ld16<1>(op[m] + ic);
        }
    }
    next_tile_lines<1, N, D>(op, i, nvec);
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    if (i < nvec) {
        __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0xffffffffu,
                                                                      0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(rd_tree<N>(val, fv), rd, (unsigned)(i * 16), 0,
                                               SAUX);
    }
}

/* Round 6 (r06v): the product's PF form with its prefetch lines issued
 * BEFORE the operand loads (the 2-operand combine gained 0.5-1.1 points at
 * 256 MiB from that order, tools/tune_order); PFM operands' lines D tiles
 * ahead, sched barriers fixing the order */
template <int N, int D, int PFM>
__global__ void __launch_bounds__(kReduceBlock)
k_multi_pffirst(float *dst, SrcList srcs, size_t nvec)
{
    UCG_MULTI_CAP_CLOBBER();
    const size_t i  = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * kReduceBlock +
                      threadIdx.x;
    const size_t ic = i < nvec ? i : nvec - 1;
    const u32x4 *op[N];
    u32x4 val[N], pf[PFM];
#pragma unroll
    for (int m = 0; m < N; m++) {
        op[m] = reinterpret_cast<const u32x4*>(srcs.p[m]);
    }
    const unsigned k  = kReduceBlock - 1 - threadIdx.x;
    const size_t want = (i - threadIdx.x + (size_t)D * kReduceBlock) + (size_t)k * 8;
    const size_t at   = (k < 1u && want < nvec) ? want : nvec - 1;
#pragma unroll
    for (int m = 0; m < PFM; m++) {
        pf[m] = ld16<0>(op[m] + at);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < N; m++) {
        val[m] = ld16<1>(op[m] + ic);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < PFM; m++) {
        asm volatile("" :: "v"(pf[m][0]));
    }
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    if (i < nvec) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + i, rd_tree<N>(val, fv));
    }
}

/* Round 6 (r06zq): the product's PF form (all operands' lines D tiles
 * ahead, after the loads or - PFO - before them) on XCD chunks of C tiles
 * (the product: 64; the 2-operand combine gained from 256 below 1 GiB) */
template <int N, int D, int PFO, unsigned C>
__global__ void __launch_bounds__(kReduceBlock)
k_multi_chunk(float *dst, SrcList srcs, size_t nvec)
{
    UCG_MULTI_CAP_CLOBBER();
    const size_t i  = (size_t)xcd_tile<C>(blockIdx.x, gridDim.x) * kReduceBlock + threadIdx.x;
    const size_t ic = i < nvec ? i : nvec - 1;
    const u32x4 *op[N];
    u32x4 val[N];
#pragma unroll
    for (int m = 0; m < N; m++) {
        op[m] = reinterpret_cast<const u32x4*>(srcs.p[m]);
    }
    if constexpr (PFO) {
        u32x4 pf[N];
        tile_lines_issue<1, N, D>(op, i, nvec, pf);
#pragma unroll
        for (int m = 0; m < N; m++) {
            val[m] = ld16<1>(op[m] + ic);
        }
        tile_lines_keep<N>(pf);
    } else {
#pragma unroll
        for (int m = 0; m < N; m++) {
            val[m] = ld16<1>(op[m] + ic);
        }
        next_tile_lines<1, N, D>(op, i, nvec);
    }
    auto fv = [](u32x4 a, u32x4 b) { return vapply<float, 0>(a, b); };
    if (i < nvec) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + i, rd_tree<N>(val, fv));
    }
}

/* the N operands read and dst written with zeros: the traffic of the
 * combine, no dependency of a store on its loads */
template <int N>
__global__ void __launch_bounds__(kReduceBlock)
k_read_store0(float *dst, SrcList srcs, size_t nvec)
{
    UCG_MULTI_CAP_CLOBBER();
    const size_t i = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * kReduceBlock +
                     threadIdx.x;
    if (i >= nvec) {
        return;
    }
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < N; m++) {
        acc ^= ld16<1>(reinterpret_cast<const u32x4*>(srcs.p[m]) + i);
    }
    st16<1>(reinterpret_cast<u32x4*>(dst) + i, u32x4{0, 0, 0, 0});
    if (acc[0] == 0x7fc00123u && acc[1] == 0x7fc00321u) {
        st16<1>(reinterpret_cast<u32x4*>(dst) + i, acc);
    }
}


/* Round 6: persistent waves - a grid of G one-wave workgroups (a multiple of
 * 8, so logical tile b + G stays on b's XCD) walks the same XCD tile map as
 * the product; PIPE issues the next tile's N loads before the current tile's
 * combine and store, so a wave always has loads in flight behind its store */
template <int N, int D, int PIPE, int CAPV = 1>
__global__ void __launch_bounds__(kReduceBlock)
k_multi_persist(float *dst, SrcList srcs, size_t nvec)
{
    if constexpr (CAPV) {
        UCG_MULTI_CAP_CLOBBER();
    }
    const unsigned ntiles = (unsigned)((nvec + kReduceBlock - 1) / kReduceBlock);
    const unsigned G = gridDim.x;
    unsigned b = blockIdx.x;
    if (b >= ntiles) {
        return;
    }
    const u32x4 *op[N];
#pragma unroll
    for (int m = 0; m < N; m++) {
        op[m] = reinterpret_cast<const u32x4*>(srcs.p[m]);
    }
    u32x4 *d4 = reinterpret_cast<u32x4*>(dst);
    auto fv = [](u32x4 a, u32x4 c) { return vapply<float, 0>(a, c); };
    size_t i = (size_t)xcd_tile<kXcdChunk>(b, ntiles) * kReduceBlock + threadIdx.x;
    u32x4 cur[N];
    {
        const size_t ic = i < nvec ? i : nvec - 1;
#pragma unroll
        for (int m = 0; m < N; m++) {
            cur[m] = ld16<1>(op[m] + ic);
        }
    }
    for (;;) {
        const unsigned bn = b + G;
        const bool more = bn < ntiles;
        const size_t in = more ? (size_t)xcd_tile<kXcdChunk>(bn, ntiles) * kReduceBlock +
                                 threadIdx.x : i;
        const size_t inc = in < nvec ? in : nvec - 1;
        /* the prefetch lines first, then the next tile's loads: waiting for
         * the prefetch (and so the current tile) leaves those in flight */
        const unsigned k  = kReduceBlock - 1 - threadIdx.x;
        const size_t want = (i - threadIdx.x + (size_t)D * kReduceBlock) + (size_t)k * 8;
        const size_t at   = (k < 1u && want < nvec) ? want : nvec - 1;
        u32x4 pf[N], nxt[N];
#pragma unroll
        for (int m = 0; m < N; m++) {
            pf[m] = ld16<0>(op[m] + at);
        }
        if constexpr (PIPE) {
#pragma unroll
            for (int m = 0; m < N; m++) {
                nxt[m] = ld16<1>(op[m] + inc);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < N; m++) {
            asm volatile("" :: "v"(pf[m][0]));
        }
        if (i < nvec) {
            st16<1>(d4 + i, rd_tree<N>(cur, fv));
        }
        if (!more) {
            break;
        }
#pragma unroll
        for (int m = 0; m < N; m++) {
            if constexpr (PIPE) {
                cur[m] = nxt[m];
            } else {
                cur[m] = ld16<1>(op[m] + inc);
            }
        }
        i = in;
        b = bn;
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
    MV("PF1, all operands, 8 tiles ahead", 1, 1, 1, N, true, 8);
    /* r06w: the product kernel with PFO = 1 (its lines issued first) */
    MV("product PFO, all operands, 2 tiles ahead", 1, 1, 1, N, true, 2, 1);
    MV("product PFO, all operands, 4 tiles ahead", 1, 1, 1, N, true, 4, 1);
    MV("product PFO, all operands, 8 tiles ahead", 1, 1, 1, N, true, 8, 1);
    MV("product PFO, operand 0, 4 tiles ahead", 1, 1, 1, 1, true, 4, 1);
#undef MV
    /* round 6: fewer waves per CU at large operands - the product form with
     * dynamic LDS bounding the workgroups (one wave each) per CU */
#define LV(label, D, LDS)                                                                 \
    vs.push_back({label, [](float *d, SrcList s, size_t nv, hipStream_t q) {             \
        hipLaunchKernelGGL((k_reduce_multi<float, 0, N, 1, 1, 1, N, D>), dim3(tiles(nv)),  \
                           dim3(kReduceBlock), LDS, q, d, s, 0u, (size_t)0, nv, (size_t)0); \
    }, true, {}})
    LV("PF1 all, 2 ahead, LDS cap 8 waves/CU", 2, 20480);
    LV("PF1 all, 4 ahead, LDS cap 8 waves/CU", 4, 20480);
    LV("PF1 all, 2 ahead, LDS cap 6 waves/CU", 2, 27306);
    LV("PF1 all, 4 ahead, LDS cap 6 waves/CU", 4, 27306);
    LV("PF1 all, 4 ahead, LDS cap 10 waves/CU", 4, 16384);
#undef LV
#define UV(label, U, D, PF, ...)                                                         \
    vs.push_back({label, [](float *d, SrcList s, size_t nv, hipStream_t q) {             \
        hipLaunchKernelGGL((k_multi_u<N, U, D, PF __VA_OPT__(,) __VA_ARGS__>),            \
                           dim3((unsigned)((nv + kReduceBlock * U - 1) / (kReduceBlock * U))), \
                           dim3(kReduceBlock), 0, q, d, s, nv);                           \
    }, true, {}})
#define BV(label, D, SAUX, ...)                                                          \
    vs.push_back({label, [](float *d, SrcList s, size_t nv, hipStream_t q) {             \
        hipLaunchKernelGGL((k_multi_buf<N, D, SAUX __VA_OPT__(,) __VA_ARGS__>), dim3(tiles(nv)), \
                           dim3(kReduceBlock), 0, q, d, s, nv);                           \
    }, true, {}})
    BV("buffer store nt (= product), 2 ahead", 2, 2);
    BV("buffer store nt, 4 ahead", 4, 2);
    BV("buffer store default policy, 4 ahead", 4, 0);
    BV("buffer store sc0, 4 ahead", 4, 1);
    BV("buffer store sc1, 4 ahead", 4, 16);
    BV("buffer store sc0 sc1, 4 ahead", 4, 17);
    BV("buffer store nt sc1, 4 ahead", 4, 18);
    BV("buffer store sc0 sc1 nt, 4 ahead", 4, 19);
    BV("buffer store sc0 nt, 4 ahead", 4, 3);
    BV("buffer loads nt + store nt, 4 ahead", 4, 2, 1, 2);
    BV("buffer loads sc1 nt + store nt, 4 ahead", 4, 2, 1, 18);
    BV("buffer loads sc0 sc1 nt + store nt, 4 ahead", 4, 2, 1, 19);
    BV("buffer loads default + store nt, 4 ahead", 4, 2, 1, 0);
#undef BV
#define SV(label, G, D)                                                                  \
    vs.push_back({label, [](float *d, SrcList s, size_t nv, hipStream_t q) {             \
        hipLaunchKernelGGL((k_multi_seg<N, G, D>), dim3(tiles(nv)), dim3(kReduceBlock), 0, q, \
                           d, s, nv);                                                     \
    }, true, {}})
    SV("segmented superchunks G=4, PF1 2 ahead", 4, 2);
    SV("segmented superchunks G=16, PF1 2 ahead", 16, 2);
    SV("segmented superchunks G=64, PF1 2 ahead", 64, 2);
    SV("segmented superchunks G=16, PF1 4 ahead", 16, 4);
#undef SV
    UV("U1, clamped loads + sched barrier, no prefetch", 1, 1, 0);
    if constexpr (N <= 8) {
        UV("U1, PF1 4 tiles ahead, temporal store", 1, 4, 1, 0);
        UV("U1, PF1 4 tiles ahead, rotated operand order", 1, 4, 1, 1, 1);
        UV("U1, PF1 2 tiles ahead, rotated operand order", 1, 2, 1, 1, 1);
        UV("U2, no prefetch", 2, 1, 0);
        UV("U2, PF1 per 64-vector row, 1 tile ahead", 2, 1, 1);
        UV("U2, PF1 per 64-vector row, 2 tiles ahead", 2, 2, 1);
        UV("U4, no prefetch", 4, 1, 0);
        UV("U4, PF1 per row, 1 tile ahead", 4, 1, 1);
    }
#undef UV
    /* round 6 (r06p): persistent waves, and occupancy between 12 and 16
     * waves per CU (uncapped registers, LDS bounding the workgroups) */
#define PV(label, G, D, PIPE, CAPV)                                                      \
    vs.push_back({label, [](float *d, SrcList s, size_t nv, hipStream_t q) {             \
        hipLaunchKernelGGL((k_multi_persist<N, D, PIPE, CAPV>), dim3(G), dim3(kReduceBlock), \
                           0, q, d, s, nv);                                               \
    }, true, {}})
    PV("persistent 12/CU, no pipeline, 4 ahead", 3072, 4, 0, 1);
    PV("persistent 12/CU, pipelined, 4 ahead", 3072, 4, 1, 1);
    PV("persistent 12/CU, pipelined, 2 ahead", 3072, 2, 1, 1);
    PV("persistent 8/CU, pipelined, 4 ahead", 2048, 4, 1, 1);
    PV("persistent 16/CU, pipelined, 4 ahead", 4096, 4, 1, 0);
    PV("persistent 16/CU, no pipeline, 4 ahead", 4096, 4, 0, 0);
#undef PV
#define CV(label, D, PFO, C)                                                             \
    vs.push_back({label, [](float *d, SrcList s, size_t nv, hipStream_t q) {             \
        hipLaunchKernelGGL((k_multi_chunk<N, D, PFO, C>), dim3(tiles(nv)),               \
                           dim3(kReduceBlock), 0, q, d, s, nv);                           \
    }, true, {}})
    CV("chunk 64, lines after, 4 ahead", 4, 0, 64);
    CV("chunk 128, lines after, 4 ahead", 4, 0, 128);
    CV("chunk 256, lines after, 4 ahead", 4, 0, 256);
    CV("chunk 64, lines first, 4 ahead", 4, 1, 64);
    CV("chunk 128, lines first, 4 ahead", 4, 1, 128);
    CV("chunk 256, lines first, 4 ahead", 4, 1, 256);
#undef CV
#define FV(label, D, PFM)                                                                \
    vs.push_back({label, [](float *d, SrcList s, size_t nv, hipStream_t q) {             \
        hipLaunchKernelGGL((k_multi_pffirst<N, D, PFM>), dim3(tiles(nv)),                 \
                           dim3(kReduceBlock), 0, q, d, s, nv);                           \
    }, true, {}})
    FV("prefetch first, all operands, 2 tiles ahead", 2, N);
    FV("prefetch first, all operands, 4 tiles ahead", 4, N);
    FV("prefetch first, operand 0, 2 tiles ahead", 2, 1);
#undef FV
#define OV(label, D, LDS)                                                                 \
    vs.push_back({label, [](float *d, SrcList s, size_t nv, hipStream_t q) {             \
        hipLaunchKernelGGL((k_reduce_multi<float, 0, N, 1, 0, 1, N, D>), dim3(tiles(nv)),  \
                           dim3(kReduceBlock), LDS, q, d, s, 0u, (size_t)0, nv, (size_t)0); \
    }, true, {}})
    OV("uncapped regs, LDS cap 12 waves/CU, 4 ahead", 4, 163840 / 12);
    OV("uncapped regs, LDS cap 13 waves/CU, 4 ahead", 4, 163840 / 13);
    OV("uncapped regs, LDS cap 14 waves/CU, 4 ahead", 4, 163840 / 14);
    OV("uncapped regs, LDS cap 16 waves/CU, 4 ahead", 4, 163840 / 16);
    OV("uncapped regs, LDS cap 20 waves/CU, 4 ahead", 4, 163840 / 20);
#undef OV
    vs.push_back({"product form, in place: dst = operand 0 (unchecked)",
                  [](float *d, SrcList s, size_t nv, hipStream_t q) {
        (void)d;
        hipLaunchKernelGGL((k_reduce_multi<float, 0, N, 1, 1, 1, N, 2>), dim3(tiles(nv)),
                           dim3(kReduceBlock), 0, q, (float*)const_cast<void*>(s.p[0]), s,
                           0u, (size_t)0, nv, (size_t)0);
    }, false, {}});
    vs.push_back({"ceiling: read N operands, store zeros (no dependency)",
                  [](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL((k_read_store0<N>), dim3(tiles(nv)), dim3(kReduceBlock), 0, q, d, s, nv);
    }, false, {}});
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
    TV("product PFO, all operands, 2 tiles ahead", 1, C, 1, NMAX, 2, 1);
    TV("product PFO, all operands, 4 tiles ahead", 1, C, 1, NMAX, 4, 1);
    TV("product PFO, root only, 1 tile ahead", 1, C, 1, 1, 1, 1);
    TV("product PFO, root only, 4 tiles ahead", 1, C, 1, 1, 4, 1);
#undef TV
}

/* Round 6: the tree fan-in built for exactly n operands (NMAX = n: no
 * reloads of the root's operand past n), in the product's n == NMAX form
 * (every operand's line two tiles ahead) and the root-only form */
template <int NX>
static void add_tree_exact(std::vector<Variant> &vs, unsigned n)
{
    vs.push_back({"exact NMAX = n, PF1 all operands, 2 tiles ahead",
                  [n](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL((k_reduce_tree<float, 0, NX, 1, 1, 1, NX, 2>), dim3(tiles(nv)),
                           dim3(kReduceBlock), 0, q, d, s, n, (size_t)0, nv, (size_t)0);
    }, true, {}});
    vs.push_back({"exact NMAX = n, PFO all operands, 2 tiles ahead",
                  [n](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL((k_reduce_tree<float, 0, NX, 1, 1, 1, NX, 2, 1>), dim3(tiles(nv)),
                           dim3(kReduceBlock), 0, q, d, s, n, (size_t)0, nv, (size_t)0);
    }, true, {}});
    vs.push_back({"exact NMAX = n, PFO all operands, 4 tiles ahead",
                  [n](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL((k_reduce_tree<float, 0, NX, 1, 1, 1, NX, 4, 1>), dim3(tiles(nv)),
                           dim3(kReduceBlock), 0, q, d, s, n, (size_t)0, nv, (size_t)0);
    }, true, {}});
    vs.push_back({"exact NMAX = n, PF1 root only, 1 tile ahead",
                  [n](float *d, SrcList s, size_t nv, hipStream_t q) {
        hipLaunchKernelGGL((k_reduce_tree<float, 0, NX, 1, 1, 1, 1, 1>), dim3(tiles(nv)),
                           dim3(kReduceBlock), 0, q, d, s, n, (size_t)0, nv, (size_t)0);
    }, true, {}});
}

int main(int argc, char **argv)
{
    if (argc < 3 || (strcmp(argv[1], "multi") && strcmp(argv[1], "tree"))) {
        fprintf(stderr, "usage: tune_multi_pf multi|tree N [lg=24] [rounds=5] [stagger=0] "
                "[separate=0]\n");
        return 2;
    }
    const bool tree  = !strcmp(argv[1], "tree");
    const unsigned N = (unsigned)atoi(argv[2]);
    const int lg     = argc > 3 ? atoi(argv[3]) : 24;
    const int rounds = argc > 4 ? atoi(argv[4]) : 5;
    /* operand m starts m * stagger bytes past m * S (a multiple of 256 B):
     * do operands a power of two apart meet in the same HBM channels? */
    const size_t stagger = argc > 5 ? (size_t)atol(argv[5]) & ~(size_t)255 : 0;
    /* layout 1: every operand and the output in an allocation of its own (as
     * N ranks' buffers are), instead of one arena S + stagger apart */
    const int separate   = argc > 6 ? atoi(argv[6]) : 0;
    /* optional: only the variants whose names contain one of these
     * ','-separated substrings (the reference variant and ceilings always) */
    const std::string only = argc > 7 ? argv[7] : "";
    const int iters  = 10;
    if ((!tree && (N != 2 && N != 4 && N != 8 && N != 16)) || (tree && (N < 2 || N > 16))) {
        fprintf(stderr, "N: multi 2/4/8/16, tree 2..16\n");
        return 2;
    }
    const size_t n = (size_t)1 << lg, nvec = n / 4, S = n * 4;
    char *arena = nullptr, *own[kMaxMulti + 2] = {};
    const size_t slot = S + stagger;
    if (!separate) {
        CHECK(hipMalloc(&arena, (N + 2) * slot));
    } else {
        for (unsigned m = 0; m < N + 2; m++) {
            CHECK(hipMalloc(&own[m], S));
        }
    }
    auto at = [&](unsigned m) { return separate ? own[m] : arena + m * slot; };
    SrcList srcs;
    for (unsigned m = 0; m < (unsigned)kMaxMulti; m++) {
        srcs.p[m] = m < N ? at(m) : nullptr;
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
    float *out = reinterpret_cast<float*>(at(N));
    float *ref = reinterpret_cast<float*>(at(N + 1));
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
    if (tree) {
        switch (N) {
        case 3:  add_tree_exact<3>(vs, N); break;
        case 6:  add_tree_exact<6>(vs, N); break;
        case 12: add_tree_exact<12>(vs, N); break;
        case 5:  add_tree_exact<5>(vs, N); break;
        case 10: add_tree_exact<10>(vs, N); break;
        case 15: add_tree_exact<15>(vs, N); break;
        default: break;
        }
    }

    if (!only.empty()) {
        std::vector<Variant> keep;
        for (size_t k = 0; k < vs.size(); k++) {
            bool hit = k == 0 || vs[k].name.rfind("ceiling", 0) == 0;
            size_t a = 0;
            while (!hit && a <= only.size()) {
                const size_t e = std::min(only.find(',', a), only.size());
                const std::string w = only.substr(a, e - a);
                hit = !w.empty() && vs[k].name.find(w) != std::string::npos;
                a = e + 1;
            }
            if (hit) {
                keep.push_back(vs[k]);
            }
        }
        vs.swap(keep);
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
           "%s, stagger %zu B\n", tree ? "tree n =" : "multi N =", N, S >> 20,
           bytes / 1048576.0, rounds, iters,
           separate ? "separate allocations" : "one arena", stagger);
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2];
        const double b = v.name.rfind("ceiling: read the N operands, no store", 0) == 0 ?
                         bytes * N / (N + 1) : bytes;
        printf("%-52s median %8.2f us  min %8.2f  %7.1f GB/s  %5.1f%% of 8 TB/s\n",
               v.name.c_str(), med * 1e3, v.ms.front() * 1e3, b / (med * 1e-3) / 1e9,
               100.0 * b / (med * 1e-3) / 8e12);
    }
    return 0;
}
