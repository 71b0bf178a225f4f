/*
 * dev_kernels.h - CDNA4 (gfx950) kernels for the UCG combine path.
 *
 *   k_reduce        dst = src (op) dst, 16-B non-temporal vector loads of
 *                   both operands, one tile of U vectors per lane, grid
 *                   sized to the data; the unaligned head and the ragged
 *                   tail (< 16 B each) are done by the first lanes of the
 *                   grid with lane-masked scalar accesses.
 *   k_reduce_shift  same contract when src and dst disagree mod 16 B:
 *                   aligned src loads realigned by a wavefront shuffle.
 *   k_reduce_scalar element-wise fallback for operands that are not even
 *                   element-aligned.
 *   k_reduce_multi  one-shot N-operand combine in the recursive-doubling
 *                   association (builtin/plan/builtin_recursive.c:158-169).
 *   k_fill          counter-based synthetic generator.
 *
 * Element-wise, HBM-bound: 3 x N x sizeof(T) algorithmic bytes per combine,
 * no reuse, so no LDS staging and no MFMA; the levers are 16-B accesses,
 * enough bytes in flight per CU and launch geometry.
 */
#ifndef UCG_DEV_KERNELS_H_
#define UCG_DEV_KERNELS_H_

#include "combine_ops.h"

namespace ucgdev {

constexpr int kBlock = 256;           /* 4 waves of 64 lanes */
constexpr int kMaxMulti = 16;         /* max operands of k_reduce_multi */
/* streaming-kernel geometry, measured on MI355X (profiles/r01/tune_*.txt):
 * one wave per workgroup and one 16-B vector per lane per operand reached
 * 85.5% of 8 TB/s on the 1 GiB fp32 combine, vs 80% for 256-lane groups
 * with 4 vectors per lane and 55% for a grid-stride loop */
constexpr int kReduceBlock = 64;      /* lanes per workgroup: one wave */
constexpr int kReduceU     = 1;       /* 16-B vectors per lane per operand */
constexpr int kMultiU      = 1;       /* same for k_reduce_multi */

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

/* Occupancy cap of the multi-operand kernels. With every CU full of one-wave
 * workgroups, each holding one 16-B load of every operand, HBM serves
 * (operands + 1) streams from up to 32 waves per CU and loses 3-5 points to
 * it; at most 12 waves per CU gains them back (tools/tune_cap,
 * profiles/r04/r04b: fp32 SUM, 64 MiB per operand, N = 4 / 8 / 16 at
 * 76.8 / 78.7 / 75.2 % of 8 TB/s uncapped, 80.2 / 81.6 / 76.8 % capped). The
 * cap is the kernel's register allocation: a clobbered v167 makes it hold 168
 * VGPRs, so floor(512 / 168) = 3 waves fit a SIMD, 12 a CU. No LDS is
 * allocated (round 3's cap was unused dynamic LDS: ADVICE r03). */
#define UCG_MULTI_CAP_CLOBBER() asm volatile("" ::: "v167")

template <int NT>
__device__ __forceinline__ u32x4 ld16(const u32x4 *p)
{
    if (NT) {
        return __builtin_nontemporal_load(p);
    }
    return *p;
}

template <int NT>
__device__ __forceinline__ void st16(u32x4 *p, u32x4 v)
{
    if (NT) {
        __builtin_nontemporal_store(v, p);
    } else {
        *p = v;
    }
}

/* apply the functor to the 16/sizeof(T) lanes of a 16-B vector */
template <typename T, int OP>
__device__ __forceinline__ u32x4 vapply(u32x4 s, u32x4 d)
{
    constexpr int V = 16 / sizeof(T);
    T a[V], b[V];
    __builtin_memcpy(a, &s, 16);
    __builtin_memcpy(b, &d, 16);
#pragma unroll
    for (int k = 0; k < V; k++) {
        b[k] = Comb<T, OP>::apply(a[k], b[k]);
    }
    u32x4 o;
    __builtin_memcpy(&o, b, 16);
    return o;
}

/* XCD-aware tile map for the realigning kernels. A wave of those reads one
 * line past its own tile (the next tile's first src vector). The dispatcher
 * deals workgroup b to XCD b % 8 (MI355X_MICROARCH.md, dispatch placement),
 * so with the identity map that line is the next workgroup's, on another
 * XCD, and is fetched into two L2s: PMC shows 1/16 more FETCH_SIZE than the
 * aligned kernel, and the kernel ran 4 points slower. Here XCD x takes chunks
 * of kXcdChunk consecutive tiles, so the neighbouring tile is processed on
 * the same XCD one workgroup earlier or later and the line is an L2 hit -
 * provided that extra load is temporal: issued non-temporally it still
 * fetched 1.04-1.12 x the algorithmic bytes (round 4, profiles/r04/r04k).
 * A bijection on [0, ntiles): whole rounds of 8 are remapped, a ragged last
 * round keeps the identity. */
constexpr unsigned kXcdChunk = 64;

template <unsigned C>
__device__ __forceinline__ unsigned xcd_tile(unsigned b, unsigned ntiles)
{
    const unsigned full = ntiles & ~7u;
    if (b >= full) {
        return b;
    }
    const unsigned T8 = full >> 3, x = b & 7, j = b >> 3;
    const unsigned R = T8 / C, r = T8 % C;   /* whole chunk rows, remainder */
    return (j < R * C) ? (j / C) * (8u * C) + x * C + (j % C)
                       : R * 8u * C + x * r + (j - R * C);
}

/*
 * The streaming combine. One tile of U 16-B vectors per lane (lane stride
 * BS), no loop: the grid is sized to the data (one dispatch covers up to 2^31
 * vectors, see launch_vec), so the hardware dispatcher streams fresh
 * workgroups onto the CUs and every wave issues its 2U loads back to back
 * before its first use. Loads and stores carry the non-temporal hint: nothing
 * is re-read. Measured on MI355X this geometry moved the 2 x 256 MiB fp32
 * combine from 56% (grid-stride loop, temporal) to 85% of 8 TB/s with
 * one-wave workgroups and U = 1 (profiles/r01). The ragged head
 * (until dst is 16-B aligned) and tail (< 16 B) are done by the first lanes.
 *
 * PF > 0 (the product's form since round 4; U = 1, one wave per workgroup):
 * the XCD-aware tile map, and the last PF lanes also load the first PF lines
 * of the next tile's src with temporal loads and discard them (PF = 1: lane
 * 63's vector, as the realigning kernel's `ex`). The next tile runs on the
 * same XCD, so those lines are fetched once and wait in L2 for their own
 * wave. The realigning kernel had run 2 points above the plain one on six
 * boxes; this form matched it, against neither the map nor the load alone
 * (tools/tune_misalign, profiles/r04/r04q-r04v). Loads are
 * clamped and unmasked behind a sched barrier, as in k_reduce_shift. ORD
 * fixes the order the three loads issue in (the product's kLoadOrder = 2:
 * those lines first, then src, then dst; round 6, tools/tune_order). XC is
 * the XCD map's chunk of tiles (kXcdChunk, or launch_vec's kReduceChunkSmall
 * below 1 GiB per operand).
 */
template <typename T, int OP, int U, int NT, int BS, int XM = 0, int PF = 0, int ORD = 0,
          unsigned XC = kXcdChunk>
__global__ void __launch_bounds__(BS)
k_reduce(T *dst, const T *src, size_t head, size_t nvec, size_t tail)
{
    constexpr int V   = 16 / sizeof(T);
    const size_t gtid = (size_t)blockIdx.x * BS + threadIdx.x;

    /* ragged edges: < V elements each, one lane per element */
    if (gtid < head) {
        dst[gtid] = Comb<T, OP>::apply(src[gtid], dst[gtid]);
    }
    if (gtid < tail) {
        const size_t j = head + nvec * V + gtid;
        dst[j] = Comb<T, OP>::apply(src[j], dst[j]);
    }

    const u32x4 *s4   = reinterpret_cast<const u32x4*>(src + head);
    u32x4 *d4         = reinterpret_cast<u32x4*>(dst + head);
    if constexpr (PF) {
        static_assert(U == 1 && BS == 64 && PF <= 8,
                      "one vector per lane, one wave per workgroup, at most a tile ahead");
        if (nvec == 0) {
            return;
        }
        const size_t i  = (size_t)xcd_tile<XC>(blockIdx.x, gridDim.x) * BS + threadIdx.x;
        const size_t ic = i < nvec ? i : nvec - 1;
        /* the last PF lanes take one 128-B line (8 vectors) each of the next
         * tile's src, lane 63 its first; every other lane reloads the last
         * vector (one line, an L2 hit), so the load needs no branch */
        const unsigned k = BS - 1 - threadIdx.x;
        const size_t want = (i - threadIdx.x + BS) + (size_t)k * 8;
        const u32x4 *at   = s4 + (k < (unsigned)PF && want < nvec ? want : nvec - 1);
        u32x4 a, b, pf;
        if constexpr (ORD == 0) {           /* the compiler's order */
            a  = ld16<NT>(s4 + ic);
            b  = ld16<NT>(d4 + ic);
            pf = ld16<0>(at);
        } else if constexpr (ORD == 1) {    /* src, the prefetch, dst */
            a  = ld16<NT>(s4 + ic);
            __builtin_amdgcn_sched_barrier(0);
            pf = ld16<0>(at);
            __builtin_amdgcn_sched_barrier(0);
            b  = ld16<NT>(d4 + ic);
        } else if constexpr (ORD == 2) {    /* the prefetch, src, dst */
            pf = ld16<0>(at);
            __builtin_amdgcn_sched_barrier(0);
            a  = ld16<NT>(s4 + ic);
            __builtin_amdgcn_sched_barrier(0);
            b  = ld16<NT>(d4 + ic);
        } else {                            /* src, dst, the prefetch */
            a  = ld16<NT>(s4 + ic);
            __builtin_amdgcn_sched_barrier(0);
            b  = ld16<NT>(d4 + ic);
            __builtin_amdgcn_sched_barrier(0);
            pf = ld16<0>(at);
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("" :: "v"(pf[0]));     /* the load stays; its value is unused */
        if (i < nvec) {
            st16<NT>(d4 + i, vapply<T, OP>(a, b));
        }
        return;
    }
    /* XM: the XCD-aware tile map, for a src whose vectors straddle 128-B
     * lines (its edge lines are then shared with the neighbouring tiles) */
    const size_t tile = XM ? xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) : blockIdx.x;
    const size_t base = tile * (BS * U) + threadIdx.x;
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * BS;
        if (i < nvec) {
            a[u] = ld16<NT>(s4 + i);
            b[u] = ld16<NT>(d4 + i);
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * BS;
        if (i < nvec) {
            st16<NT>(d4 + i, vapply<T, OP>(a[u], b[u]));
        }
    }
}

/*
 * The streaming combine when src and dst disagree mod 16 B (a fragment landing
 * at an arbitrary remote_offset, a peer's buffer at another offset). After the
 * head, dst is 16-B aligned and src sits r = 4Q + rb bytes past a 16-B
 * boundary A. Lane L loads the aligned src vector A[i] (i = its dst vector);
 * the vector after it, A[i+1], is lane L+1's load, fetched with a wavefront
 * shuffle (ds_bpermute), and lane 63 loads it itself. The src bytes under
 * dst vector i are then funnel-shifted out of the 32-B pair (v_alignbyte).
 * Every src vector is loaded once (lane 63's extra load aside), so the HBM
 * traffic is the aligned kernel's. The aligned vectors A[0] and A[nvec] each
 * hold bytes of the operand, so they lie in its pages even where they reach
 * past its ends.
 */
/* lane L gets lane L+1's value (lane 63: undefined, overwritten by the
 * caller), through ds_bpermute (the LDS crossbar; no LDS allocated) */
__device__ __forceinline__ uint32_t from_next_lane(uint32_t x)
{
    return __shfl_down(x, 1, 64);
}

template <typename T, int OP, int Q, int PF = 1>
__global__ void __launch_bounds__(kReduceBlock)
k_reduce_shift(T *dst, const T *src, size_t head, size_t nvec, size_t tail,
               unsigned rb)
{
    static_assert(PF >= 1 && PF <= 8, "lane 63's load is the next tile's first vector");
    constexpr int V   = 16 / sizeof(T);
    constexpr int BS  = kReduceBlock;
    const size_t gtid = (size_t)blockIdx.x * BS + threadIdx.x;

    if (gtid < head) {
        dst[gtid] = Comb<T, OP>::apply(src[gtid], dst[gtid]);
    }
    if (gtid < tail) {
        const size_t j = head + nvec * V + gtid;
        dst[j] = Comb<T, OP>::apply(src[j], dst[j]);
    }
    if (nvec == 0) {
        return;
    }

    const char *sp  = reinterpret_cast<const char*>(src + head);
    const u32x4 *a4 = reinterpret_cast<const u32x4*>(sp - (4 * Q + rb));
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst + head);
    /* the wave's tile: 64 vectors; lane L holds column L */
    const size_t i       = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * BS +
                           threadIdx.x;
    const bool last_lane = threadIdx.x == BS - 1;
    /* every load in flight before the first wait; lanes past the end load
     * the last vector again (unmasked loads keep the compiler from
     * serialising them) and store nothing */
    const u32x4 b  = ld16<1>(d4 + (i < nvec ? i : nvec - 1));
    const u32x4 lo = ld16<1>(a4 + (i < nvec ? i : nvec));
    /* temporal: that vector is the next tile's first, which its own wave
     * loads non-temporally; a non-temporal load here could evict the line
     * before the neighbour's load and fetch it from HBM twice.
     * Lanes 63 - 1 .. 63 - (PF - 1) load the next tile's following lines in
     * the same instruction and discard them (k_reduce's PF form); lane 63's
     * is A[i + 1] itself. A[nvec] holds src bytes (rb or Q > 0). */
    const unsigned k  = BS - 1 - threadIdx.x;
    const size_t want = (i - threadIdx.x + BS) + (size_t)k * 8;
    const u32x4 ex = ld16<0>(a4 + (k < (unsigned)PF && want <= nvec ? want : nvec));
    __builtin_amdgcn_sched_barrier(0);  /* keep the shuffles behind all loads */
    /* A[i + 1]: the next lane's load; lane 63 loaded it itself */
    u32x4 hi;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        hi[k] = from_next_lane(lo[k]);
    }
    if (last_lane) {
        hi = ex;
    }
    if (i < nvec) {
        const uint32_t w[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        u32x4 sv;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            sv[k] = __builtin_amdgcn_alignbyte(w[Q + k + 1], w[Q + k], rb);
        }
        st16<1>(d4 + i, vapply<T, OP>(sv, b));
    }
}

template <typename T, int OP>
__global__ void __launch_bounds__(kBlock)
k_reduce_scalar(T *dst, const T *src, size_t count)
{
    constexpr int U   = 4;
    const size_t nthr = (size_t)gridDim.x * kBlock;
    size_t i          = (size_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + (U - 1) * nthr < count; i += U * nthr) {
        T a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            a[u] = src[i + u * nthr];
            b[u] = dst[i + u * nthr];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            dst[i + u * nthr] = Comb<T, OP>::apply(a[u], b[u]);
        }
    }
    for (; i < count; i += nthr) {
        dst[i] = Comb<T, OP>::apply(src[i], dst[i]);
    }
}

/* ---- recursive-doubling association ------------------------------------ */
struct SrcList {
    const void *p[kMaxMulti];
};

/* val[m] holds member (self ^ m). Level j (h = 2^(j-1)) computes, for every m
 * with its low j bits clear, V(self^m, j) = V(self^m^h, j-1) (op) V(self^m,
 * j-1): the incoming (src) operand is the partner's accumulator. */
template <int N, typename E, typename F>
__device__ __forceinline__ E rd_tree(E (&val)[N], F f)
{
#pragma unroll
    for (int h = 1; h < N; h <<= 1) {
#pragma unroll
        for (int m = 0; m < N; m += 2 * h) {
            val[m] = f(val[m + h], val[m]);
        }
    }
    return val[0];
}

/* The next-tile prefetch of k_reduce's PF form, for the in-phase multi-operand
 * kernels (k_reduce_multi, k_reduce_tree): with the XCD-aware tile map, the
 * last PF lanes of a wave load the first PF 128-B lines of the tile D tiles
 * ahead of each of the operands `ops[0 .. PFM)` with temporal loads and
 * discard them;
 * every other lane reloads the operand's last vector (one line, an L2 hit),
 * so no branch separates the loads. The loads are issued with the tile's own
 * and kept alive by an empty asm after the sched barrier. */
template <int PF, int PFM, int D>
__device__ __forceinline__ void next_tile_lines(const u32x4 *const (&ops)[PFM > 0 ? PFM : 1],
                                                size_t i, size_t nvec)
{
    if constexpr (PF > 0 && PFM > 0) {
        const unsigned k  = kReduceBlock - 1 - threadIdx.x;
        const size_t want = (i - threadIdx.x + (size_t)D * kReduceBlock) + (size_t)k * 8;
        const size_t at   = (k < (unsigned)PF && want < nvec) ? want : nvec - 1;
        u32x4 pf[PFM];
#pragma unroll
        for (int m = 0; m < PFM; m++) {
            pf[m] = ld16<0>(ops[m] + at);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < PFM; m++) {
            asm volatile("" :: "v"(pf[m][0]));    /* the load stays; its value is unused */
        }
    } else {
        (void)ops; (void)i; (void)nvec;
    }
}

/* The same lines issued BEFORE the tile's own loads (PFO = 1 in the
 * multi-operand kernels): tile_lines_issue, a sched barrier, the operand
 * loads, then tile_lines_keep. Issued first, the lines are in flight while
 * the wave waits for its operands (the 2-operand combine's ORD 2). */
template <int PF, int PFM, int D>
__device__ __forceinline__ void tile_lines_issue(const u32x4 *const (&ops)[PFM > 0 ? PFM : 1],
                                                 size_t i, size_t nvec,
                                                 u32x4 (&pf)[PFM > 0 ? PFM : 1])
{
    const unsigned k  = kReduceBlock - 1 - threadIdx.x;
    const size_t want = (i - threadIdx.x + (size_t)D * kReduceBlock) + (size_t)k * 8;
    const size_t at   = (k < (unsigned)PF && want < nvec) ? want : nvec - 1;
#pragma unroll
    for (int m = 0; m < PFM; m++) {
        pf[m] = ld16<0>(ops[m] + at);
    }
    __builtin_amdgcn_sched_barrier(0);
}

template <int PFM>
__device__ __forceinline__ void tile_lines_keep(const u32x4 (&pf)[PFM > 0 ? PFM : 1])
{
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < PFM; m++) {
        asm volatile("" :: "v"(pf[m][0]));    /* the load stays; its value is unused */
    }
}

template <typename T, int OP, int N, int XM = 0, int CAP = 0, int PF = 0, int PFM = 0,
          int PFD = 1, int PFO = 0>
__global__ void __launch_bounds__(kReduceBlock)
k_reduce_multi(T *dst, SrcList srcs, unsigned self, size_t head, size_t nvec,
               size_t tail)
{
    if constexpr (CAP) {
        UCG_MULTI_CAP_CLOBBER();
    }
    constexpr int V    = 16 / sizeof(T);
    const size_t gtid  = (size_t)blockIdx.x * kReduceBlock + threadIdx.x;
    auto fs = [](T a, T b) { return Comb<T, OP>::apply(a, b); };
    auto fv = [](u32x4 a, u32x4 b) { return vapply<T, OP>(a, b); };

    if (gtid < head || gtid < tail) {
#pragma unroll
        for (int part = 0; part < 2; part++) {
            size_t j;
            if (part == 0) {
                if (gtid >= head) continue;
                j = gtid;
            } else {
                if (gtid >= tail) continue;
                j = head + nvec * V + gtid;
            }
            T val[N];
#pragma unroll
            for (int m = 0; m < N; m++) {
                val[m] = static_cast<const T*>(srcs.p[self ^ m])[j];
            }
            dst[j] = rd_tree<N>(val, fs);
        }
    }

    u32x4 *d4 = reinterpret_cast<u32x4*>(dst + head);
    if constexpr (PF > 0) {
        /* PF form: always on the XCD tile map, loads clamped and unmasked
         * (one tile of one vector per lane, kMultiU == 1) */
        static_assert(kMultiU == 1 && PFM <= N, "one vector per lane; prefetch operands <= N");
        if (nvec == 0) {
            return;
        }
        const size_t i  = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * kReduceBlock +
                          threadIdx.x;
        const size_t ic = i < nvec ? i : nvec - 1;
        const u32x4 *op[N];
        u32x4 val[N];
        if constexpr (PFO) {
            /* the next tiles' lines first (tile_lines_issue) */
            const u32x4 *pops[PFM > 0 ? PFM : 1];
            u32x4 pf[PFM > 0 ? PFM : 1];
#pragma unroll
            for (int m = 0; m < N; m++) {
                op[m] = reinterpret_cast<const u32x4*>(static_cast<const T*>(srcs.p[self ^ m]) +
                                                       head);
            }
#pragma unroll
            for (int m = 0; m < (PFM > 0 ? PFM : 1); m++) {
                pops[m] = op[m];
            }
            tile_lines_issue<PF, PFM, PFD>(pops, i, nvec, pf);
#pragma unroll
            for (int m = 0; m < N; m++) {
                val[m] = ld16<1>(op[m] + ic);
            }
            tile_lines_keep<PFM>(pf);
        } else {
#pragma unroll
            for (int m = 0; m < N; m++) {
                op[m]  = reinterpret_cast<const u32x4*>(static_cast<const T*>(srcs.p[self ^ m]) +
                                                        head);
                val[m] = ld16<1>(op[m] + ic);
            }
            const u32x4 *pops[PFM > 0 ? PFM : 1];
#pragma unroll
            for (int m = 0; m < (PFM > 0 ? PFM : 1); m++) {
                pops[m] = op[m];
            }
            next_tile_lines<PF, PFM, PFD>(pops, i, nvec);
        }
        if (i < nvec) {
            st16<1>(d4 + i, rd_tree<N>(val, fv));
        }
        return;
    }
    const size_t tile = XM ? xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) : blockIdx.x;
    const size_t base = tile * (kReduceBlock * kMultiU) + threadIdx.x;
#pragma unroll
    for (int u = 0; u < kMultiU; u++) {
        const size_t i = base + (size_t)u * kReduceBlock;
        if (i < nvec) {
            u32x4 val[N];
#pragma unroll
            for (int m = 0; m < N; m++) {
                val[m] = ld16<1>(reinterpret_cast<const u32x4*>(
                             static_cast<const T*>(srcs.p[self ^ m]) + head) + i);
            }
            st16<1>(d4 + i, rd_tree<N>(val, fv));
        }
    }
}

/* bytes [r, r + 16) of the 32-B pair (lo, hi); r uniform, 0..15 */
__device__ __forceinline__ u32x4 funnel16(u32x4 lo, u32x4 hi, unsigned r)
{
    const unsigned rb = r & 3;
    uint32_t w[5];
    switch (r >> 2) {
    case 0:  w[0] = lo[0]; w[1] = lo[1]; w[2] = lo[2]; w[3] = lo[3]; w[4] = hi[0]; break;
    case 1:  w[0] = lo[1]; w[1] = lo[2]; w[2] = lo[3]; w[3] = hi[0]; w[4] = hi[1]; break;
    case 2:  w[0] = lo[2]; w[1] = lo[3]; w[2] = hi[0]; w[3] = hi[1]; w[4] = hi[2]; break;
    default: w[0] = lo[3]; w[1] = hi[0]; w[2] = hi[1]; w[3] = hi[2]; w[4] = hi[3]; break;
    }
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        o[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], rb);
    }
    return o;
}

/*
 * k_reduce_multi when some operand disagrees with dst mod 16 B (a peer's
 * buffer at another offset). Every operand is read in aligned 16-B vectors
 * and realigned as in k_reduce_shift, each with its own phase (computed from
 * its pointer: uniform per operand); an operand in phase with dst takes the
 * plain path. All loads are issued before the first shuffle. Same
 * association as k_reduce_multi, so the same bits.
 */
template <typename T, int OP, int N, int CAP = 0>
__global__ void __launch_bounds__(kReduceBlock)
k_reduce_multi_shift(T *dst, SrcList srcs, unsigned self, size_t head, size_t nvec,
                     size_t tail)
{
    if constexpr (CAP) {
        UCG_MULTI_CAP_CLOBBER();
    }
    constexpr int V    = 16 / sizeof(T);
    const size_t gtid  = (size_t)blockIdx.x * kReduceBlock + threadIdx.x;
    auto fs = [](T a, T b) { return Comb<T, OP>::apply(a, b); };
    auto fv = [](u32x4 a, u32x4 b) { return vapply<T, OP>(a, b); };

    if (gtid < head || gtid < tail) {
#pragma unroll
        for (int part = 0; part < 2; part++) {
            size_t j;
            if (part == 0) {
                if (gtid >= head) continue;
                j = gtid;
            } else {
                if (gtid >= tail) continue;
                j = head + nvec * V + gtid;
            }
            T val[N];
#pragma unroll
            for (int m = 0; m < N; m++) {
                val[m] = static_cast<const T*>(srcs.p[self ^ m])[j];
            }
            dst[j] = rd_tree<N>(val, fs);
        }
    }
    if (nvec == 0) {
        return;
    }

    u32x4 *d4            = reinterpret_cast<u32x4*>(dst + head);
    const size_t i       = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * kReduceBlock +
                           threadIdx.x;
    const bool last_lane = threadIdx.x == kReduceBlock - 1;
    const u32x4 *a4[N];
    unsigned r[N];
    u32x4 val[N], ex[N];
#pragma unroll
    for (int m = 0; m < N; m++) {
        const char *p = reinterpret_cast<const char*>(
            static_cast<const T*>(srcs.p[self ^ m]) + head);
        r[m]  = (unsigned)((uintptr_t)p & 15);
        a4[m] = reinterpret_cast<const u32x4*>(p - r[m]);
        /* clamped, unmasked loads with no branch between them (see
         * k_reduce_shift); an out-of-phase operand also needs A[nvec] */
        const size_t lim = nvec - (r[m] == 0);
        val[m] = ld16<1>(a4[m] + (i < lim ? i : lim));
        ex[m]  = ld16<0>(a4[m] + (last_lane && i < lim ? i + 1 : lim));   /* temporal */
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < N; m++) {
        if (r[m]) {
            u32x4 hi;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                hi[k] = from_next_lane(val[m][k]);
            }
            if (last_lane) {
                hi = ex[m];
            }
            val[m] = funnel16(val[m], hi, r[m]);
        }
    }
    if (i < nvec) {
        st16<1>(d4 + i, rd_tree<N>(val, fv));
    }
}

/*
 * One-shot tree fan-in: the association of the reference's tree plan at its
 * root (builtin/plan/builtin_tree.c:262-380 on one host; the root's
 * recv.buffer starts as its own send buffer, builtin_control.c:43-47, and
 * every child's message is reduced into it as it arrives, dst = child (op)
 * dst, builtin_comp_step.inl:213-221): acc = srcs[0]; acc = srcs[m] (op) acc
 * for m = 1 .. n-1, srcs[0] being the root and the rest the children in
 * arrival order. Any n <= NMAX (the plan for groups that are not a power of
 * two, and for MPI_Reduce). Operands past n load srcs[0] again (an L2 hit,
 * no branch between the loads) and are not combined.
 */
template <typename T, int OP, int NMAX, int XM = 0, int CAP = 0, int PF = 0, int PFM = 0,
          int PFD = 1, int PFO = 0>
__global__ void __launch_bounds__(kReduceBlock)
k_reduce_tree(T *dst, SrcList srcs, unsigned n, size_t head, size_t nvec, size_t tail)
{
    if constexpr (CAP) {
        UCG_MULTI_CAP_CLOBBER();
    }
    constexpr int V    = 16 / sizeof(T);
    const size_t gtid  = (size_t)blockIdx.x * kReduceBlock + threadIdx.x;

    if (gtid < head || gtid < tail) {
#pragma unroll
        for (int part = 0; part < 2; part++) {
            size_t j;
            if (part == 0) {
                if (gtid >= head) continue;
                j = gtid;
            } else {
                if (gtid >= tail) continue;
                j = head + nvec * V + gtid;
            }
            T acc = static_cast<const T*>(srcs.p[0])[j];
            for (unsigned m = 1; m < n; m++) {
                acc = Comb<T, OP>::apply(static_cast<const T*>(srcs.p[m])[j], acc);
            }
            dst[j] = acc;
        }
    }

    if constexpr (PF > 0) {
        /* PF form (see k_reduce_multi): XCD tile map, clamped unmasked loads,
         * the first PFM operands' next-tile lines loaded ahead */
        static_assert(PFM <= NMAX, "prefetch operands <= NMAX");
        if (nvec == 0) {
            return;
        }
        const size_t i  = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * kReduceBlock +
                          threadIdx.x;
        const size_t ic = i < nvec ? i : nvec - 1;
        const u32x4 *op[NMAX];
        u32x4 val[NMAX];
        if constexpr (PFO) {
            /* the next tiles' lines first (tile_lines_issue) */
            const u32x4 *pops[PFM > 0 ? PFM : 1];
            u32x4 pf[PFM > 0 ? PFM : 1];
#pragma unroll
            for (int m = 0; m < NMAX; m++) {
                op[m] = reinterpret_cast<const u32x4*>(
                    static_cast<const T*>(srcs.p[(unsigned)m < n ? m : 0]) + head);
            }
#pragma unroll
            for (int m = 0; m < (PFM > 0 ? PFM : 1); m++) {
                pops[m] = op[m];
            }
            tile_lines_issue<PF, PFM, PFD>(pops, i, nvec, pf);
#pragma unroll
            for (int m = 0; m < NMAX; m++) {
                val[m] = ld16<1>(op[m] + ic);
            }
            tile_lines_keep<PFM>(pf);
        } else {
#pragma unroll
            for (int m = 0; m < NMAX; m++) {
                op[m]  = reinterpret_cast<const u32x4*>(
                    static_cast<const T*>(srcs.p[(unsigned)m < n ? m : 0]) + head);
                val[m] = ld16<1>(op[m] + ic);
            }
            const u32x4 *pops[PFM > 0 ? PFM : 1];
#pragma unroll
            for (int m = 0; m < (PFM > 0 ? PFM : 1); m++) {
                pops[m] = op[m];
            }
            next_tile_lines<PF, PFM, PFD>(pops, i, nvec);
        }
        if (i < nvec) {
            u32x4 acc = val[0];
#pragma unroll
            for (int m = 1; m < NMAX; m++) {
                if ((unsigned)m < n) {
                    acc = vapply<T, OP>(val[m], acc);
                }
            }
            st16<1>(reinterpret_cast<u32x4*>(dst + head) + i, acc);
        }
        return;
    }

    const size_t i = (XM ? xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) : blockIdx.x) *
                         kReduceBlock + threadIdx.x;
    if (i < nvec) {
        u32x4 val[NMAX];
#pragma unroll
        for (int m = 0; m < NMAX; m++) {
            const void *p = srcs.p[(unsigned)m < n ? m : 0];
            val[m] = ld16<1>(reinterpret_cast<const u32x4*>(static_cast<const T*>(p) + head) + i);
        }
        u32x4 acc = val[0];
#pragma unroll
        for (int m = 1; m < NMAX; m++) {
            if ((unsigned)m < n) {
                acc = vapply<T, OP>(val[m], acc);
            }
        }
        st16<1>(reinterpret_cast<u32x4*>(dst + head) + i, acc);
    }
}

/*
 * k_reduce_tree when some operand disagrees with dst mod 16 B (a child's
 * fragment or buffer at another offset). Operands are read in aligned 16-B
 * vectors and realigned in registers as in k_reduce_multi_shift, each with
 * its own uniform phase, on the same XCD-aware tile map; the association is
 * k_reduce_tree's (acc = srcs[m] (op) acc, m = 1 .. n-1), so the same bits.
 * Operands past n load srcs[0] again and are not combined.
 */
template <typename T, int OP, int NMAX, int CAP = 0>
__global__ void __launch_bounds__(kReduceBlock)
k_reduce_tree_shift(T *dst, SrcList srcs, unsigned n, size_t head, size_t nvec, size_t tail)
{
    if constexpr (CAP) {
        UCG_MULTI_CAP_CLOBBER();
    }
    constexpr int V   = 16 / sizeof(T);
    const size_t gtid = (size_t)blockIdx.x * kReduceBlock + threadIdx.x;

    if (gtid < head || gtid < tail) {
#pragma unroll
        for (int part = 0; part < 2; part++) {
            size_t j;
            if (part == 0) {
                if (gtid >= head) continue;
                j = gtid;
            } else {
                if (gtid >= tail) continue;
                j = head + nvec * V + gtid;
            }
            T acc = static_cast<const T*>(srcs.p[0])[j];
            for (unsigned m = 1; m < n; m++) {
                acc = Comb<T, OP>::apply(static_cast<const T*>(srcs.p[m])[j], acc);
            }
            dst[j] = acc;
        }
    }
    if (nvec == 0) {
        return;
    }

    u32x4 *d4            = reinterpret_cast<u32x4*>(dst + head);
    const size_t i       = (size_t)xcd_tile<kXcdChunk>(blockIdx.x, gridDim.x) * kReduceBlock +
                           threadIdx.x;
    const bool last_lane = threadIdx.x == kReduceBlock - 1;
    const u32x4 *a4[NMAX];
    unsigned r[NMAX];
    u32x4 val[NMAX], ex[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        const char *p = reinterpret_cast<const char*>(
            static_cast<const T*>(srcs.p[(unsigned)m < n ? m : 0]) + head);
        r[m]  = (unsigned)((uintptr_t)p & 15);
        a4[m] = reinterpret_cast<const u32x4*>(p - r[m]);
        const size_t lim = nvec - (r[m] == 0);
        val[m] = ld16<1>(a4[m] + (i < lim ? i : lim));
        ex[m]  = ld16<0>(a4[m] + (last_lane && i < lim ? i + 1 : lim));   /* temporal */
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < NMAX; m++) {
        if ((unsigned)m < n && r[m]) {
            u32x4 hi;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                hi[k] = from_next_lane(val[m][k]);
            }
            if (last_lane) {
                hi = ex[m];
            }
            val[m] = funnel16(val[m], hi, r[m]);
        }
    }
    if (i < nvec) {
        u32x4 acc = val[0];
#pragma unroll
        for (int m = 1; m < NMAX; m++) {
            if ((unsigned)m < n) {
                acc = vapply<T, OP>(val[m], acc);
            }
        }
        st16<1>(d4 + i, acc);
    }
}

/* ---- synthetic generator (== ucg_oracle_fill) --------------------------- */
__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__constant__ uint32_t c_spec_f32[22] = {
    0x00000000, 0x80000000, 0x3f800000, 0xbf800000, 0x3fc00000, 0x00000001,
    0x007fffff, 0x00800000, 0x7f7fffff, 0xff7fffff, 0x7f800000, 0xff800000,
    0x7fc00000, 0x7fc12345, 0xffc54321, 0x7f800001, 0xff812345, 0x4b800000,
    0x33800000, 0x3dcccccd, 0x80000001, 0x40400000};
__constant__ uint64_t c_spec_f64[22] = {
    0x0000000000000000ull, 0x8000000000000000ull, 0x3ff0000000000000ull,
    0xbff0000000000000ull, 0x3ff8000000000000ull, 0x0000000000000001ull,
    0x000fffffffffffffull, 0x0010000000000000ull, 0x7fefffffffffffffull,
    0xffefffffffffffffull, 0x7ff0000000000000ull, 0xfff0000000000000ull,
    0x7ff8000000000000ull, 0x7ff8000000012345ull, 0xfff8000000054321ull,
    0x7ff0000000000001ull, 0xfff0000000012345ull, 0x4340000000000000ull,
    0x3ca0000000000000ull, 0x3fb999999999999aull, 0x8000000000000001ull,
    0x4008000000000000ull};
__constant__ uint16_t c_spec_f16[22] = {
    0x0000, 0x8000, 0x3c00, 0xbc00, 0x3e00, 0x0001, 0x03ff, 0x0400, 0x7bff,
    0xfbff, 0x7c00, 0xfc00, 0x7e00, 0x7e45, 0xfe21, 0x7c01, 0xfc23, 0x6800,
    0x1000, 0x2e66, 0x8001, 0x4200};
__constant__ uint16_t c_spec_bf16[22] = {
    0x0000, 0x8000, 0x3f80, 0xbf80, 0x3fc0, 0x0001, 0x007f, 0x0080, 0x7f7f,
    0xff7f, 0x7f80, 0xff80, 0x7fc0, 0x7fc5, 0xffc3, 0x7f81, 0xff85, 0x4380,
    0x3b80, 0x3dcd, 0x8001, 0x4040};

__device__ __forceinline__ uint64_t spec_int(unsigned bits, unsigned idx)
{
    const uint64_t m  = (bits == 64) ? ~0ull : ((1ull << bits) - 1);
    const uint64_t mx = m >> 1;
    switch (idx) {
    case 0:  return 0;
    case 1:  return 1;
    case 2:  return m;
    case 3:  return 2;
    case 4:  return mx;
    case 5:  return mx + 1;
    case 6:  return mx - 1;
    case 7:  return mx + 2;
    case 8:  return 0x5555555555555555ull & m;
    case 9:  return 0xaaaaaaaaaaaaaaaaull & m;
    case 10: return 3;
    case 11: return m - 6;
    case 12: return 0x0f0f0f0f0f0f0f0full & m;
    case 13: return 0xf0f0f0f0f0f0f0f0ull & m;
    case 14: return 0x100 & m;
    default: return m - 0xff;
    }
}

template <int DT>
__device__ __forceinline__ uint64_t gen_bits(int dist, uint64_t h)
{
    const uint64_t sign = h >> 63;
    if (dist == UCG_DEV_DIST_SPECIAL) {
        if (DT == UCG_DEV_DT_FLOAT32)  return c_spec_f32[h % 22];
        if (DT == UCG_DEV_DT_FLOAT64)  return c_spec_f64[h % 22];
        if (DT == UCG_DEV_DT_FLOAT16)  return c_spec_f16[h % 22];
        if (DT == UCG_DEV_DT_BFLOAT16) return c_spec_bf16[h % 22];
        return spec_int(8 * sizeof(typename DtType<DT>::T), (unsigned)(h % 16));
    }
    if (dist == UCG_DEV_DIST_EXACT) {
        const int64_t v = (int64_t)(h % 2049u) - 1024;
        if (DT == UCG_DEV_DT_FLOAT16)  return f2h_rne((float)v);
        if (DT == UCG_DEV_DT_BFLOAT16) return f2b_rne((float)v);
        if (DT == UCG_DEV_DT_FLOAT32)  return __float_as_uint((float)v);
        if (DT == UCG_DEV_DT_FLOAT64)  return (uint64_t)__double_as_longlong((double)v);
        return (uint64_t)v;
    }
    if (DT == UCG_DEV_DT_FLOAT16) {
        const uint64_t e = ((h >> 10) & 0xff) % 17;
        return (sign << 15) | ((e + 7) << 10) | (h & 0x3ff);
    }
    if (DT == UCG_DEV_DT_BFLOAT16) {
        const uint64_t e = ((h >> 7) & 0xff) % 17;
        return (sign << 15) | ((e + 119) << 7) | (h & 0x7f);
    }
    if (DT == UCG_DEV_DT_FLOAT32) {
        const uint64_t e = ((h >> 23) & 0xff) % 17;
        return (sign << 31) | ((e + 119) << 23) | (h & 0x7fffff);
    }
    if (DT == UCG_DEV_DT_FLOAT64) {
        const uint64_t e = ((h >> 52) & 0x7ff) % 17;
        return (sign << 63) | ((e + 1015) << 52) | (h & 0xfffffffffffffull);
    }
    return h;
}

template <int DT>
__global__ void __launch_bounds__(kBlock)
k_fill(void *dst, int dist, uint64_t key, size_t count)
{
    typedef typename DtType<DT>::T T;
    const size_t nthr = (size_t)gridDim.x * kBlock;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < count;
         i += nthr) {
        const uint64_t b = gen_bits<DT>(dist, splitmix64(key ^ (uint64_t)i));
        switch (sizeof(T)) {
        case 1:  static_cast<uint8_t*>(dst)[i]  = (uint8_t)b;  break;
        case 2:  static_cast<uint16_t*>(dst)[i] = (uint16_t)b; break;
        case 4:  static_cast<uint32_t*>(dst)[i] = (uint32_t)b; break;
        default: static_cast<uint64_t*>(dst)[i] = b;           break;
        }
    }
}

} /* namespace ucgdev */

#endif
