/*
 * dev_launch.h - launchers of the combine kernels and the per-dtype rows of
 * the dispatch tables. Each dtype's kernels are instantiated in their own
 * translation unit (dev_inst.hip, compiled once per dtype) so the library
 * builds in parallel; dev_combine.hip assembles the tables from rows<DT>().
 */
#ifndef UCG_DEV_LAUNCH_H_
#define UCG_DEV_LAUNCH_H_

#include <hip/hip_runtime.h>

#include <array>
#include <type_traits>
#include <utility>

#include "ucg_builtin_dev.h"
#include "dev_kernels.h"

namespace ucgdev {

/* UCX_BUILTIN_DEV_MAX_BLOCKS: grid cap of the looping (element-wise) kernels;
 * defined in dev_combine.hip */
int launch_max_blocks();
/* whether the multi-operand kernels run under their occupancy cap
 * (UCX_BUILTIN_DEV_MULTI_CAP, ucg_builtin_dev_set_multi_cap; default yes);
 * likewise */
bool multi_capped();

inline size_t div_up(size_t a, size_t b) { return (a + b - 1) / b; }

inline unsigned grid_for(size_t work_items, size_t per_block, int cap)
{
    size_t g = div_up(work_items, per_block);
    if (g < 1) {
        g = 1;
    }
    if (g > (size_t)cap) {
        g = (size_t)cap;
    }
    return (unsigned)g;
}

/* ------------------------------------------------------------------------ */
/* reduce launchers                                                         */
/* ------------------------------------------------------------------------ */
typedef hipError_t (*reduce_fn_t)(void *dst, const void *src, size_t count,
                                  hipStream_t st);

/* A dispatch packet counts work-items in 32 bits, so one launch covers at
 * most 2^31 16-B vectors (32 GiB per operand); larger operands (HBM holds
 * 288 GB) are cut into such chunks, the ragged head in the first and the tail
 * in the last. */
constexpr size_t kMaxVecPerLaunch = (size_t)1 << 31;

/* The ragged head ends where dst reaches a 128-B line, not merely 16 B: a
 * wave stores 64 x 16 B, and a span that starts inside a line shares its
 * first and last lines with the neighbouring waves (on other XCDs under the
 * identity block map), so every line at a span edge is written twice, in
 * halves. Measured (scripts/dst_offset_probe.py): dst and src 16 B past a
 * line, with 16-B heads, ran at 69 % of 8 TB/s against 84 % on a line. The
 * head is at most 127 B, done by the first lanes of the grid. */
constexpr uintptr_t kLine = 128;

template <typename T>
inline size_t line_head(const void *dst, size_t count)
{
    const uintptr_t ml = (uintptr_t)dst & (kLine - 1);
    const size_t h     = ml ? (kLine - ml) / sizeof(T) : 0;
    return h < count ? h : count;
}

/* XCD-aware tile map when a source's vectors straddle lines (k_reduce_multi,
 * k_reduce_tree; the 2-operand combine always takes it, k_reduce's PF form) */
inline bool straddles_lines(const void *p)
{
    return ((uintptr_t)p & (kLine - 1)) != 0;
}

/* lines of the next tile's src each wave of the 2-operand combine loads
 * ahead (k_reduce's PF form) */
constexpr int kPrefetchLines = 3;

/* the order its three loads issue in (k_reduce's ORD): the next tile's lines
 * first, then src, then dst. The compiler's own order varied with the
 * (dtype, op) and the translation unit; at 256 MiB per operand this order read
 * 0.5-1.1 points above the others for all 7 pairs timed, on two boxes, and at
 * 1 GiB within 0.4 of the best (tools/tune_order, profiles/r06/order/) */
constexpr int kLoadOrder = 2;

/* ... and its XCD map's chunk: 256 tiles per XCD chunk below 1 GiB per
 * operand, the common 64 from there (tools/tune_order, profiles/r06/order/
 * r06zl_*, r06zm_*, fp32 SUM with the order above, one process per size):
 * 256-tile chunks read 86.8 against 83.7 % of 8 TB/s at 64 MiB, 87.9
 * against 86.9 % at 128 MiB, 89.3-89.4 against 88.5 % at 256 MiB (two
 * boxes), 90.1 against 89.0 % at 512 MiB, but 86.1 against 87.1 % at 1 GiB
 * (round 4 found the same with 128-tile chunks: +0.2-0.5 at 256 MiB, -1.4
 * at 1 GiB). */
constexpr unsigned kReduceChunkSmall = 256;
constexpr size_t kReduceChunkSmallMaxVecs = (size_t)1 << 26;   /* 1 GiB per operand */

/* The in-phase multi-operand kernels' PF form (round 5):
 * one line of the next tile per prefetched operand (tools/tune_multi_pf,
 * profiles/r05/pf, 64 MiB per operand, A/B in one process): N = 8 and 16,
 * every operand: 82.3 / 81.2 % of 8 TB/s against 79.7 / 80.5 % for round
 * 4's form (three lines: 82.5 % at 64 MiB but 74.3 % at 256 MiB); N = 4
 * lost 5 points with any prefetch and keeps round 4's form. Tree fan-in:
 * n = NMAX (8, 16) every operand, 85.0 % against 80.5 % at n = 8; otherwise
 * the root's operand only, 83.0 % against 77.7 % at n = 3 and 82.4 against
 * 80.5 % at n = 12 (operands past n reload the root's, so prefetching them
 * fetches its lines again: n = 6 read 78.4 % with every operand). */
constexpr int kMultiPrefetchLines = 1;

/* How far ahead that line lies, in tiles (tools/tune_multi_pf, profiles/r05/
 * pf3 and pf4, A/B in one process). Every operand prefetched: two tiles
 * ahead; k_reduce_multi N = 8 at 64 MiB per operand 84.3 / 85.4 % of 8 TB/s
 * (two runs) against 82.2 / 84.4 % one tile ahead, 80.0 against 78.6 % at
 * 256 MiB, N = 16 81.7 / 81.5 against 81.4 / 81.2 %; the tree fan-in at
 * n = NMAX = 8 85.1 against 83.8 %, equal at 256 MiB and at NMAX = 16. Four
 * and eight tiles are no better. The root's operand alone (tree, n < NMAX):
 * one tile ahead; two lost 1.1 points at n = 3 and were equal at n = 12. */
constexpr int kFullPrefetchTiles = 2;
constexpr int kRootPrefetchTiles = 1;

/* Round 6: k_reduce_multi N = 8 with operands of 128 MiB and
 * more takes its line four tiles ahead (since the lines-first form below
 * took the sizes under 256 MiB, from 256 MiB on; tools/tune_multi_pf, profiles/r06/
 * multi, A/B in one process on four boxes): at 512 MiB per operand (C4's
 * shard) 85.3 / 80.7 / 79.9 / 78.6 % of 8 TB/s against 84.3 / 79.4 / 78.6 /
 * 77.7 % two tiles ahead, at 256 MiB 81.5 / 81.6 / 81.2 against 80.9 / 80.9 /
 * 80.4 %; at 64 MiB two tiles stay ahead by 0.1-0.6 points, and N = 16 loses
 * 2 points at four tiles. (N = 16 without any prefetch read 77.2 against
 * 75.2 % at 256 MiB but 77.5 against 81.1 % at 512 MiB, r06m / r06n: not
 * taken.) PMC at 512 MiB: 1.0101 x the algorithmic bytes
 * against 1.0123 x two tiles ahead (profiles/r06/multi/pmc_by_kernel.txt). */
constexpr int kLargePrefetchTiles = 4;
constexpr size_t kLargePrefetchVecs = (size_t)1 << 23;   /* 128 MiB per operand */

/* Round 6, last: below 256 MiB per operand the every-operand PF forms
 * (k_reduce_multi N = 8 and 16, the tree fan-in at n = NMAX and the exact-n
 * kernels) issue their lines four tiles ahead BEFORE the operand loads (PFO,
 * tile_lines_issue; the 2-operand combine's kLoadOrder). tools/tune_multi_pf,
 * profiles/r06/pfo/, A/B in one process on two boxes: k_reduce_multi N = 8
 * 87.8 / 87.3 % of 8 TB/s at 64 MiB per operand against 86.1 / 84.1 %, 88.5 /
 * 88.1 against 85.2 / 85.2 % at 128 MiB; N = 16 84.6 against 82.2 % at 64 MiB;
 * tree n = 8 87.9 against 85.4 %, exact n = 12 87.4 against 83.5 % and 87.9
 * against 84.5 % at 128 MiB, exact n = 6 87.6 against 84.7 %. At 256 MiB it
 * lost 1.5 points at N = 8 and n = 6 (79.8 against 81.3 %, 83.0 against
 * 84.6 %), so from there the forms above stay. */
constexpr int kPfoTiles = 4;
constexpr size_t kPfoMaxVecs = (size_t)1 << 24;          /* 256 MiB per operand */

/* ... except the tree fan-ins of 9 operands and more, which gained at every
 * size measured (profiles/r06/pfo/r06zg_*, r06zh_*): exact n = 10 79.9 against
 * 77.3 % at 256 MiB and 81.0 against 78.4 % at 512 MiB, n = 12 81.1 against
 * 79.2 % and 76.3 against 75.3 %, n = 16 level at 256 MiB and 84.6 against
 * 81.9 % at 512 MiB. (The multi-operand kernel at N = 16 lost 1.2 points at
 * 256 MiB and gained 2.0 at 512 MiB: not taken.) */
constexpr int kPfoAnySizeOperands = 9;

template <typename T, int OP>
void launch_vec(T *d, const T *s, size_t head, size_t nvec, size_t tail, hipStream_t st)
{
    constexpr size_t V = 16 / sizeof(T);
    size_t done = 0;
    do {
        const size_t chunk = nvec - done < kMaxVecPerLaunch ? nvec - done : kMaxVecPerLaunch;
        const bool first = (done == 0), last = (done + chunk == nvec);
        const size_t off = first ? 0 : head + done * V;
        /* one tile of U vectors per lane: grid sized to the chunk (no loop),
         * and to the head's lanes */
        unsigned grid = grid_for(chunk, (size_t)kReduceBlock, 0x7fffffff);
        if (first && div_up(head, kReduceBlock) > grid) {
            grid = (unsigned)div_up(head, kReduceBlock);
        }
        if (chunk < kReduceChunkSmallMaxVecs) {
            hipLaunchKernelGGL((k_reduce<T, OP, 1, 1, kReduceBlock, 1, kPrefetchLines, kLoadOrder,
                                         kReduceChunkSmall>),
                               dim3(grid), dim3(kReduceBlock), 0, st, d + off, s + off,
                               first ? head : 0, chunk, last ? tail : 0);
        } else {
            hipLaunchKernelGGL((k_reduce<T, OP, 1, 1, kReduceBlock, 1, kPrefetchLines, kLoadOrder>),
                               dim3(grid), dim3(kReduceBlock), 0, st, d + off, s + off,
                               first ? head : 0, chunk, last ? tail : 0);
        }
        done += chunk;
    } while (done < nvec);
}

/* k_reduce_shift, chunked like launch_vec. Q = (src - dst) mod 16 B in
 * whole words, rb the remaining bytes; pairs a dtype cannot produce (rb != 0
 * for 4-B elements, anything but Q = 2 for 8-B ones) are not instantiated. */
template <typename T, int OP, int Q>
void launch_shift(T *d, const T *s, size_t head, size_t nvec, size_t tail,
                  unsigned rb, hipStream_t st)
{
    constexpr size_t V = 16 / sizeof(T);
    if constexpr ((sizeof(T) == 8 && Q != 2) || (sizeof(T) == 4 && Q == 0)) {
        (void)d; (void)s; (void)head; (void)nvec; (void)tail; (void)rb; (void)st;
        return;
    } else {
        size_t done = 0;
        do {
            const size_t chunk = nvec - done < kMaxVecPerLaunch ? nvec - done
                                                                : kMaxVecPerLaunch;
            const bool first = (done == 0), last = (done + chunk == nvec);
            const size_t off = first ? 0 : head + done * V;
            size_t items = chunk;
            if (first && head > items) items = head;
            if (last && tail > items) items = tail;
            const unsigned grid = grid_for(items, (size_t)kReduceBlock, 0x7fffffff);
            hipLaunchKernelGGL((k_reduce_shift<T, OP, Q, kPrefetchLines>), dim3(grid),
                               dim3(kReduceBlock),
                               0, st, d + off, s + off, first ? head : 0, chunk,
                               last ? tail : 0, rb);
            done += chunk;
        } while (done < nvec);
    }
}

template <int DT, int OP>
hipError_t launch_reduce(void *dst, const void *src, size_t count, hipStream_t st)
{
    typedef typename DtType<DT>::T T;
    constexpr size_t sz = sizeof(T);
    constexpr size_t V  = 16 / sz;
    T *d       = static_cast<T*>(dst);
    const T *s = static_cast<const T*>(src);
    const uintptr_t md = (uintptr_t)dst & 15, ms = (uintptr_t)src & 15;

    if (md != ms && (md | ms) % sz != 0) {
        /* not even element-aligned: element loop */
        const unsigned grid = grid_for(count, (size_t)kBlock * 4,
                                       launch_max_blocks());
        hipLaunchKernelGGL((k_reduce_scalar<T, OP>), dim3(grid), dim3(kBlock),
                           0, st, d, s, count);
        return hipGetLastError();
    }
    const size_t head = line_head<T>(dst, count);
    const size_t rem  = count - head;
    const size_t nvec = rem / V, tail = rem % V;

    if (md != ms) {
        /* operands disagree mod 16 B: src realigned in registers */
        const unsigned r = (unsigned)((ms + 16 - md) & 15);
        switch (r >> 2) {
        case 0:  launch_shift<T, OP, 0>(d, s, head, nvec, tail, r & 3, st); break;
        case 1:  launch_shift<T, OP, 1>(d, s, head, nvec, tail, r & 3, st); break;
        case 2:  launch_shift<T, OP, 2>(d, s, head, nvec, tail, r & 3, st); break;
        default: launch_shift<T, OP, 3>(d, s, head, nvec, tail, r & 3, st); break;
        }
        return hipGetLastError();
    }
    launch_vec<T, OP>(d, s, head, nvec, tail, st);
    return hipGetLastError();
}

template <int DT, int OP>
constexpr reduce_fn_t reduce_entry()
{
    if constexpr (pair_supported(DT, OP)) {
        return &launch_reduce<DT, OP>;
    } else {
        return nullptr;
    }
}

template <int DT, int... OPS>
constexpr std::array<reduce_fn_t, UCG_DEV_OP_LAST>
reduce_row(std::integer_sequence<int, OPS...>)
{
    return {reduce_entry<DT, OPS>()...};
}


/* ---- multi-operand (recursive-doubling association) --------------------- */
typedef hipError_t (*multi_fn_t)(void *dst, const SrcList &srcs, unsigned n,
                                 unsigned self, size_t count, hipStream_t st);

/* Occupancy cap of the multi-operand kernels (UCG_MULTI_CAP_CLOBBER,
 * dev_kernels.h): with 4 or more operands (tree: NMAX 8 or 16) the aligned
 * and the realigning forms run capped. The uncapped forms
 * are also built for fp32 and fp64 SUM, for A/B runs in one process
 * (ucg_builtin_dev_set_multi_cap(0): bench.py's one-shot reduce-scatter over
 * xGMI); every other pair always runs capped. */
template <typename T, int OP>
constexpr bool uncapped_ab()
{
    return OP == UCG_DEV_OP_SUM && (std::is_same<T, float>::value ||
                                    std::is_same<T, double>::value);
}

template <typename T, int OP, int N>
hipError_t launch_multi_n(void *dst, const SrcList &srcs, unsigned self,
                                 size_t count, hipStream_t st)
{
    constexpr size_t sz = sizeof(T), V = 16 / sz;
    const uintptr_t md = (uintptr_t)dst & 15;
    bool aligned = true;
    for (int m = 0; m < N; m++) {
        aligned = aligned && (((uintptr_t)srcs.p[m] & 15) == md);
    }
    T *d = static_cast<T*>(dst);
    const size_t head = line_head<T>(dst, count);
    bool xm = false;
    for (int m = 0; m < N; m++) {
        xm = xm || straddles_lines(static_cast<const T*>(srcs.p[m]) + head);
    }
    /* capped: always with 4+ operands, unless switched off for an A/B pair */
    constexpr bool can_cap = N >= 4;
    const bool cap = can_cap && (!uncapped_ab<T, OP>() || multi_capped());
    const size_t rem = count - head, nvec = rem / V, tail = rem % V;
    size_t done = 0;
    do {
        const size_t chunk = nvec - done < kMaxVecPerLaunch ? nvec - done : kMaxVecPerLaunch;
        const bool first = (done == 0), last = (done + chunk == nvec);
        const size_t off = first ? 0 : head + done * V;
        SrcList sl;
        for (int m = 0; m < kMaxMulti; m++) {
            sl.p[m] = srcs.p[m] ? static_cast<const T*>(srcs.p[m]) + off : nullptr;
        }
        const size_t h = first ? head : 0, t = last ? tail : 0;
        if (aligned) {
            unsigned grid = grid_for(chunk, (size_t)kReduceBlock * kMultiU, 0x7fffffff);
            if (first && div_up(head, kReduceBlock) > grid) {
                grid = (unsigned)div_up(head, kReduceBlock);
            }
            const dim3 g(grid), b(kReduceBlock);
            if constexpr (N >= 8) {
                if (cap && chunk < kPfoMaxVecs) {
                    /* the PF form, lines issued first (PFO), four tiles ahead */
                    hipLaunchKernelGGL((k_reduce_multi<T, OP, N, 1, 1, kMultiPrefetchLines, N,
                                                       kPfoTiles, 1>),
                                       g, b, 0, st, d + off, sl, self, h, chunk, t);
                } else if (cap && N == 8 && chunk >= kLargePrefetchVecs) {
                    /* the PF form, large operands: the line four tiles ahead */
                    hipLaunchKernelGGL((k_reduce_multi<T, OP, N, 1, 1, kMultiPrefetchLines, N,
                                                       kLargePrefetchTiles>),
                                       g, b, 0, st, d + off, sl, self, h, chunk, t);
                } else if (cap) {
                    /* the PF form: XCD map, the next tile's line of every operand */
                    hipLaunchKernelGGL((k_reduce_multi<T, OP, N, 1, 1, kMultiPrefetchLines, N,
                                                       kFullPrefetchTiles>),
                                       g, b, 0, st, d + off, sl, self, h, chunk, t);
                } else if constexpr (uncapped_ab<T, OP>()) {
                    if (xm)
                        hipLaunchKernelGGL((k_reduce_multi<T, OP, N, 1, 0>), g, b, 0, st,
                                           d + off, sl, self, h, chunk, t);
                    else
                        hipLaunchKernelGGL((k_reduce_multi<T, OP, N, 0, 0>), g, b, 0, st,
                                           d + off, sl, self, h, chunk, t);
                }
            } else if (cap) {
                if (xm)
                    hipLaunchKernelGGL((k_reduce_multi<T, OP, N, 1, can_cap>), g, b, 0, st,
                                       d + off, sl, self, h, chunk, t);
                else
                    hipLaunchKernelGGL((k_reduce_multi<T, OP, N, 0, can_cap>), g, b, 0, st,
                                       d + off, sl, self, h, chunk, t);
            } else if constexpr (!can_cap || uncapped_ab<T, OP>()) {
                if (xm)
                    hipLaunchKernelGGL((k_reduce_multi<T, OP, N, 1, 0>), g, b, 0, st,
                                       d + off, sl, self, h, chunk, t);
                else
                    hipLaunchKernelGGL((k_reduce_multi<T, OP, N, 0, 0>), g, b, 0, st,
                                       d + off, sl, self, h, chunk, t);
            }
        } else {
            /* some operand out of phase with dst: realigned in registers,
             * capped as the aligned form (round 4: with its next-tile loads
             * temporal, 84.8 % capped against 78.1 % uncapped) */
            size_t items = chunk;
            if (first && head > items) items = head;
            if (last && tail > items) items = tail;
            const unsigned grid = grid_for(items, kReduceBlock, 0x7fffffff);
            if (cap) {
                hipLaunchKernelGGL((k_reduce_multi_shift<T, OP, N, can_cap>), dim3(grid),
                                   dim3(kReduceBlock), 0, st, d + off, sl, self, h, chunk, t);
            } else if constexpr (!can_cap || uncapped_ab<T, OP>()) {
                hipLaunchKernelGGL((k_reduce_multi_shift<T, OP, N, 0>), dim3(grid),
                                   dim3(kReduceBlock), 0, st, d + off, sl, self, h, chunk, t);
            }
        }
        done += chunk;
    } while (done < nvec);
    return hipGetLastError();
}

template <int DT, int OP>
hipError_t launch_multi(void *dst, const SrcList &srcs, unsigned n,
                               unsigned self, size_t count, hipStream_t st)
{
    typedef typename DtType<DT>::T T;
    switch (n) {
    case 1:  return launch_multi_n<T, OP, 1>(dst, srcs, self, count, st);
    case 2:  return launch_multi_n<T, OP, 2>(dst, srcs, self, count, st);
    case 4:  return launch_multi_n<T, OP, 4>(dst, srcs, self, count, st);
    case 8:  return launch_multi_n<T, OP, 8>(dst, srcs, self, count, st);
    case 16: return launch_multi_n<T, OP, 16>(dst, srcs, self, count, st);
    default: return hipErrorInvalidValue;
    }
}

template <int DT, int OP>
constexpr multi_fn_t multi_entry()
{
    if constexpr (pair_supported(DT, OP)) {
        return &launch_multi<DT, OP>;
    } else {
        return nullptr;
    }
}

template <int DT, int... OPS>
constexpr std::array<multi_fn_t, UCG_DEV_OP_LAST>
multi_row(std::integer_sequence<int, OPS...>)
{
    return {multi_entry<DT, OPS>()...};
}


/* ---- generator ---------------------------------------------------------- */
typedef void (*fill_fn_t)(void *dst, int dist, uint64_t key, size_t count,
                          hipStream_t st);

template <int DT>
void launch_fill(void *dst, int dist, uint64_t key, size_t count,
                        hipStream_t st)
{
    const unsigned grid = grid_for(count, kBlock, 4096);
    hipLaunchKernelGGL((k_fill<DT>), dim3(grid), dim3(kBlock), 0, st, dst, dist,
                       key, count);
}



/* ---- tree fan-in (sequential association) ------------------------------- */
typedef hipError_t (*tree_fn_t)(void *dst, const SrcList &srcs, unsigned n,
                                size_t count, hipStream_t st);

template <typename T, int OP, int NMAX>
void launch_tree_n(T *d, const SrcList &srcs, unsigned n, size_t head, size_t nvec,
                   size_t tail, bool aligned, bool xm, hipStream_t st)
{
    constexpr size_t V = 16 / sizeof(T);
    /* capped from 5 operands on (NMAX 8 and 16), as launch_multi_n */
    constexpr bool can_cap = NMAX >= 8;
    const bool cap = can_cap && (!uncapped_ab<T, OP>() || multi_capped());
    size_t done = 0;
    do {
        const size_t chunk = nvec - done < kMaxVecPerLaunch ? nvec - done : kMaxVecPerLaunch;
        const bool first = (done == 0), last = (done + chunk == nvec);
        const size_t off = first ? 0 : head + done * V;
        SrcList sl;
        for (int m = 0; m < kMaxMulti; m++) {
            sl.p[m] = srcs.p[m] ? static_cast<const T*>(srcs.p[m]) + off : nullptr;
        }
        const size_t h = first ? head : 0, t = last ? tail : 0;
        if (aligned) {
            unsigned grid = grid_for(chunk, kReduceBlock, 0x7fffffff);
            if (first && div_up(head, kReduceBlock) > grid) {
                grid = (unsigned)div_up(head, kReduceBlock);
            }
            const dim3 g(grid), b(kReduceBlock);
            constexpr int L = kMultiPrefetchLines;
            constexpr int D = kRootPrefetchTiles, DF = kFullPrefetchTiles;
            if constexpr (!can_cap) {
                /* the PF form: the root's next line */
                hipLaunchKernelGGL((k_reduce_tree<T, OP, NMAX, 1, 0, L, 1, D>), g, b, 0, st,
                                   d + off, sl, n, h, chunk, t);
            } else if (cap) {
                /* the PF form, capped: every operand's next line when n fills
                 * NMAX, else the root's only */
                if (n == (unsigned)NMAX && (NMAX >= kPfoAnySizeOperands || chunk < kPfoMaxVecs))
                    hipLaunchKernelGGL((k_reduce_tree<T, OP, NMAX, 1, 1, L, NMAX, kPfoTiles, 1>),
                                       g, b, 0, st, d + off, sl, n, h, chunk, t);
                else if (n == (unsigned)NMAX)
                    hipLaunchKernelGGL((k_reduce_tree<T, OP, NMAX, 1, 1, L, NMAX, DF>), g, b, 0, st,
                                       d + off, sl, n, h, chunk, t);
                else
                    hipLaunchKernelGGL((k_reduce_tree<T, OP, NMAX, 1, 1, L, 1, D>), g, b, 0, st,
                                       d + off, sl, n, h, chunk, t);
            } else if constexpr (uncapped_ab<T, OP>()) {
                if (xm)
                    hipLaunchKernelGGL((k_reduce_tree<T, OP, NMAX, 1, 0>), g, b, 0, st,
                                       d + off, sl, n, h, chunk, t);
                else
                    hipLaunchKernelGGL((k_reduce_tree<T, OP, NMAX, 0, 0>), g, b, 0, st,
                                       d + off, sl, n, h, chunk, t);
            }
        } else {
            /* some operand out of phase with dst: realigned in registers */
            size_t items = chunk;
            if (first && head > items) items = head;
            if (last && tail > items) items = tail;
            const unsigned grid = grid_for(items, kReduceBlock, 0x7fffffff);
            /* capped as k_reduce_multi_shift */
            if (cap) {
                hipLaunchKernelGGL((k_reduce_tree_shift<T, OP, NMAX, can_cap>), dim3(grid),
                                   dim3(kReduceBlock), 0, st, d + off, sl, n, h, chunk, t);
            } else if constexpr (!can_cap || uncapped_ab<T, OP>()) {
                hipLaunchKernelGGL((k_reduce_tree_shift<T, OP, NMAX, 0>), dim3(grid),
                                   dim3(kReduceBlock), 0, st, d + off, sl, n, h, chunk, t);
            }
        }
        done += chunk;
    } while (done < nvec);
}

/* Round 6 (tree n = 12 at 82.4 %): in-phase operands of a
 * fan-in that does not fill its NMAX bucket (5-7, 9-15 children and root)
 * take a kernel built for exactly n operands - no reloads of the root's
 * operand past n - in the n == NMAX form (capped, every operand's line two
 * tiles ahead). tools/tune_multi_pf, profiles/r06/multi/r06m_pf_tree_*:
 * n = 12 84.2 % of 8 TB/s at 64 MiB per operand against 82.0 % (the bucket's
 * root-only form) and 76.8 against 75.4 % at 256 MiB; n = 6 84.5 against
 * 82.1 %. Prefetching every operand in the NMAX = 16 kernel instead lost
 * (76.7 %: its registers pass the occupancy cap). n <= 4 keeps the
 * uncapped bucket (an exact capped n = 3 read 69 %). */
template <typename T, int OP, int NX>
void launch_tree_exact(T *d, const SrcList &srcs, size_t head, size_t nvec, size_t tail,
                       hipStream_t st)
{
    constexpr size_t V = 16 / sizeof(T);
    size_t done = 0;
    do {
        const size_t chunk = nvec - done < kMaxVecPerLaunch ? nvec - done : kMaxVecPerLaunch;
        const bool first = (done == 0), last = (done + chunk == nvec);
        const size_t off = first ? 0 : head + done * V;
        SrcList sl;
        for (int m = 0; m < kMaxMulti; m++) {
            sl.p[m] = srcs.p[m] ? static_cast<const T*>(srcs.p[m]) + off : nullptr;
        }
        unsigned grid = grid_for(chunk, kReduceBlock, 0x7fffffff);
        if (first && div_up(head, kReduceBlock) > grid) {
            grid = (unsigned)div_up(head, kReduceBlock);
        }
        if (NX >= kPfoAnySizeOperands || chunk < kPfoMaxVecs) {
            hipLaunchKernelGGL((k_reduce_tree<T, OP, NX, 1, 1, kMultiPrefetchLines, NX,
                                              kPfoTiles, 1>),
                               dim3(grid), dim3(kReduceBlock), 0, st, d + off, sl,
                               (unsigned)NX, first ? head : 0, chunk, last ? tail : 0);
        } else {
            hipLaunchKernelGGL((k_reduce_tree<T, OP, NX, 1, 1, kMultiPrefetchLines, NX,
                                              kFullPrefetchTiles>),
                               dim3(grid), dim3(kReduceBlock), 0, st, d + off, sl,
                               (unsigned)NX, first ? head : 0, chunk, last ? tail : 0);
        }
        done += chunk;
    } while (done < nvec);
}

template <int DT, int OP>
hipError_t launch_tree(void *dst, const SrcList &srcs, unsigned n, size_t count,
                       hipStream_t st)
{
    typedef typename DtType<DT>::T T;
    constexpr size_t sz = sizeof(T), V = 16 / sz;
    const uintptr_t md = (uintptr_t)dst & 15;
    bool aligned = true;
    for (unsigned m = 0; m < n; m++) {
        aligned = aligned && (((uintptr_t)srcs.p[m] & 15) == md);
    }
    T *d = static_cast<T*>(dst);
    const size_t head = line_head<T>(dst, count);
    bool xm = false;
    for (unsigned m = 0; m < n; m++) {
        xm = xm || straddles_lines(static_cast<const T*>(srcs.p[m]) + head);
    }
    const size_t rem = count - head, nvec = rem / V, tail = rem % V;
    if (aligned && n > 4 && n != 8 && n != 16 && (!uncapped_ab<T, OP>() || multi_capped())) {
        switch (n) {
        case 5:  launch_tree_exact<T, OP, 5>(d, srcs, head, nvec, tail, st); break;
        case 6:  launch_tree_exact<T, OP, 6>(d, srcs, head, nvec, tail, st); break;
        case 7:  launch_tree_exact<T, OP, 7>(d, srcs, head, nvec, tail, st); break;
        case 9:  launch_tree_exact<T, OP, 9>(d, srcs, head, nvec, tail, st); break;
        case 10: launch_tree_exact<T, OP, 10>(d, srcs, head, nvec, tail, st); break;
        case 11: launch_tree_exact<T, OP, 11>(d, srcs, head, nvec, tail, st); break;
        case 12: launch_tree_exact<T, OP, 12>(d, srcs, head, nvec, tail, st); break;
        case 13: launch_tree_exact<T, OP, 13>(d, srcs, head, nvec, tail, st); break;
        case 14: launch_tree_exact<T, OP, 14>(d, srcs, head, nvec, tail, st); break;
        default: launch_tree_exact<T, OP, 15>(d, srcs, head, nvec, tail, st); break;
        }
        return hipGetLastError();
    }
    if (n <= 4) {
        launch_tree_n<T, OP, 4>(d, srcs, n, head, nvec, tail, aligned, xm, st);
    } else if (n <= 8) {
        launch_tree_n<T, OP, 8>(d, srcs, n, head, nvec, tail, aligned, xm, st);
    } else {
        launch_tree_n<T, OP, 16>(d, srcs, n, head, nvec, tail, aligned, xm, st);
    }
    return hipGetLastError();
}

template <int DT, int OP>
constexpr tree_fn_t tree_entry()
{
    if constexpr (pair_supported(DT, OP)) {
        return &launch_tree<DT, OP>;
    } else {
        return nullptr;
    }
}

template <int DT, int... OPS>
constexpr std::array<tree_fn_t, UCG_DEV_OP_LAST>
tree_row(std::integer_sequence<int, OPS...>)
{
    return {tree_entry<DT, OPS>()...};
}


/* every launcher of one dtype */
struct RowSet {
    std::array<reduce_fn_t, UCG_DEV_OP_LAST> reduce;
    std::array<multi_fn_t, UCG_DEV_OP_LAST>  multi;
    std::array<tree_fn_t, UCG_DEV_OP_LAST>   tree;
    fill_fn_t                                fill;
};

template <int DT>
RowSet make_rows()
{
    return {reduce_row<DT>(std::make_integer_sequence<int, UCG_DEV_OP_LAST>()),
            multi_row<DT>(std::make_integer_sequence<int, UCG_DEV_OP_LAST>()),
            tree_row<DT>(std::make_integer_sequence<int, UCG_DEV_OP_LAST>()),
            &launch_fill<DT>};
}

/* defined in dev_inst.hip, one translation unit per dtype */
template <int DT> RowSet rows();
template <> RowSet rows<0>();
template <> RowSet rows<1>();
template <> RowSet rows<2>();
template <> RowSet rows<3>();
template <> RowSet rows<4>();
template <> RowSet rows<5>();
template <> RowSet rows<6>();
template <> RowSet rows<7>();
template <> RowSet rows<8>();
template <> RowSet rows<9>();
template <> RowSet rows<10>();
template <> RowSet rows<11>();
static_assert(UCG_DEV_DT_LAST == 12, "one rows<> specialisation per dtype");

}  // namespace ucgdev

#endif
