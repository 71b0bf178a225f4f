/*
 * tune_combine.hip - standalone A/B harness for the fp32 SUM combine kernel
 * geometry on MI355X (not part of the product libraries).
 *
 *   hipcc -O3 --offload-arch=gfx950 -I../../include tune_combine.hip -o tune
 *   ./tune [count_log2=26] [rounds=5]
 *
 * Every variant runs on the same buffers, interleaved over `rounds` rounds
 * (cdna_hip_programming.md rule 24); prints min/median us and GB/s on the
 * 3N-byte algorithmic basis. Results are checked against the baseline
 * variant's output bit for bit.
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

#define CHECK(x)                                                               \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,          \
                    hipGetErrorString(e_));                                    \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

/* variant A: grid-stride loop, U vectors per lane per iteration (the first
 * product kernel, kept here as the A/B reference) */
template <int U, int NT>
__global__ void __launch_bounds__(256)
k_gridstride(float *dst, const float *src, size_t nvec)
{
    const size_t nthr = (size_t)gridDim.x * 256;
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (size_t)(U - 1) * nthr < nvec; i += (size_t)U * nthr) {
        u32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            a[u] = ld16<NT>(s4 + i + u * nthr);
            b[u] = ld16<NT>(d4 + i + u * nthr);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            st16<NT>(d4 + i + u * nthr, vapply<float, 0>(a[u], b[u]));
        }
    }
    for (; i < nvec; i += nthr) {
        st16<NT>(d4 + i, vapply<float, 0>(ld16<NT>(s4 + i), ld16<NT>(d4 + i)));
    }
}

/* variant E: oneshot with separate temporal choice for loads and stores,
 * optional XCD-contiguous block remap */
template <int U, int NTL, int NTS, int XCD>
__global__ void __launch_bounds__(256)
k_oneshot2(float *dst, const float *src, size_t nvec)
{
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
    size_t blk = blockIdx.x;
    if (XCD) {
        const size_t nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = blk % 8;
        blk = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + blk / 8;
    }
    const size_t base = blk * 256 * U + threadIdx.x;
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + u * 256;
        if (i < nvec) {
            a[u] = ld16<NTL>(s4 + i);
            b[u] = ld16<NTL>(d4 + i);
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + u * 256;
        if (i < nvec) {
            st16<NTS>(d4 + i, vapply<float, 0>(a[u], b[u]));
        }
    }
}

/* variant F: oneshot, block size BS, U vectors per lane; CONTIG=1 gives each
 * lane U consecutive 16-B vectors (32/64 B contiguous per lane); DFIRST
 * loads dst before src */
template <int U, int BS, int CONTIG, int DFIRST>
__global__ void __launch_bounds__(BS)
k_oneshot3(float *dst, const float *src, size_t nvec)
{
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
    const size_t blk = (size_t)blockIdx.x * BS * U;
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = CONTIG ? blk + threadIdx.x * U + u : blk + threadIdx.x + u * BS;
        if (i < nvec) {
            if (DFIRST) {
                b[u] = ld16<1>(d4 + i);
                a[u] = ld16<1>(s4 + i);
            } else {
                a[u] = ld16<1>(s4 + i);
                b[u] = ld16<1>(d4 + i);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = CONTIG ? blk + threadIdx.x * U + u : blk + threadIdx.x + u * BS;
        if (i < nvec) {
            st16<1>(d4 + i, vapply<float, 0>(a[u], b[u]));
        }
    }
}

/* variant X: the product geometry (one wave, one vector per lane) with the
 * workgroup -> tile map made XCD-aware. The dispatcher deals workgroup b to
 * XCD b % 8; here XCD x takes chunks of C consecutive tiles (C = 0: one
 * contiguous eighth of the buffer), so each XCD's UTCL2 and L2 see 1/8 of
 * the pages instead of all of them. Tests the TLB-reach hypothesis for the
 * 1 GiB operands (2 GiB working set). */
template <int C>
__global__ void __launch_bounds__(64)
k_xcd(float *dst, const float *src, size_t nvec, unsigned ntiles)
{
    const unsigned b = blockIdx.x;
    const unsigned x = b & 7, j = b >> 3;
    const unsigned full = ntiles & ~7u;           /* tiles in whole rounds of 8 */
    const unsigned T = full >> 3;                 /* tiles per XCD */
    unsigned tile;
    if (b >= full) {
        tile = b;                                 /* ragged last round: identity */
    } else if (C == 0) {
        tile = x * T + j;
    } else {
        const unsigned R = T / C, r = T % C;      /* whole chunk rows, remainder */
        tile = (j < R * C) ? (j / C) * (8u * C) + x * C + (j % C)
                           : R * 8u * C + x * r + (j - R * C);
    }
    const size_t i = (size_t)tile * 64 + threadIdx.x;
    if (i < nvec) {
        const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
        u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
        u32x4 a = ld16<1>(s4 + i);
        u32x4 v = ld16<1>(d4 + i);
        st16<1>(d4 + i, vapply<float, 0>(a, v));
    }
}

/* Ceiling probes in the product geometry (one wave, one 16-B vector per lane
 * per stream, non-temporal), to place the combine's 2-read + 1-write mix:
 *   K=0 read-only   both operands loaded, XOR-folded, one word stored per
 *                   wave only if the fold hits a sentinel (never)
 *   K=1 write-only  dst overwritten with a constant
 *   K=2 copy        dst = src (1 read + 1 write)
 * Bytes counted per variant: 2N, N and 2N (reported on the 3N scale by the
 * harness; multiply by 2/3, 1/3 and 2/3 for their own rate). */
template <int K>
__global__ void __launch_bounds__(64)
k_ceiling(float *dst, const float *src, size_t nvec)
{
    const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= nvec) {
        return;
    }
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
    if (K == 0) {
        const u32x4 a = ld16<1>(s4 + i);
        const u32x4 b = ld16<1>(d4 + i);
        const unsigned x = a[0] ^ a[1] ^ a[2] ^ a[3] ^ b[0] ^ b[1] ^ b[2] ^ b[3];
        if (x == 0x9e3779b9u && threadIdx.x == 0) {
            reinterpret_cast<unsigned*>(d4)[i * 4] = x;
        }
    } else if (K == 1) {
        st16<1>(d4 + i, u32x4{1u, 2u, 3u, 4u});
    } else {
        st16<1>(d4 + i, ld16<1>(s4 + i));
    }
}

/* variant H: one-wave workgroups on a capped grid, each looping over tiles
 * (fewer workgroups for the dispatcher to launch); PIPE = 1 loads the next
 * tile before storing the current one */
template <int PIPE>
__global__ void __launch_bounds__(64)
k_gs64(float *dst, const float *src, size_t nvec)
{
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
    const size_t stride = (size_t)gridDim.x * 64;
    size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (!PIPE) {
        for (; i < nvec; i += stride) {
            st16<1>(d4 + i, vapply<float, 0>(ld16<1>(s4 + i), ld16<1>(d4 + i)));
        }
        return;
    }
    if (i >= nvec) {
        return;
    }
    u32x4 a = ld16<1>(s4 + i), b = ld16<1>(d4 + i);
    for (;;) {
        const size_t j = i + stride;
        const bool more = j < nvec;
        u32x4 a2, b2;
        if (more) {
            a2 = ld16<1>(s4 + j);
            b2 = ld16<1>(d4 + j);
        }
        st16<1>(d4 + i, vapply<float, 0>(a, b));
        if (!more) {
            break;
        }
        a = a2;
        b = b2;
        i = j;
    }
}

/* variant G: oneshot with buffer loads/stores and explicit cache-policy aux
 * bits (gfx950: bit0 sc0, bit1 nt, bit4 sc1); byte offsets < 4 GiB */
template <int U, int AUXL, int AUXS, int BS = 256>
__global__ void __launch_bounds__(BS)
k_oneshot_buf(float *dst, const float *src, size_t nvec)
{
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)src, 0, (int)0xFFFFFFFF, 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        (void*)dst, 0, (int)0xFFFFFFFF, 0x00020000);
    const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + u * BS;
        if (i < nvec) {
            a[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)(i * 16), 0, AUXL));
            b[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, (unsigned)(i * 16), 0, AUXL));
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + u * BS;
        if (i < nvec) {
            __builtin_amdgcn_raw_buffer_store_b128(vapply<float, 0>(a[u], b[u]), rd, (unsigned)(i * 16), 0, AUXS);
        }
    }
}

/* variant B: each block owns one contiguous chunk of vectors */
template <int U, int NT, int BS>
__global__ void __launch_bounds__(BS)
k_chunked(float *dst, const float *src, size_t nvec, size_t per_block)
{
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
    size_t beg = (size_t)blockIdx.x * per_block;
    size_t end = beg + per_block < nvec ? beg + per_block : nvec;
    size_t i   = beg + threadIdx.x;
    for (; i + (U - 1) * BS < end; i += U * BS) {
        u32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            a[u] = ld16<NT>(s4 + i + u * BS);
            b[u] = ld16<NT>(d4 + i + u * BS);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            st16<NT>(d4 + i + u * BS, vapply<float, 0>(a[u], b[u]));
        }
    }
    for (; i < end; i += BS) {
        st16<NT>(d4 + i, vapply<float, 0>(ld16<NT>(s4 + i), ld16<NT>(d4 + i)));
    }
}

/* variant C: no loop, one tile of U vectors per thread, huge grid */
template <int U, int NT, int BS>
__global__ void __launch_bounds__(BS)
k_oneshot(float *dst, const float *src, size_t nvec)
{
    const u32x4 *s4 = reinterpret_cast<const u32x4*>(src);
    u32x4 *d4       = reinterpret_cast<u32x4*>(dst);
    const size_t base = (size_t)blockIdx.x * BS * U + threadIdx.x;
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + u * BS;
        if (i < nvec) {
            a[u] = ld16<NT>(s4 + i);
            b[u] = ld16<NT>(d4 + i);
        }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + u * BS;
        if (i < nvec) {
            st16<NT>(d4 + i, vapply<float, 0>(a[u], b[u]));
        }
    }
}

/* variant D: loads of both operands with sc0/sc1/nt bits via the buffer
 * intrinsic (aux), product loop structure */
template <int U, int AUXL, int AUXS, int BS>
__global__ void __launch_bounds__(BS)
k_buffer(float *dst, const float *src, size_t nvec)
{
    /* nvec * 16 <= 2^32 assumed by the harness sizes */
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)src, 0, (int)0xFFFFFFFF, 0x00020000);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        (void*)dst, 0, (int)0xFFFFFFFF, 0x00020000);
    const size_t nthr = (size_t)gridDim.x * BS;
    size_t i = (size_t)blockIdx.x * BS + threadIdx.x;
    for (; i + (U - 1) * nthr < nvec; i += U * nthr) {
        u32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const unsigned off = (unsigned)((i + u * nthr) * 16);
            a[u] = __builtin_bit_cast(u32x4,
                       __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUXL));
            b[u] = __builtin_bit_cast(u32x4,
                       __builtin_amdgcn_raw_buffer_load_b128(rd, off, 0, AUXL));
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const unsigned off = (unsigned)((i + u * nthr) * 16);
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int,
                                   vapply<float, 0>(a[u], b[u])),
                rd, off, 0, AUXS);
        }
    }
    for (; i < nvec; i += nthr) {
        const unsigned off = (unsigned)(i * 16);
        u32x4 a = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUXL));
        u32x4 b = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, off, 0, AUXL));
        __builtin_amdgcn_raw_buffer_store_b128(vapply<float, 0>(a, b), rd, off, 0, AUXS);
    }
}

struct Variant {
    std::string name;
    std::function<void(float*, const float*, size_t, hipStream_t)> run;
    std::vector<float> us;
};

int main(int argc, char **argv)
{
    const int lg     = argc > 1 ? atoi(argv[1]) : 26;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int iters  = 20;
    const size_t n = (size_t)1 << lg, nvec = n / 4;
    float *src, *dst, *ref;
    CHECK(hipMalloc(&src, n * 4));
    CHECK(hipMalloc(&dst, n * 4));
    CHECK(hipMalloc(&ref, n * 4));
    hipStream_t st;
    CHECK(hipStreamCreate(&st));

    std::vector<Variant> vs;
    /* product kernel first: everything is checked against its output */
    vs.push_back({"product k_reduce<f32,SUM,1,NT1,bs64>", [=](float *d, const float *s, size_t nv, hipStream_t q) {
        unsigned g = (unsigned)((nv + kReduceBlock * kReduceU - 1) / (kReduceBlock * kReduceU));
        hipLaunchKernelGGL((k_reduce<float, 0, kReduceU, 1, kReduceBlock>), dim3(g), dim3(kReduceBlock), 0, q, d, s, (size_t)0, nv, (size_t)0);
    }, {}});
    vs.push_back({"previous k_reduce<f32,SUM,4,NT1,bs256>", [=](float *d, const float *s, size_t nv, hipStream_t q) {
        unsigned g = (unsigned)((nv + 1023) / 1024);
        hipLaunchKernelGGL((k_reduce<float, 0, 4, 1, 256>), dim3(g), dim3(256), 0, q, d, s, (size_t)0, nv, (size_t)0);
    }, {}});
    auto xcd = [&](int C) {
        char buf[128];
        snprintf(buf, sizeof(buf), "xcd-aware bs64 U1 chunk%d", C);
        vs.push_back({buf, [=](float *d, const float *s, size_t nv, hipStream_t q) {
            unsigned g = (unsigned)((nv + 63) / 64);
#define XC(A) if (C == A) hipLaunchKernelGGL((k_xcd<A>), dim3(g), dim3(64), 0, q, d, s, nv, g)
            XC(0); XC(16); XC(32); XC(64); XC(128); XC(256); XC(2048);
#undef XC
        }, {}});
    };
    if (getenv("TUNE_CEILING")) {
        const char *names[3] = {"ceiling read-only 2N (x3/2 for own rate)",
                                "ceiling write-only N (x3 for own rate)",
                                "ceiling copy 2N (x3/2 for own rate)"};
        for (int k = 0; k < 3; k++) {
            vs.push_back({names[k], [=](float *d, const float *s, size_t nv, hipStream_t q) {
                unsigned g = (unsigned)((nv + 63) / 64);
                if (k == 0) hipLaunchKernelGGL((k_ceiling<0>), dim3(g), dim3(64), 0, q, d, s, nv);
                if (k == 1) hipLaunchKernelGGL((k_ceiling<1>), dim3(g), dim3(64), 0, q, d, s, nv);
                if (k == 2) hipLaunchKernelGGL((k_ceiling<2>), dim3(g), dim3(64), 0, q, d, s, nv);
            }, {}});
        }
        goto run;
    }
    if (getenv("TUNE_OCC")) {
        /* occupancy A/B: the product kernel with dynamic LDS that the kernel
         * does not use, so that at most W one-wave workgroups fit a CU
         * (160 KiB of LDS per CU); fewer loads in flight per CU */
        for (int W : {4, 8, 12, 16, 20, 24, 28}) {
            const size_t lds = (size_t)163840 / W / 512 * 512;
            char buf[128];
            snprintf(buf, sizeof(buf), "product, <= %d waves per CU (LDS %zu B)", W, lds);
            vs.push_back({buf, [=](float *d, const float *s, size_t nv, hipStream_t q) {
                unsigned g = (unsigned)((nv + kReduceBlock - 1) / kReduceBlock);
                hipLaunchKernelGGL((k_reduce<float, 0, kReduceU, 1, kReduceBlock>), dim3(g),
                                   dim3(kReduceBlock), lds, q, d, s, (size_t)0, nv, (size_t)0);
            }, {}});
        }
        goto run;
    }
    if (getenv("TUNE_XCD_ONLY")) {
        xcd(0);
        xcd(16);
        xcd(32);
        xcd(64);
        xcd(128);
        xcd(256);
        xcd(2048);
        goto run;
    }
    {
    auto grid_stride = [&](int U, int NT, int maxb) {
        char buf[128];
        snprintf(buf, sizeof(buf), "gridstride U%d NT%d blocks%d", U, NT, maxb);
        vs.push_back({buf, [=](float *d, const float *s, size_t nv, hipStream_t q) {
            unsigned g = (unsigned)std::min<size_t>((nv + 256 * U - 1) / (256 * U), maxb);
            if (U == 4 && NT == 0) hipLaunchKernelGGL((k_gridstride<4, 0>), dim3(g), dim3(256), 0, q, d, s, nv);
            if (U == 2 && NT == 1) hipLaunchKernelGGL((k_gridstride<2, 1>), dim3(g), dim3(256), 0, q, d, s, nv);
        }, {}});
    };
    grid_stride(4, 0, 2048);
    auto oneshot2 = [&](int U, int NTL, int NTS, int XCD) {
        char buf[128];
        snprintf(buf, sizeof(buf), "oneshot2 U%d NTL%d NTS%d XCD%d", U, NTL, NTS, XCD);
        vs.push_back({buf, [=](float *d, const float *s, size_t nv, hipStream_t q) {
            unsigned g = (unsigned)((nv + 256 * U - 1) / (256 * U));
#define O2(A, B, C, D) if (U == A && NTL == B && NTS == C && XCD == D) hipLaunchKernelGGL((k_oneshot2<A, B, C, D>), dim3(g), dim3(256), 0, q, d, s, nv)
            O2(4, 1, 1, 0); O2(4, 1, 0, 0); O2(4, 0, 1, 0); O2(4, 1, 1, 1);
            O2(2, 1, 1, 0); O2(1, 1, 1, 0); O2(3, 1, 1, 0); O2(6, 1, 1, 0);
            O2(2, 1, 1, 1);
#undef O2
        }, {}});
    };
    oneshot2(1, 1, 1, 0);

    auto os3 = [&](int U, int BS, int CONTIG, int DFIRST) {
        char buf[128];
        snprintf(buf, sizeof(buf), "oneshot3 U%d bs%d contig%d dfirst%d", U, BS, CONTIG, DFIRST);
        vs.push_back({buf, [=](float *d, const float *s, size_t nv, hipStream_t q) {
            unsigned g = (unsigned)((nv + (size_t)BS * U - 1) / ((size_t)BS * U));
#define O3(A, B, C, D) if (U == A && BS == B && CONTIG == C && DFIRST == D) hipLaunchKernelGGL((k_oneshot3<A, B, C, D>), dim3(g), dim3(B), 0, q, d, s, nv)
            O3(1, 64, 0, 0); O3(2, 64, 0, 0); O3(4, 64, 0, 0); O3(1, 64, 0, 1);
            O3(2, 128, 0, 0); O3(1, 128, 0, 0);
#undef O3
        }, {}});
    };
    os3(1, 64, 0, 0);
    os3(2, 64, 0, 0);
    os3(4, 64, 0, 0);
    os3(1, 64, 0, 1);
    os3(2, 128, 0, 0);
    os3(1, 128, 0, 0);
    auto gs64 = [&](int PIPE, unsigned G) {
        char buf[128];
        snprintf(buf, sizeof(buf), "gs64 pipe%d grid%u", PIPE, G);
        vs.push_back({buf, [=](float *d, const float *s, size_t nv, hipStream_t q) {
            unsigned g = (unsigned)std::min<size_t>((nv + 63) / 64, G);
            if (PIPE) hipLaunchKernelGGL((k_gs64<1>), dim3(g), dim3(64), 0, q, d, s, nv);
            else      hipLaunchKernelGGL((k_gs64<0>), dim3(g), dim3(64), 0, q, d, s, nv);
        }, {}});
    };
    gs64(0, 8192);
    gs64(0, 32768);
    gs64(0, 131072);
    gs64(1, 8192);
    gs64(1, 32768);
    gs64(1, 131072);
    if (nvec * 16 <= 0xFFFFFFFFull) {
        auto osb = [&](int U, int AL, int AS, int BS) {
            char buf[128];
            snprintf(buf, sizeof(buf), "oneshot_buf U%d auxL%d auxS%d bs%d", U, AL, AS, BS);
            vs.push_back({buf, [=](float *d, const float *s, size_t nv, hipStream_t q) {
                unsigned g = (unsigned)((nv + (size_t)BS * U - 1) / ((size_t)BS * U));
#define OB(A, B, C, D) if (U == A && AL == B && AS == C && BS == D) hipLaunchKernelGGL((k_oneshot_buf<A, B, C, D>), dim3(g), dim3(D), 0, q, d, s, nv)
                OB(1, 2, 2, 64); OB(1, 18, 2, 64); OB(1, 3, 2, 64); OB(2, 18, 2, 64); OB(1, 18, 18, 64);
#undef OB
            }, {}});
        };
        osb(1, 2, 2, 64);
        osb(1, 18, 2, 64);
        osb(1, 3, 2, 64);
        osb(2, 18, 2, 64);
        osb(1, 18, 18, 64);
    }
    }
    xcd(0);
    xcd(2048);
run:
    /* init */
    hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, st,
                       (void*)src, 0, 1ull, n);
    hipLaunchKernelGGL((k_fill<UCG_DEV_DT_FLOAT32>), dim3(4096), dim3(256), 0, st,
                       (void*)ref, 0, 2ull, n);
    CHECK(hipStreamSynchronize(st));

    /* correctness: each variant once from the same start vs variant 0 */
    std::vector<uint32_t> want(n), got(n);
    for (size_t v = 0; v < vs.size(); v++) {
        CHECK(hipMemcpy(dst, ref, n * 4, hipMemcpyDeviceToDevice));
        vs[v].run(dst, src, nvec, st);
        CHECK(hipGetLastError());
        CHECK(hipStreamSynchronize(st));
        CHECK(hipMemcpy(v == 0 ? want.data() : got.data(), dst, n * 4,
                        hipMemcpyDeviceToHost));
        if (v && memcmp(want.data(), got.data(), n * 4) &&
            vs[v].name.rfind("ceiling", 0) != 0) {
            printf("MISMATCH %s\n", vs[v].name.c_str());
        }
    }

    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; r++) {
        for (auto &v : vs) {
            v.run(dst, src, nvec, st);  /* warm */
            CHECK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; i++) {
                v.run(dst, src, nvec, st);
            }
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            v.us.push_back(1000.f * ms / iters);
        }
    }
    const double bytes = 3.0 * n * 4;
    printf("n=2^%d (%.0f MiB per operand), %d rounds x %d iters\n", lg,
           n * 4 / 1048576.0, rounds, iters);
    for (auto &v : vs) {
        std::sort(v.us.begin(), v.us.end());
        double med = v.us[v.us.size() / 2], mn = v.us[0];
        printf("%-36s min %8.1f us  med %8.1f us  %7.0f GB/s (%.1f%% of 8 TB/s)\n",
               v.name.c_str(), mn, med, bytes / (med * 1e-6) / 1e9,
               100.0 * bytes / (med * 1e-6) / 8e12);
    }
    return 0;
}
