/*
 * va_reuse_probe.hip - does a virtual address mapped again to other physical
 * memory read through stale translations? (round 4: peers read old data and
 * zeros through fresh fd-based imports when the exporter's new allocation sat
 * at its old address, r04e). One process, `iters` rounds per mode; every
 * round makes a new allocation, writes the round's value into it by DMA
 * (hipMemcpy from the host) and checks it by a kernel (every word) and by DMA
 * (first and last words), then writes another value by a kernel and reads
 * that back by DMA: a stale translation on either path shows as a mismatch:
 *   same     one reservation kept; each round maps a new physical allocation
 *            at the SAME address (unmap + release between rounds)
 *   fresh    each round maps its allocation at a NEW reservation; the old
 *            one is unmapped and released but its address never freed
 *   reserve  each round reserves, maps, then unmaps, releases AND frees the
 *            address (the runtime may hand the same address out again)
 *   malloc   hipMalloc / hipFree per round
 *
 *   va_reuse_probe [iters = 200] [MiB = 6]
 *
 * Built by `make -C xucg_amd/csrc tune` into tools/ (not part of the product).
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("FAIL %s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void k_set(uint32_t *p, size_t n, uint32_t v)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        p[i] = v;
    }
}

__global__ void k_count(const uint32_t *p, size_t n, uint32_t v, unsigned *bad, unsigned *zero)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t x = p[i];
        if (x != v) {
            atomicAdd(bad, 1u);
            if (x == 0) atomicAdd(zero, 1u);
        }
    }
}

static hipMemAllocationProp prop()
{
    hipMemAllocationProp p;
    memset(&p, 0, sizeof(p));
    p.type = hipMemAllocationTypePinned;
    p.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = 0;
    return p;
}

static void map_rw(void *va, size_t bytes, hipMemGenericAllocationHandle_t h)
{
    CHECK(hipMemMap(va, bytes, 0, h, 0));
    hipMemAccessDesc d;
    memset(&d, 0, sizeof(d));
    d.location.type = hipMemLocationTypeDevice;
    d.location.id = 0;
    d.flags = hipMemAccessFlagsProtReadWrite;
    CHECK(hipMemSetAccess(va, bytes, &d, 1));
}

struct Stats {
    int rounds = 0, kernel_bad = 0, dma_bad = 0, dma_after_kernel_bad = 0, same_va = 0;
    unsigned long long bad_words = 0, zero_words = 0;
};

static void check_round(uint32_t *p, size_t n, uint32_t v, unsigned *ctr, Stats &s)
{
    static std::vector<uint32_t> host;
    host.assign(n, v);
    CHECK(hipMemcpy(p, host.data(), n * 4, hipMemcpyHostToDevice));       /* DMA write */
    CHECK(hipMemset(ctr, 0, 8));
    hipLaunchKernelGGL(k_count, dim3(1024), dim3(256), 0, 0, p, n, v, ctr, ctr + 1);
    unsigned c[2];
    CHECK(hipMemcpy(c, ctr, 8, hipMemcpyDeviceToHost));
    uint32_t h[2];
    CHECK(hipMemcpy(&h[0], p, 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&h[1], p + n - 1, 4, hipMemcpyDeviceToHost));
    s.rounds++;
    s.kernel_bad += c[0] != 0;
    s.bad_words += c[0];
    s.zero_words += c[1];
    s.dma_bad += (h[0] != v || h[1] != v);
    const uint32_t w = v ^ 0xF0000000u;
    hipLaunchKernelGGL(k_set, dim3(1024), dim3(256), 0, 0, p, n, w);    /* kernel write */
    CHECK(hipMemcpy(&h[0], p, 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&h[1], p + n - 1, 4, hipMemcpyDeviceToHost));
    s.dma_after_kernel_bad += (h[0] != w || h[1] != w);
}

int main(int argc, char **argv)
{
    setvbuf(stdout, nullptr, _IOLBF, 0);
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    const size_t bytes = (size_t)(argc > 2 ? atoi(argv[2]) : 6) << 20, n = bytes / 4;
    CHECK(hipSetDevice(0));
    unsigned *ctr;
    CHECK(hipMalloc(&ctr, 8));
    hipMemAllocationProp pr = prop();
    for (const char *mode : {"same", "fresh", "reserve", "malloc"}) {
        Stats s;
        void *keep = nullptr, *last = nullptr;
        if (!strcmp(mode, "same")) {
            CHECK(hipMemAddressReserve(&keep, bytes, 2 << 20, nullptr, 0));
        }
        for (int i = 0; i < iters; i++) {
            const uint32_t v = 0x10000u + (uint32_t)i;
            if (!strcmp(mode, "malloc")) {
                void *p;
                CHECK(hipMalloc(&p, bytes));
                s.same_va += p == last;
                last = p;
                check_round((uint32_t*)p, n, v, ctr, s);
                CHECK(hipFree(p));
                continue;
            }
            hipMemGenericAllocationHandle_t h;
            CHECK(hipMemCreate(&h, bytes, &pr, 0));
            void *va = keep;
            if (!va) {
                CHECK(hipMemAddressReserve(&va, bytes, 2 << 20, nullptr, 0));
            }
            s.same_va += va == last;
            last = va;
            map_rw(va, bytes, h);
            check_round((uint32_t*)va, n, v, ctr, s);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemUnmap(va, bytes));
            CHECK(hipMemRelease(h));
            if (!strcmp(mode, "reserve")) {
                CHECK(hipMemAddressFree(va, bytes));
            }
        }
        printf("%-8s rounds %d, same address as the previous round %d: after a DMA write, "
               "a kernel saw wrong words in %d rounds (%llu words, %llu zeros) and DMA in %d; "
               "after a kernel write, DMA in %d\n", mode, s.rounds, s.same_va, s.kernel_bad,
               s.bad_words, s.zero_words, s.dma_bad, s.dma_after_kernel_bad);
    }
    return 0;
}
